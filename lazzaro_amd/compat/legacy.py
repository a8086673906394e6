"""Implementations of the legacy shims (see package docstring)."""
from __future__ import annotations

import os
import pickle
import shutil
from typing import Any, Dict, List, Optional

from ..core.vector_store import HBMStore


class LanceDBVectorStore:
    """Pre-v0.3 vector store: ``add(nodes)``, ``search(emb, limit)``, ``delete(ids)``."""

    def __init__(self, db_dir: str = "db", user_id: str = "default", **kw):
        self._store = HBMStore(db_dir=db_dir, **kw)
        self.user_id = user_id

    def add(self, nodes: List[Dict[str, Any]]) -> None:
        self._store.add_nodes(nodes, user_id=self.user_id)

    def search(self, query_emb, limit: int = 5) -> List[str]:
        return self._store.search_nodes(query_emb, user_id=self.user_id, limit=limit)

    def delete(self, node_ids: List[str]) -> None:
        if node_ids:
            self._store.delete_nodes(node_ids, user_id=self.user_id)

    def close(self) -> None:
        self._store.close()


class PersistenceManager:
    """Snapshot file manager: atomic write, previous snapshot kept as ``.bak``."""

    def __init__(self, db_dir: str = "db", filename: str = "lazzaro.pkl"):
        self.db_dir = db_dir
        os.makedirs(db_dir, exist_ok=True)
        self.filepath = os.path.join(db_dir, filename)

    def save(self, data: Dict[str, Any]) -> bool:
        tmp = self.filepath + ".tmp"
        try:
            with open(tmp, "wb") as f:
                pickle.dump(data, f, protocol=pickle.HIGHEST_PROTOCOL)
            if os.path.exists(self.filepath):
                shutil.copy2(self.filepath, self.filepath + ".bak")
            os.replace(tmp, self.filepath)
            return True
        except OSError:
            return False

    def load(self) -> Optional[Dict[str, Any]]:
        for p in (self.filepath, self.filepath + ".bak"):
            if os.path.exists(p):
                try:
                    with open(p, "rb") as f:  # files written by save() above only
                        return pickle.load(f)
                except Exception:
                    continue
        return None
