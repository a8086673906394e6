"""HBMStore: the ``Store`` protocol over the native columnar store + per-tenant
HBM vector arenas (replaces reference ``core/vector_store.py:7-244``,
``LanceDBStore``; exported under that name too for drop-in use).

* Persistence: three versioned columnar tables ``nodes``, ``edges``,
  ``profiles`` under ``{db_dir}/lancedb/`` with the reference's column names and
  types. Every committed write bumps the table version, which
  is what ``get_latest_version``/``MemorySystem.check_for_updates`` poll.
* Search: each tenant (``user_id``) has its own :class:`VectorArena` in HBM --
  the tenant "segment" replaces LanceDB's BTREE ``user_id`` prefilter (no mask,
  no scan of other tenants). ``search_nodes`` runs the fused MFMA top-k kernel;
  metric defaults to L2 like LanceDB (SURVEY.md §7.4 risk 4).
* Arenas are built lazily from the table and kept in sync with this process's
  own writes; writes from other processes are picked up when the table version
  moves (checked at most every ``consistency_interval`` seconds).
* A ``MemorySystem`` *attaches* its tenant graph (:meth:`attach`): that
  tenant's searches then run over the graph's own HBM rows (no second copy of
  the vectors), store membership is the graph's ``stored`` column, and
  persistence is incremental (:meth:`commit_tenant` upserts changed rows and
  deletes removed ones in one version per table; :meth:`load_tenant` returns
  raw columns for a bulk reload).
"""
from __future__ import annotations

import json
import os
import threading
import time
from typing import Sequence, Any, Dict, List, Optional

import numpy as np
import torch

from ..index.arena import VectorArena
from ..store.colstore import EDGE_SCHEMA, NODE_SCHEMA, PROFILE_SCHEMA, ColumnarTable
from ..utils.device import default_device


def _json(v, default):
    if v is None:
        return json.dumps(default)
    return v if isinstance(v, str) else json.dumps(v)


def _unjson(v, default):
    if isinstance(v, str):
        try:
            return json.loads(v)
        except Exception:
            return default
    return v if v is not None else default


class HBMStore:
    def __init__(self, db_dir: str = "db", device=None, metric: str = "l2",
                 consistency_interval: float = 0.5, keep_fp32: bool = True, index: str = "flat",
                 nlist: int = 4096, nprobe: int = 32, pq_m: int = 64, ivf_min_rows: int = 1_000_000):
        """index="ivfpq": a tenant arena with >= ivf_min_rows live rows is served
        by IVF-PQ candidates re-ranked exactly (smaller tenants stay exact flat)."""
        if index not in ("flat", "ivfpq"):
            raise ValueError("index must be 'flat' or 'ivfpq'")
        self.index, self.ivf_params = index, dict(nlist=nlist, nprobe=nprobe, m=pq_m, min_rows=ivf_min_rows)
        self.db_dir = db_dir
        self._uri = os.path.join(db_dir, "lancedb")
        os.makedirs(self._uri, exist_ok=True)
        self.device = device if device is not None else default_device()
        self.metric = metric
        self.keep_fp32 = keep_fp32
        self.consistency_interval = consistency_interval
        self.nodes_table_name, self.edges_table_name, self.profile_table_name = "nodes", "edges", "profiles"
        self._nodes_table = ColumnarTable(self._uri, "nodes", NODE_SCHEMA)
        self._edges_table = ColumnarTable(self._uri, "edges", EDGE_SCHEMA)
        self._profile_table = ColumnarTable(self._uri, "profiles", PROFILE_SCHEMA)
        self._arenas: Dict[str, VectorArena] = {}
        self._synced: Dict[str, int] = {}
        self._last_check: Dict[str, float] = {}
        self._lock = threading.RLock()
        self._dim: Optional[int] = None
        self._graphs: Dict[str, object] = {}

    # ------------------------------------------------------------ attached tenant graphs
    def attach(self, user_id: str, graph) -> None:
        """Serve ``user_id``'s vector search from ``graph`` (a TenantGraph)."""
        with self._lock:
            self._graphs[user_id] = graph
            self._arenas.pop(user_id, None)
            self._synced.pop(user_id, None)
            if self.index == "ivfpq":  # large tenants: IVF-PQ candidates + exact fp32 re-rank on the graph
                graph.ann_cfg = dict(self.ivf_params)

    def detach(self, user_id: str) -> None:
        with self._lock:
            self._graphs.pop(user_id, None)

    def bound_graph(self, user_id: str):
        return self._graphs.get(user_id)

    def commit_tenant(self, user_id: str, node_cols: Dict, delete_ids: Sequence[str], edge_cols: Dict,
                      delete_edge_ids: Sequence[str]) -> int:
        """Incremental commit of one tenant: upsert the given node / edge rows
        and delete the given ids, one version per touched table. Returns the
        nodes table version."""
        with self._lock:
            up = list(node_cols.get("id", []))
            if up or delete_ids:
                n = len(up)
                if n and self._dim is None and node_cols["vector"].shape[1]:
                    self._dim = node_cols["vector"].shape[1]
                cols = self._nodes_table.fill_columns({k: v for k, v in node_cols.items()
                                                       if k not in ("count", "fresh")}, n, {"user_id": user_id})
                if n == 0:
                    cols["vector"] = np.zeros((0, self._table_dim() or 0), dtype=np.float32)
                # ids never committed before (``fresh``) cannot be in the table:
                # only the others (and the deletions) go through the key index
                fresh = node_cols.get("fresh")
                if fresh is not None and len(fresh) == n:
                    old = np.nonzero(~np.asarray(fresh, dtype=bool))[0]
                    keys = [up[j] for j in old.tolist()] + list(delete_ids)
                else:
                    keys = up + list(delete_ids)
                if keys:
                    self._nodes_table.upsert_columns([("user_id", user_id)], "id", keys, cols)
                else:
                    self._nodes_table.add_columns(cols)
            eu = list(edge_cols.get("id", []))
            if eu or delete_edge_ids:
                cols = self._edges_table.fill_columns({k: v for k, v in edge_cols.items() if k != "count"}, len(eu),
                                                      {"user_id": user_id})
                self._edges_table.upsert_columns([("user_id", user_id)], "id", eu + list(delete_edge_ids), cols)
            return self._nodes_table.version

    def load_tenant(self, user_id: str):
        """(node columns, edge columns) of one tenant, as stored."""
        # the columns the graph loader reads (not user_id / metadata: at 10M
        # rows every string column costs seconds of Python objects)
        want = [c for c, _, _ in self._nodes_table.schema if c not in ("user_id", "metadata")]
        # the vector column as zero-copy pieces of the mapped fragments: the
        # loader streams them to the device (no 30 GB host copy to allocate,
        # fill and free for a 10M x 768 tenant)
        nc = self._nodes_table.scan_columns([("user_id", user_id)], want=want, vec_pieces=True)
        if not nc or not len(nc.get("id", [])):
            return {"id": []}, {"id": []}
        v = nc["vector"]
        d = next((int(x.shape[1]) for x in v if x.shape[1]), 0) if isinstance(v, list) else \
            (int(v.shape[1]) if v.ndim == 2 else 0)
        if d:
            self._dim = self._dim or d
        ec = self._edges_table.scan_columns([("user_id", user_id)])
        return nc, (ec if ec else {"id": []})

    # ------------------------------------------------------------ helpers
    def _table_dim(self) -> Optional[int]:
        if self._dim is None:
            for n, t, d in self._nodes_table.schema:
                if n == "vector" and d:
                    self._dim = d
        return self._dim

    def _arena(self, user_id: str) -> VectorArena:
        """Tenant arena, rebuilt from the table if another writer moved it."""
        with self._lock:
            a = self._arenas.get(user_id)
            now = time.time()
            if a is not None and now - self._last_check.get(user_id, 0.0) < self.consistency_interval:
                return a
            self._last_check[user_id] = now
            v = self._nodes_table.version
            if a is not None and self._synced.get(user_id) == v:
                return a
            cols = self._nodes_table.scan_columns([("user_id", user_id)], want=["id", "vector"])
            a = VectorArena(device=self.device, keep_fp32=self.keep_fp32)
            if self.index == "ivfpq":
                a.enable_ivf(**self.ivf_params)
            ids = cols.get("id", [])
            if len(ids):
                vec = cols["vector"]
                a.add(ids, vec)
            self._arenas[user_id] = a
            self._synced[user_id] = v
            return a

    def _after_write(self, user_id: str, prev_version, new_version: int) -> None:
        # our write landed directly on the version the arena reflects -> the
        # arena (already updated in place) is in sync; otherwise another
        # process wrote in between: force a rebuild on next use.
        if prev_version is not None and prev_version + 1 == new_version:
            self._synced[user_id] = new_version
        else:
            self._synced.pop(user_id, None)
            self._last_check.pop(user_id, None)

    # ------------------------------------------------------------ nodes
    def _node_rows(self, nodes: List[Dict[str, Any]], user_id: str) -> List[Dict[str, Any]]:
        rows = []
        dim = self._table_dim()
        for n in nodes:
            emb = n.get("embedding", n.get("vector")) or []
            if dim is None and len(emb):
                dim = self._dim = len(emb)
            rows.append({
                "id": n["id"], "user_id": user_id, "content": n["content"],
                "vector": list(emb) if len(emb) else [0.0] * (dim or 0),
                "type": n.get("type", "semantic"),
                "timestamp": float(n.get("timestamp", 0.0)),
                "access_count": int(n.get("access_count", 0)),
                "last_accessed": float(n.get("last_accessed", 0.0)),
                "salience": float(n.get("salience", 0.5)),
                "is_super_node": bool(n.get("is_super_node", False)),
                "child_ids": _json(n.get("child_ids", []), []),
                "parent_id": n.get("parent_id") or "",
                "shard_key": n.get("shard_key", "default"),
                "metadata": _json(n.get("metadata", {}), {}),
                "decay_clock": float(n.get("decay_clock", 0.0)),
            })
        return rows

    def add_nodes(self, nodes: List[Dict[str, Any]], user_id: str = "default") -> None:
        if not nodes:
            return
        rows = self._node_rows(nodes, user_id)
        with self._lock:
            g = self._graphs.get(user_id)
            if g is not None:
                self._nodes_table.add_rows(rows)
                self._graph_store_rows(g, rows)
                return
            a = self._arena(user_id)
            prev = self._synced.get(user_id)
            v = self._nodes_table.add_rows(rows)
            a.add([r["id"] for r in rows], np.asarray([r["vector"] for r in rows], dtype=np.float32))
            self._after_write(user_id, prev, v)

    @staticmethod
    def _graph_store_rows(g, rows: List[Dict[str, Any]]) -> None:
        """Rows written to an attached tenant join its searchable set: known
        ids are flagged; unknown ids become store-only (ghost) rows."""
        known = [g.row_of.get(r["id"], -1) for r in rows]
        g.mark_stored([k for k in known if k >= 0])
        new = [r for r, k in zip(rows, known) if k < 0]
        if new:
            g.add_nodes([r["id"] for r in new], [r["content"] for r in new], [r["vector"] for r in new],
                        shard=[g.shard_id(r["shard_key"], live=False) for r in new], stored=True, ghost=True)

    def replace_user_nodes(self, nodes: List[Dict[str, Any]], user_id: str = "default") -> None:
        """Atomic per-tenant rewrite (one committed version): the delete-all +
        add-all of the reference's ``_save_to_persistence`` (memory_system.py:
        1275-1302) without the window in which the tenant has no rows."""
        rows = self._node_rows(nodes, user_id)
        with self._lock:
            a = self._arena(user_id)
            prev = self._synced.get(user_id)
            _, v = self._nodes_table.replace_rows([("user_id", user_id)], rows)
            a.clear()
            if rows:
                a.add([r["id"] for r in rows], np.asarray([r["vector"] for r in rows], dtype=np.float32))
            self._after_write(user_id, prev, v)

    def get_nodes(self, user_id: str = "default") -> List[Dict[str, Any]]:
        rows = self._nodes_table.scan([("user_id", user_id)])
        for r in rows:
            r["child_ids"] = _unjson(r.get("child_ids"), [])
            r["metadata"] = _unjson(r.get("metadata"), {})
        return rows

    def search_nodes(self, query_emb, user_id: str = "default", limit: int = 5) -> List[str]:
        if query_emb is None or len(query_emb) == 0:
            return []
        g = self._graphs.get(user_id)
        if g is not None:
            q = query_emb if torch.is_tensor(query_emb) else torch.from_numpy(
                np.asarray(query_emb, dtype=np.float32))
            with g.lock:  # the tenant's graph lock: a consolidation may be writing
                if g.dim is None or q.shape[-1] != g.dim:
                    return []
                return g.search_ids(q, int(limit), self.metric)[0]
        with self._lock:  # writers (add/delete/replace) mutate the arena in place
            a = self._arena(user_id)
            if len(a) == 0 or a.dim != len(query_emb):
                return []
            return a.search(query_emb, int(limit), self.metric)[0]

    def search_nodes_batch(self, query_embs, user_id: str = "default", limit: int = 5) -> List[List[str]]:
        """Batched variant (one kernel launch for all queries). ``query_embs``
        may be a device tensor (kept on the device end to end)."""
        g = self._graphs.get(user_id)
        if g is not None:
            Q = query_embs if torch.is_tensor(query_embs) else torch.as_tensor(
                np.asarray(query_embs, dtype=np.float32))
            if len(Q) == 0:
                return []
            with g.lock:
                if g.dim is None or Q.shape[-1] != g.dim:
                    return [[] for _ in range(len(Q))]
                return g.search_ids(Q, int(limit), self.metric)
        with self._lock:
            a = self._arena(user_id)
            if len(a) == 0 or len(query_embs) == 0:
                return [[] for _ in range(len(query_embs))]
            return a.search(query_embs, int(limit), self.metric)

    def search_nodes_multi(self, query_embs, user_ids: Sequence[str], limit: int = 5) -> List[List[str]]:
        """Multi-tenant batch: query i searches tenant ``user_ids[i]`` only, all
        in one kernel launch (serving many users per GPU, BASELINE config 3)."""
        from ..index.arena import multi_arena_search
        if len(user_ids) == 0:
            return []
        with self._lock:
            return self._search_multi(query_embs, user_ids, limit)

    def _search_multi(self, query_embs, user_ids, limit):
        from ..index.arena import multi_arena_search
        arenas = [self._arena(u) for u in user_ids]
        dims = {a.dim for a in arenas if len(a)}
        if len(dims) > 1 or any(a.dim is not None and len(a) and a.dim != len(query_embs[0]) for a in arenas):
            return [self.search_nodes(q, u, limit) for q, u in zip(query_embs, user_ids)]
        if not dims:
            return [[] for _ in user_ids]
        s, r = multi_arena_search(arenas, query_embs, int(limit), self.metric)
        s, r = s.cpu().tolist(), r.cpu().tolist()
        out = []
        for a, rs, ss in zip(arenas, r, s):
            out.append([a.ids[x] for x, v in zip(rs, ss) if x >= 0 and v != float("-inf") and a.ids[x] is not None])
        return out

    def delete_nodes(self, node_ids: Optional[List[str]], user_id: str = "default",
                     graph_unstored: bool = False) -> None:
        """``graph_unstored``: the bound graph already cleared the rows'
        stored bits (TenantGraph.segment_end(unstore=True)); only the
        persisted table rows go."""
        g = self._graphs.get(user_id)
        if g is not None:
            with self._lock:
                if not node_ids:
                    self._nodes_table.delete([("user_id", user_id)])
                    g.unstore(list(g.ids))
                else:
                    self._nodes_table.delete([("user_id", user_id)], "id", list(node_ids))
                    if not graph_unstored:
                        g.unstore(node_ids)
            return
        with self._lock:
            a = self._arena(user_id)
            prev = self._synced.get(user_id)
            if not node_ids:
                n, v = self._nodes_table.delete([("user_id", user_id)])
                a.clear()
            else:
                n, v = self._nodes_table.delete([("user_id", user_id)], "id", list(node_ids))
                a.delete(node_ids)
            if n:
                self._after_write(user_id, prev, v)

    def get_latest_version(self) -> int:
        return self._nodes_table.version

    def list_users(self) -> List[str]:
        cols = self._nodes_table.scan_columns(want=["user_id"])
        return sorted(set(cols.get("user_id", [])))

    # ------------------------------------------------------------ edges
    @staticmethod
    def _edge_rows(edges: List[Dict[str, Any]], user_id: str) -> List[Dict[str, Any]]:
        rows = []
        for e in edges:
            src = e.get("source") or e.get("source_id")
            tgt = e.get("target") or e.get("target_id")
            rows.append({
                "id": e.get("id", f"{src}_{tgt}"), "user_id": user_id,
                "source_id": src, "target_id": tgt,
                "weight": float(e.get("weight", 1.0)),
                "edge_type": e.get("edge_type") or e.get("type", "relates_to"),
                "co_occurrence": int(e.get("co_occurrence", 1)),
                "last_updated": float(e.get("last_updated", 0.0)),
                "metadata": _json(e.get("metadata", {}), {}),
            })
        return rows

    def add_edges(self, edges: List[Dict[str, Any]], user_id: str = "default") -> None:
        if not edges:
            return
        self._edges_table.add_rows(self._edge_rows(edges, user_id))

    def replace_user_edges(self, edges: List[Dict[str, Any]], user_id: str = "default") -> None:
        """Atomic per-tenant edge rewrite (see :meth:`replace_user_nodes`)."""
        self._edges_table.replace_rows([("user_id", user_id)], self._edge_rows(edges, user_id))

    def delete_edges(self, source_id: Optional[str] = None, user_id: str = "default") -> None:
        eq = [("user_id", user_id)]
        if source_id:
            eq.append(("source_id", source_id))
        self._edges_table.delete(eq)

    def get_edges(self, source_id: Optional[str] = None, user_id: str = "default") -> List[Dict[str, Any]]:
        eq = [("user_id", user_id)]
        if source_id:
            eq.append(("source_id", source_id))
        rows = self._edges_table.scan(eq)
        for r in rows:
            r["type"] = r.get("edge_type")
            r["metadata"] = _unjson(r.get("metadata"), {})
        return rows

    # ------------------------------------------------------------ profiles
    def save_profile(self, profile_data: Dict[str, Any], user_id: str = "default") -> None:
        self._profile_table.replace_rows([("user_id", user_id)], [{"user_id": user_id, "data": json.dumps(profile_data),
                                                                   "updated_at": time.time()}])

    def load_profile(self, user_id: str = "default") -> Optional[Dict[str, Any]]:
        rows = self._profile_table.scan([("user_id", user_id)])
        return json.loads(rows[-1]["data"]) if rows else None

    # ------------------------------------------------------------ legacy aliases
    def add(self, nodes: List[Dict[str, Any]], user_id: str = "default") -> None:
        """pre-v0.3 ``VectorStore.add`` (reference tests/test_lancedb_integration.py)"""
        self.add_nodes(nodes, user_id=user_id)

    def search(self, query_emb, limit: int = 5, user_id: str = "default") -> List[str]:
        return self.search_nodes(query_emb, user_id=user_id, limit=limit)

    def delete(self, node_ids: List[str], user_id: str = "default") -> None:
        if node_ids:
            self.delete_nodes(node_ids, user_id=user_id)

    # ------------------------------------------------------------ misc
    def compact(self) -> None:
        for t in (self._nodes_table, self._edges_table, self._profile_table):
            t.compact()

    def close(self) -> None:
        self._graphs.clear()
        self._arenas.clear()
        self._synced.clear()


LanceDBStore = HBMStore  # drop-in name used by reference code
