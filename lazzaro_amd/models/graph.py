"""Memory graph data model: :class:`Node` (memory unit) and :class:`Edge`
(association).

API parity with reference ``src/lazzaro/models/graph.py:6-104``: same field
names, order and defaults, ``from_dict`` ignores unknown keys, ``to_dict`` is a
plain-data dict. The embedding stays a Python list at this layer (that is the
public contract); the engine keeps a device copy in the tenant's HBM arena
(see :mod:`lazzaro_amd.index.arena`), so hot paths never iterate these lists.
"""
from __future__ import annotations

import dataclasses
import time
from dataclasses import dataclass, field
from typing import Any, Dict, List, Optional


def _now() -> float:
    return time.time()


class _DictMixin:
    @classmethod
    def from_dict(cls, data: Dict[str, Any]):
        names = {f.name for f in dataclasses.fields(cls)}
        return cls(**{k: v for k, v in data.items() if k in names})

    def to_dict(self) -> Dict[str, Any]:
        out = {}
        for f in dataclasses.fields(self):
            v = getattr(self, f.name)
            if isinstance(v, list):
                v = list(v)
            out[f.name] = v
        return out


@dataclass
class Node(_DictMixin):
    """An atomic memory: text, embedding and biologically-inspired metrics.

    ``salience`` in [0, 1] decays towards 0.2 every conversation; super-nodes
    summarise a shard (``child_ids``) and carry the mean child embedding.
    """

    id: str
    content: str
    embedding: List[float] = field(default_factory=list)
    type: str = "semantic"
    timestamp: float = field(default_factory=_now)
    access_count: int = 0
    last_accessed: float = field(default_factory=_now)
    salience: float = 0.5
    is_super_node: bool = False
    child_ids: List[str] = field(default_factory=list)
    parent_id: Optional[str] = None
    shard_key: str = "default"


@dataclass
class Edge(_DictMixin):
    """A directed association ``source -> target`` (neighbour queries treat it
    as undirected). ``weight`` in [0, 1] decays and is pruned below a threshold."""

    source: str
    target: str
    weight: float = 1.0
    edge_type: str = "relates_to"
    co_occurrence: int = 1
    last_updated: float = field(default_factory=_now)
