"""MemoryShard: a topic-partitioned subgraph (reference
``src/lazzaro/core/memory_shard.py:7-88``).

Public surface is identical (``nodes`` dict, ``edges`` dict keyed by
``(source, target)``, ``add_node/add_edge/get_neighbors/apply_temporal_decay/
prune_weak_edges/size``). Differences that are engine-level, not behavioural:

* ``edges`` is an :class:`EdgeMap` -- a dict that maintains a per-node incidence
  index on every mutation, so ``get_neighbors`` is O(degree) instead of the
  reference's O(E) scan (``memory_shard.py:54-62``) while returning neighbours in
  the same (edge-insertion) order. Direct ``del shard.edges[k]`` keeps working.
* decay/prune keep the reference's arithmetic exactly (edge ``w *= 1-r``;
  salience ``0.2 + (s-0.2)(1-r)`` with floor 0.2; prune ``w < thr``). Bulk
  decay/prune of a tenant's device-resident graph runs in the fused HIP
  kernel ``tg_decay_kernel`` (``ops.tenant_ops.decay``, ``TenantGraph.decay``).
"""
from __future__ import annotations

import time
from typing import Dict, Iterable, List, Tuple

from ..models.graph import Edge, Node

Key = Tuple[str, str]

SALIENCE_FLOOR = 0.2


class EdgeMap(dict):
    """``{(src, tgt): Edge}`` with an insertion-ordered incidence index."""

    __slots__ = ("_inc",)

    def __init__(self, *a, **kw):
        super().__init__()
        self._inc: Dict[str, Dict[Key, None]] = {}
        if a or kw:
            self.update(*a, **kw)

    # -- index maintenance -------------------------------------------------
    def _link(self, key: Key) -> None:
        s, t = key
        self._inc.setdefault(s, {})[key] = None
        if t != s:
            self._inc.setdefault(t, {})[key] = None

    def _unlink(self, key: Key) -> None:
        for n in (key[0], key[1]):
            d = self._inc.get(n)
            if d is not None:
                d.pop(key, None)
                if not d:
                    del self._inc[n]

    def __setitem__(self, key, value):
        if key not in self:
            self._link(key)
        super().__setitem__(key, value)

    def __delitem__(self, key):
        super().__delitem__(key)
        self._unlink(key)

    def pop(self, key, *default):
        if key in self:
            self._unlink(key)
        return super().pop(key, *default)

    def popitem(self):
        k, v = super().popitem()
        self._unlink(k)
        return k, v

    def clear(self):
        super().clear()
        self._inc.clear()

    def update(self, *a, **kw):
        for k, v in dict(*a, **kw).items():
            self[k] = v

    def setdefault(self, key, default=None):
        if key not in self:
            self[key] = default
        return self[key]

    def incident(self, node_id: str) -> Iterable[Key]:
        """Edge keys touching ``node_id`` in insertion order."""
        d = self._inc.get(node_id)
        return list(d.keys()) if d else []

    def copy(self):
        return EdgeMap(self)

    def __reduce__(self):
        return (EdgeMap, (dict(self),))


class MemoryShard:
    """A semantically isolated subgraph (one topic) of a tenant's memory."""

    def __init__(self, shard_key: str):
        self.shard_key = shard_key
        self.nodes: Dict[str, Node] = {}
        self.edges: EdgeMap = EdgeMap()
        self.last_accessed = time.time()
        self.access_count = 0

    def __setattr__(self, name, value):
        # keep the incidence index valid if a caller swaps the dict wholesale
        if name == "edges" and not isinstance(value, EdgeMap):
            value = EdgeMap(value)
        object.__setattr__(self, name, value)

    def add_node(self, node: Node) -> None:
        node.shard_key = self.shard_key
        self.nodes[node.id] = node

    def add_edge(self, edge: Edge) -> None:
        key = (edge.source, edge.target)
        cur = self.edges.get(key)
        if cur is None:
            self.edges[key] = edge
            return
        # re-observing an association strengthens it (reference :48-50)
        cur.weight = min(1.0, cur.weight + 0.1)
        cur.co_occurrence += 1

    def get_neighbors(self, node_id: str, min_weight: float = 0.3) -> List[str]:
        out = []
        for key in self.edges.incident(node_id):
            e = self.edges[key]
            if e.weight < min_weight:
                continue
            s, t = key
            out.append(t if s == node_id else s)
        return out

    def apply_temporal_decay(self, decay_rate: float = 0.01) -> None:
        keep = 1.0 - decay_rate
        for e in self.edges.values():
            e.weight *= keep
        for n in self.nodes.values():
            s = n.salience
            n.salience = SALIENCE_FLOOR + (s - SALIENCE_FLOOR) * keep if s > SALIENCE_FLOOR else SALIENCE_FLOOR

    def prune_weak_edges(self, threshold: float = 0.5) -> int:
        dead = [k for k, e in self.edges.items() if e.weight < threshold]
        for k in dead:
            del self.edges[k]
        return len(dead)

    def size(self) -> Tuple[int, int]:
        return len(self.nodes), len(self.edges)

    def remove_node(self, node_id: str) -> bool:
        """Drop a node and every edge of this shard touching it."""
        if node_id not in self.nodes:
            return False
        del self.nodes[node_id]
        for k in self.edges.incident(node_id):
            del self.edges[k]
        return True
