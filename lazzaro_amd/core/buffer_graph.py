"""BufferGraph: the composite view over all shards + super-nodes (reference
``src/lazzaro/core/buffer_graph.py:6-141``).

Behavioural parity notes:

* ``nodes``/``edges`` return fresh merged dicts (super-nodes first, then shards
  in insertion order), like the reference.
* ``add_edge`` routes to the source node's shard, else ``"default"`` if it
  exists, else drops the edge (reference :51-61).
* ``get_neighbors`` consults only the node's own shard (so an edge stored in
  another shard is visible from its source side only -- the reference's
  directed visibility, which ``get_connected_components`` inherits).
* ``get_connected_components`` returns the same sets as the reference's
  recursive DFS but runs iteratively, so a 1,500-node chain no longer hits
  ``RecursionError`` (SURVEY.md §6 probe, reference :107-112). Device-scale
  graphs use the ``uf_union_kernel`` union-find (``TenantGraph.component_digest``).
"""
from __future__ import annotations

import time
from typing import Dict, List, Optional, Set, Tuple

from ..models.graph import Edge, Node
from .memory_shard import MemoryShard

DEFAULT_SHARD = "default"


class BufferGraph:
    def __init__(self, shards: Dict[str, MemoryShard], super_nodes: Dict[str, Node]):
        self.shards = shards
        self.super_nodes = super_nodes

    # ---- merged views ------------------------------------------------------
    @property
    def nodes(self) -> Dict[str, Node]:
        merged = dict(self.super_nodes)
        for sh in self.shards.values():
            merged.update(sh.nodes)
        return merged

    @property
    def edges(self) -> Dict[Tuple[str, str], Edge]:
        merged: Dict[Tuple[str, str], Edge] = {}
        for sh in self.shards.values():
            merged.update(sh.edges)
        return merged

    def _shard_of(self, node_id: str) -> Optional[MemoryShard]:
        for sh in self.shards.values():
            if node_id in sh.nodes:
                return sh
        return None

    # ---- mutation ------------------------------------------------------------
    def add_node(self, node: Node) -> None:
        key = node.shard_key or DEFAULT_SHARD
        sh = self.shards.get(key)
        if sh is None:
            sh = self.shards[key] = MemoryShard(key)
        sh.add_node(node)

    def add_edge(self, edge: Edge) -> None:
        sh = self._shard_of(edge.source)
        if sh is None:
            sh = self.shards.get(DEFAULT_SHARD)
        if sh is not None:
            sh.add_edge(edge)

    # ---- lookup ----------------------------------------------------------------
    def get_node(self, node_id: str) -> Optional[Node]:
        n = self.super_nodes.get(node_id)
        if n is not None:
            return n
        sh = self._shard_of(node_id)
        return sh.nodes[node_id] if sh is not None else None

    def get_neighbors(self, node_id: str, min_weight: float = 0.3) -> List[str]:
        sh = self._shard_of(node_id)
        return sh.get_neighbors(node_id, min_weight) if sh is not None else []

    def update_access(self, node_id: str) -> None:
        n = self.get_node(node_id)
        if n is not None:
            n.access_count += 1
            n.last_accessed = time.time()
            n.salience = min(1.0, n.salience + 0.05)

    # ---- maintenance -----------------------------------------------------------
    def apply_temporal_decay(self, decay_rate: float = 0.01) -> None:
        for sh in self.shards.values():
            sh.apply_temporal_decay(decay_rate)

    def prune_weak_edges(self, threshold: float = 0.5) -> int:
        return sum(sh.prune_weak_edges(threshold) for sh in self.shards.values())

    def get_connected_components(self) -> List[Set[str]]:
        """Components in first-visit order of ``self.nodes`` (iterative DFS)."""
        visited: Set[str] = set()
        comps: List[Set[str]] = []
        for start in self.nodes:
            if start in visited:
                continue
            comp = {start}
            visited.add(start)
            stack = [start]
            while stack:
                cur = stack.pop()
                for nb in self.get_neighbors(cur, min_weight=0.0):
                    if nb not in visited:
                        visited.add(nb)
                        comp.add(nb)
                        stack.append(nb)
            comps.append(comp)
        return comps

    def size(self) -> Tuple[int, int]:
        n = len(self.super_nodes) + sum(len(s.nodes) for s in self.shards.values())
        e = sum(len(s.edges) for s in self.shards.values())
        return n, e

    def get_all_nodes_summary(self) -> List[Dict]:
        out = []
        for n in sorted(self.nodes.values(), key=lambda x: x.timestamp, reverse=True):
            c = n.content
            out.append({
                "id": n.id,
                "content": (c[:100] + "...") if len(c) > 100 else c,
                "type": n.type,
                "salience": n.salience,
                "access_count": n.access_count,
                "shard": n.shard_key,
            })
        return out
