"""Reference-shaped views over a :class:`TenantGraph`.

The reference's public surface hands out live Python objects: ``Node`` and
``Edge`` dataclasses inside ``MemoryShard.nodes/edges`` dicts, a
``BufferGraph`` that merges them, ``MemorySystem.shards`` /
``super_nodes`` dicts (``core/memory_shard.py``, ``core/buffer_graph.py``,
``memory_system.py:99-102``). Tests, the CLI, the dashboard and the
integrations read and mutate those objects directly.

Here the data lives in the tenant graph's device columns, and these classes
are thin façades materialised on demand:

* :class:`NodeView` / :class:`EdgeView` subclass ``Node`` / ``Edge``; every
  field is a property reading (host mirror, refreshed when the graph version
  moves) or writing (device scatter) the graph's columns. A ``Node`` or
  ``Edge`` handed to ``add_node`` / ``add_edge`` is *adopted*: it becomes a
  view of its row, so later attribute writes reach the graph as they reach the
  reference's dict entry.
* :class:`ShardView` is a ``MemoryShard`` bound to one shard code;
  :class:`ShardsMap`, :class:`SuperNodesMap` and :class:`GraphBuffer` play
  ``MemorySystem.shards``, ``.super_nodes`` and ``.buffer``.

None of this is on a hot path: consolidation, retrieval, decay, eviction and
the boost call the engine directly.
"""
from __future__ import annotations

import time
from collections.abc import MutableMapping, Sequence
from typing import Dict, Iterator, List, Optional, Set, Tuple

import numpy as np
import torch

from ..core.memory_shard import MemoryShard
from ..core.buffer_graph import BufferGraph
from ..models.graph import Edge, Node
from .tenant_graph import GHOST, NODE, SHARD_MASK, TYPE_MASK, TYPE_SHIFT, EDIRTY, TenantGraph

DEFAULT_SHARD = "default"
SALIENCE_FLOOR = 0.2


# ---------------------------------------------------------------- nodes
def _node_prop(col: str, conv):
    def get(self):
        return conv(self._g.get_scalar(self._r, col))

    def set_(self, v):
        self._g.set_scalar(self._r, col, v)
    return property(get, set_)


class NodeView(Node):
    """A ``Node`` whose fields live in a :class:`TenantGraph` row."""

    @classmethod
    def of(cls, g: TenantGraph, r: int) -> "NodeView":
        cache = g.__dict__.setdefault("_node_views", {})
        v = cache.get(r)
        if v is None:
            v = object.__new__(cls)
            v.__dict__["_g"] = g
            v.__dict__["_r"] = r
            cache[r] = v
        return v

    @classmethod
    def of_rows(cls, g: TenantGraph, rows_lists) -> List[List["NodeView"]]:
        """``[[of(g, r) for r in rows if r >= 0] for rows in rows_lists]`` with
        the view cache bound once (the per-batch result mapping of the search
        paths: ~10k rows per 1024-query batch)."""
        cache = g.__dict__.setdefault("_node_views", {})
        get = cache.get
        new = object.__new__
        out = []
        for rows in rows_lists:
            lst = []
            for r in rows:
                if r < 0:
                    continue
                v = get(r)
                if v is None:
                    v = new(cls)
                    d = v.__dict__
                    d["_g"] = g
                    d["_r"] = r
                    cache[r] = v
                lst.append(v)
            out.append(lst)
        return out

    @classmethod
    def adopt(cls, node: Node, g: TenantGraph, r: int) -> "NodeView":
        cache = g.__dict__.setdefault("_node_views", {})
        if type(node) is Node:
            node.__dict__.clear()
            node.__class__ = cls
            node.__dict__["_g"] = g
            node.__dict__["_r"] = r
            cache[r] = node
            return node
        return cls.of(g, r)

    id = property(lambda self: self._g.ids[self._r])
    salience = _node_prop("sal", float)
    access_count = _node_prop("acc", int)
    last_accessed = _node_prop("last", float)
    timestamp = _node_prop("ts", float)
    is_super_node = property(lambda self: bool(self._g.get_scalar(self._r, "sup")))

    @property
    def content(self) -> str:
        return self._g.content[self._r]

    @content.setter
    def content(self, v: str) -> None:
        self._g.content[self._r] = v
        self._g.set_scalar(self._r, "dirty", 1)

    @property
    def type(self) -> str:
        return self._g.types[self._r]

    @type.setter
    def type(self, v: str) -> None:
        self._g.types[self._r] = v
        self._g.set_scalar(self._r, "dirty", 1)

    @property
    def embedding(self) -> list:
        return self._g.embedding(self._r)

    @embedding.setter
    def embedding(self, v) -> None:
        self._g.set_embedding(self._r, v)

    @property
    def child_ids(self) -> list:
        return self._g.children.setdefault(self._r, []) if self.is_super_node else self._g.children.get(self._r, [])

    @child_ids.setter
    def child_ids(self, v) -> None:
        self._g.children[self._r] = list(v)
        self._g.set_scalar(self._r, "dirty", 1)

    @property
    def parent_id(self) -> Optional[str]:
        p = int(self._g.get_scalar(self._r, "parent"))
        return self._g.ids[p] if p >= 0 else None

    @parent_id.setter
    def parent_id(self, v: Optional[str]) -> None:
        self._g.set_scalar(self._r, "parent", self._g._ensure_row(v) if v else -1)

    @property
    def shard_key(self) -> str:
        s = int(self._g.get_scalar(self._r, "shard"))
        return self._g.shard_names[s] if s >= 0 else DEFAULT_SHARD

    @shard_key.setter
    def shard_key(self, v: str) -> None:
        # moving a node between shards is a graph operation (counters, edges):
        # only the label changes here, like assigning the reference's attribute
        g = self._g
        old = int(g.get_scalar(self._r, "shard"))
        new = g.shard_id(v)
        if old == new:
            return
        if g.kind_h(self._r) == NODE and not g.sup_h(self._r):
            if old >= 0:
                g.shard_count[old] -= 1
            g.shard_count[new] += 1
        g.set_scalar(self._r, "shard", new)
        g._bump(edges=True)

    def __eq__(self, other):
        if isinstance(other, NodeView):
            return self._g is other._g and self._r == other._r
        return Node.__eq__(self, other)

    __hash__ = object.__hash__


class NodeList(Sequence):
    """One query's search result -- the list of ``Node`` views the reference
    returns (memory_system.py:1460-1472) -- backed by the result's row array.
    A :class:`NodeView` is made when an element is read, so a serving step
    that only passes results along allocates no Python object per row (the
    collector then has nothing new to walk; bench.py needs no gc.freeze).
    Compares equal to a list of the same nodes."""
    __slots__ = ("_g", "_rows")

    def __init__(self, g: TenantGraph, rows: np.ndarray):
        self._g, self._rows = g, rows

    @property
    def rows(self) -> np.ndarray:
        return self._rows

    def __len__(self) -> int:
        return int(self._rows.shape[0])

    def __getitem__(self, i):
        if isinstance(i, slice):
            return [NodeView.of(self._g, r) for r in self._rows[i].tolist()]
        return NodeView.of(self._g, int(self._rows[i]))

    def __iter__(self):
        g = self._g
        for r in self._rows.tolist():
            yield NodeView.of(g, r)

    def __eq__(self, other):
        if isinstance(other, (list, tuple, Sequence)) and not isinstance(other, str):
            return list(self) == list(other)
        return NotImplemented

    def __add__(self, other):
        return list(self) + list(other)

    def __radd__(self, other):
        return list(other) + list(self)

    def __repr__(self) -> str:
        return repr(list(self))


class ResultBatch(Sequence):
    """A batch's search results: ``res[q]`` is query q's :class:`NodeList`.
    Holds the [nq, k] row array (-1 = empty slot or a row that is not a
    node, marked on the device) and nothing per row."""
    __slots__ = ("_g", "_rows")

    def __init__(self, g: TenantGraph, rows: np.ndarray):
        self._g, self._rows = g, np.asarray(rows, dtype=np.int64)

    @property
    def rows(self) -> np.ndarray:
        return self._rows

    def __len__(self) -> int:
        return int(self._rows.shape[0])

    def _one(self, q: int) -> NodeList:
        r = self._rows[q]
        return NodeList(self._g, r[r >= 0])

    def __getitem__(self, i):
        if isinstance(i, slice):
            return [self._one(q) for q in range(len(self))[i]]
        if i < 0:
            i += len(self)
        if not 0 <= i < len(self):
            raise IndexError("ResultBatch index out of range")
        return self._one(i)

    def __iter__(self):
        for q in range(len(self)):
            yield self._one(q)

    def __eq__(self, other):
        if isinstance(other, (list, tuple, Sequence)) and not isinstance(other, str):
            return len(self) == len(other) and all(a == b for a, b in zip(self, other))
        return NotImplemented

    def __repr__(self) -> str:
        return repr([list(x) for x in self])


def _node_kwargs(node: Node) -> Dict:
    return {f: getattr(node, f) for f in ("id", "content", "embedding", "type", "timestamp", "access_count",
                                          "last_accessed", "salience", "is_super_node", "child_ids", "parent_id",
                                          "shard_key")}


def import_nodes(g: TenantGraph, nodes: List[Node], shard_names: List[str], supers: Optional[List[bool]] = None,
                 stored: bool = False, adopt: bool = True) -> torch.Tensor:
    """Add Python ``Node`` objects (a batch) to the graph; adopt them as views."""
    if not nodes:
        return torch.zeros(0, dtype=torch.long)
    kws = [_node_kwargs(n) for n in nodes]
    codes = [g.shard_id(s) for s in shard_names]
    sup = supers if supers is not None else [bool(k["is_super_node"]) for k in kws]
    children = {j: list(k["child_ids"]) for j, k in enumerate(kws) if k["child_ids"] or sup[j]}
    rows = g.add_nodes([k["id"] for k in kws], [k["content"] for k in kws], [k["embedding"] for k in kws],
                       shard=codes, types=[k["type"] for k in kws], sal=[float(k["salience"]) for k in kws],
                       acc=[int(k["access_count"]) for k in kws], last=[float(k["last_accessed"]) for k in kws],
                       ts=[float(k["timestamp"]) for k in kws], sup=[1 if s else 0 for s in sup],
                       parents=[k["parent_id"] for k in kws], children=children, stored=stored)
    if adopt:
        for n, r in zip(nodes, rows.tolist()):
            if not isinstance(n, NodeView) or n._g is not g:
                NodeView.adopt(n, g, r)
    return rows


# ---------------------------------------------------------------- edges
class EdgeView(Edge):
    """An ``Edge`` whose fields live in the graph's edge columns. It is keyed
    by (shard, source row, target row); the column index is re-resolved when
    the edge list has been compacted since it was last looked up."""

    @classmethod
    def of(cls, g: TenantGraph, shard_code: int, s: int, d: int, idx: int = -1) -> "EdgeView":
        v = object.__new__(cls)
        v.__dict__.update(_g=g, _sc=shard_code, _s=s, _d=d, _i=idx, _ver=g.edge_version if idx >= 0 else -1)
        return v

    @classmethod
    def adopt(cls, edge: Edge, g: TenantGraph, shard_code: int, s: int, d: int) -> "EdgeView":
        if type(edge) is Edge:
            edge.__dict__.clear()
            edge.__class__ = cls
            edge.__dict__.update(_g=g, _sc=shard_code, _s=s, _d=d, _i=-1, _ver=-1)
            return edge
        return cls.of(g, shard_code, s, d)

    def _idx(self) -> int:
        g = self._g
        if self._ver != g.edge_version or self._i < 0:
            self.__dict__["_i"] = g.edge_index(self._s, self._d, self._sc)
            self.__dict__["_ver"] = g.edge_version
        if self._i < 0:
            raise KeyError(f"edge {self.source}->{self.target} no longer exists")
        return self._i

    def _get(self, col):
        with self._g.on_stream():
            return self._g.e[col][self._idx()].item()

    def _set(self, col, v):
        g = self._g
        i = self._idx()
        with g.on_stream():
            g.e[col][i] = v
            g.e["meta"][i] = int(g.e["meta"][i].item()) | EDIRTY
        if col == "w":
            g._bump(edges=True)
            self.__dict__["_ver"] = g.edge_version

    source = property(lambda self: self._g.ids[self._s])
    target = property(lambda self: self._g.ids[self._d])
    weight = property(lambda self: float(self._get("w")), lambda self, v: self._set("w", float(v)))
    co_occurrence = property(lambda self: int(self._get("co")), lambda self, v: self._set("co", int(v)))
    last_updated = property(lambda self: float(self._get("lu")), lambda self, v: self._set("lu", float(v)))

    @property
    def edge_type(self) -> str:
        return self._g.etype_names[(int(self._get("meta")) >> TYPE_SHIFT) & TYPE_MASK]

    @edge_type.setter
    def edge_type(self, v: str) -> None:
        c = self._g.etype(v)
        m = int(self._get("meta"))
        self._set("meta", (m & ~(TYPE_MASK << TYPE_SHIFT)) | (c << TYPE_SHIFT))

    def __eq__(self, other):
        if isinstance(other, EdgeView):
            return (self._g is other._g and self._sc == other._sc and self._s == other._s and self._d == other._d)
        return Edge.__eq__(self, other)

    __hash__ = object.__hash__


def import_edges(g: TenantGraph, edges: List[Edge], shard_names: List[str], adopt: bool = True) -> None:
    """``MemoryShard.add_edge`` for a batch of ``Edge`` objects (upsert)."""
    if not edges:
        return
    src = [g._ensure_row(e.source) for e in edges]
    dst = [g._ensure_row(e.target) for e in edges]
    codes = [g.shard_id(s) for s in shard_names]
    et = [g.etype(e.edge_type or "relates_to") for e in edges]
    dev = g.device
    g.upsert_edges(torch.as_tensor(src), torch.as_tensor(dst), torch.as_tensor([float(e.weight) for e in edges]),
                   torch.as_tensor(codes, dtype=torch.int32), torch.as_tensor(et, dtype=torch.int32),
                   co=torch.as_tensor([int(e.co_occurrence) for e in edges], dtype=torch.int32),
                   lu=torch.as_tensor([float(e.last_updated) for e in edges], dtype=torch.float64))
    if adopt:
        for e, s, d, c in zip(edges, src, dst, codes):
            if not isinstance(e, EdgeView):
                EdgeView.adopt(e, g, c, s, d)


# ---------------------------------------------------------------- shard
class _ShardNodes(MutableMapping):
    def __init__(self, g: TenantGraph, code: int):
        self._g, self._c = g, code

    def _rows(self) -> np.ndarray:
        return self._g.node_rows_where(self._c, super_=False)

    def __getitem__(self, k):
        r = self._g.row_of.get(k)
        if r is None or not self._has(r):
            raise KeyError(k)
        return NodeView.of(self._g, r)

    def _has(self, r: int) -> bool:
        g = self._g
        return g.kind_h(r) == NODE and not g.sup_h(r) and int(g.mirror("shard")[r]) == self._c

    def __contains__(self, k) -> bool:
        r = self._g.row_of.get(k)
        return r is not None and self._has(r)

    def __setitem__(self, k, node: Node) -> None:
        import_nodes(self._g, [node], [self._g.shard_names[self._c]], supers=[False])

    def __delitem__(self, k) -> None:
        r = self._g.row_of.get(k)
        if r is None or not self._has(r):
            raise KeyError(k)
        self._g.remove_nodes([r], drop_edges=False)

    def __iter__(self) -> Iterator[str]:
        ids = self._g.ids
        return iter([ids[r] for r in self._rows()])

    def __len__(self) -> int:
        return self._g.shard_count[self._c]

    def values(self):
        g = self._g
        return [NodeView.of(g, int(r)) for r in self._rows()]

    def items(self):
        g = self._g
        return [(g.ids[r], NodeView.of(g, int(r))) for r in self._rows()]


class _ShardEdges(MutableMapping):
    def __init__(self, g: TenantGraph, code: int):
        self._g, self._c = g, code

    def _idx(self):
        g = self._g
        idx = g.edges_of_shard(self._c)
        with g.on_stream():
            s = g.e["src"][idx].tolist()
            d = g.e["dst"][idx].tolist()
        return idx.tolist(), s, d

    def __getitem__(self, key):
        g = self._g
        a, b = g.row_of.get(key[0]), g.row_of.get(key[1])
        if a is None or b is None:
            raise KeyError(key)
        i = g.edge_index(a, b, self._c)
        if i < 0:
            raise KeyError(key)
        return EdgeView.of(g, self._c, a, b, i)

    def __contains__(self, key) -> bool:
        try:
            self[key]
            return True
        except KeyError:
            return False

    def __setitem__(self, key, edge: Edge) -> None:
        g = self._g
        if key in self:
            v = self[key]
            v.weight, v.co_occurrence, v.last_updated = edge.weight, edge.co_occurrence, edge.last_updated
            v.edge_type = edge.edge_type
            return
        import_edges(g, [edge], [g.shard_names[self._c]])

    def __delitem__(self, key) -> None:
        v = self[key]
        self._g.remove_edges(torch.as_tensor([v._idx()], dtype=torch.long))

    def pop(self, key, *default):
        try:
            v = self[key]
        except KeyError:
            if default:
                return default[0]
            raise
        snap = Edge(source=v.source, target=v.target, weight=v.weight, edge_type=v.edge_type,
                    co_occurrence=v.co_occurrence, last_updated=v.last_updated)
        self._g.remove_edges(torch.as_tensor([v._idx()], dtype=torch.long))
        return snap

    def __iter__(self):
        _, s, d = self._idx()
        ids = self._g.ids
        return iter([(ids[a], ids[b]) for a, b in zip(s, d)])

    def __len__(self) -> int:
        return int(self._g.edges_of_shard(self._c).numel())

    def items(self):
        idx, s, d = self._idx()
        g, ids = self._g, self._g.ids
        return [((ids[a], ids[b]), EdgeView.of(g, self._c, a, b, i)) for i, a, b in zip(idx, s, d)]

    def values(self):
        return [v for _, v in self.items()]

    def incident(self, node_id: str) -> List[Tuple[str, str]]:
        g = self._g
        r = g.row_of.get(node_id)
        if r is None:
            return []
        idx = g.edges_incident(r, self._c)
        with g.on_stream():
            s, d = g.e["src"][idx].tolist(), g.e["dst"][idx].tolist()
        return [(g.ids[a], g.ids[b]) for a, b in zip(s, d)]


class ShardView(MemoryShard):
    """``MemoryShard`` bound to one shard of a tenant graph."""

    def __init__(self, g: TenantGraph, code: int):
        object.__setattr__(self, "_g", g)
        object.__setattr__(self, "_c", code)
        meta = g.__dict__.setdefault("_shard_meta", {})
        meta.setdefault(code, {"last_accessed": time.time(), "access_count": 0})

    def __setattr__(self, name, value):
        if name in ("last_accessed", "access_count"):
            self._g._shard_meta[self._c][name] = value
        elif name in ("nodes", "edges"):
            raise AttributeError(f"assign items of shard.{name} instead of replacing the mapping")
        else:
            object.__setattr__(self, name, value)

    shard_key = property(lambda self: self._g.shard_names[self._c])
    nodes = property(lambda self: _ShardNodes(self._g, self._c))
    edges = property(lambda self: _ShardEdges(self._g, self._c))
    last_accessed = property(lambda self: self._g._shard_meta[self._c]["last_accessed"])
    access_count = property(lambda self: self._g._shard_meta[self._c]["access_count"])

    def add_node(self, node: Node) -> None:
        import_nodes(self._g, [node], [self.shard_key], supers=[False])

    def add_edge(self, edge: Edge) -> None:
        import_edges(self._g, [edge], [self.shard_key])

    def get_neighbors(self, node_id: str, min_weight: float = 0.3) -> List[str]:
        g = self._g
        r = g.row_of.get(node_id)
        if r is None:
            return []
        idx = g.edges_incident(r, self._c)
        with g.on_stream():
            w = g.e["w"][idx]
            idx = idx[w >= min_weight]
            s, d = g.e["src"][idx].tolist(), g.e["dst"][idx].tolist()
        return [g.ids[b] if a == r else g.ids[a] for a, b in zip(s, d)]

    def apply_temporal_decay(self, decay_rate: float = 0.01) -> None:
        g = self._g
        keep = 1.0 - decay_rate
        with g.on_stream():
            m = (g.e["meta"] & SHARD_MASK) == self._c
            g.e["w"] = torch.where(m, g.e["w"] * keep, g.e["w"])
            n = g.n
            nm = (g.shard[:n] == self._c) & (g.kind[:n] == NODE) & (g.sup[:n] == 0)
            s = g.sal[:n]
            dec = torch.where(s > SALIENCE_FLOOR, SALIENCE_FLOOR + (s - SALIENCE_FLOOR) * keep,
                              torch.full_like(s, SALIENCE_FLOOR))
            g.sal[:n] = torch.where(nm, dec, s)
        g._bump(edges=True)

    def prune_weak_edges(self, threshold: float = 0.5) -> int:
        g = self._g
        with g.on_stream():
            m = ((g.e["meta"] & SHARD_MASK) == self._c) & (g.e["w"] < threshold)
            idx = torch.nonzero(m).flatten()
        g.remove_edges(idx)
        return int(idx.numel())

    def size(self) -> Tuple[int, int]:
        return len(self.nodes), len(self.edges)

    def remove_node(self, node_id: str) -> bool:
        g = self._g
        r = g.row_of.get(node_id)
        if r is None or r not in set(self.nodes._rows().tolist()):
            return False
        g.remove_nodes([r], drop_edges=True)
        return True


class ShardsMap(MutableMapping):
    """``MemorySystem.shards``: shard name -> :class:`ShardView` (creation order)."""

    def __init__(self, g: TenantGraph):
        self._g = g

    def __getitem__(self, k: str) -> ShardView:
        c = self._g.shard_code.get(k)
        if c is None or not self._g.shard_live[c]:
            raise KeyError(k)
        return ShardView(self._g, c)

    def __setitem__(self, k: str, shard: MemoryShard) -> None:
        g = self._g
        if isinstance(shard, ShardView) and shard._g is g and shard.shard_key == k:
            return
        if k in self:
            del self[k]
        g.shard_id(k)
        nodes = list(shard.nodes.values())
        for n in nodes:
            n.shard_key = k if not isinstance(n, NodeView) else n.shard_key
        import_nodes(g, [n for n in nodes], [k] * len(nodes), supers=[False] * len(nodes))
        edges = list(shard.edges.values())
        import_edges(g, edges, [k] * len(edges))

    def __delitem__(self, k: str) -> None:
        g = self._g
        c = g.shard_code.get(k)
        if c is None or not g.shard_live[c]:
            raise KeyError(k)
        rows = g.node_rows_where(c, super_=False)
        g.remove_nodes(rows.tolist(), drop_edges=True)
        g.remove_edges(g.edges_of_shard(c))
        g.shard_live[c] = False

    def __iter__(self):
        return iter(self._g.live_shards())

    def __len__(self) -> int:
        return len(self._g.live_shards())

    def __contains__(self, k) -> bool:
        c = self._g.shard_code.get(k)
        return c is not None and self._g.shard_live[c]

    def get(self, k, default=None):
        return self[k] if k in self else default


class SuperNodesMap(MutableMapping):
    """``MemorySystem.super_nodes``: id -> super-node view (insertion order)."""

    def __init__(self, g: TenantGraph):
        self._g = g

    def _rows(self):
        return self._g.node_rows_where(super_=True)

    def __getitem__(self, k: str) -> NodeView:
        r = self._g.row_of.get(k)
        if r is None or self._g.kind_h(r) != NODE or not self._g.sup_h(r):
            raise KeyError(k)
        return NodeView.of(self._g, r)

    def __contains__(self, k) -> bool:
        r = self._g.row_of.get(k)
        return r is not None and self._g.kind_h(r) == NODE and bool(self._g.sup_h(r))

    def __setitem__(self, k: str, node: Node) -> None:
        import_nodes(self._g, [node], [node.shard_key or DEFAULT_SHARD], supers=[True])

    def __delitem__(self, k: str) -> None:
        r = self._g.row_of.get(k)
        if r is None or k not in self:
            raise KeyError(k)
        self._g.remove_nodes([r], drop_edges=False)

    def __iter__(self):
        ids = self._g.ids
        return iter([ids[r] for r in self._rows()])

    def __len__(self) -> int:
        return self._g.n_super

    def values(self):
        return [NodeView.of(self._g, int(r)) for r in self._rows()]

    def items(self):
        return [(self._g.ids[r], NodeView.of(self._g, int(r))) for r in self._rows()]


class GraphBuffer(BufferGraph):
    """``BufferGraph`` over a tenant graph (same methods and orderings)."""

    def __init__(self, g: TenantGraph):
        self._g = g

    shards = property(lambda self: ShardsMap(self._g))
    super_nodes = property(lambda self: SuperNodesMap(self._g))

    @property
    def nodes(self) -> Dict[str, Node]:
        g = self._g
        return {g.ids[r]: NodeView.of(g, int(r)) for r in g.ordered_node_rows()}

    @property
    def edges(self) -> Dict[Tuple[str, str], Edge]:
        g = self._g
        merged: Dict[Tuple[str, str], Edge] = {}
        for name in g.live_shards():
            merged.update(_ShardEdges(g, g.shard_code[name]).items())
        return merged

    def add_node(self, node: Node) -> None:
        key = node.shard_key or DEFAULT_SHARD
        import_nodes(self._g, [node], [key], supers=[False])

    def add_edge(self, edge: Edge) -> None:
        g = self._g
        r = g.node_row(edge.source, include_super=False)
        if r >= 0:
            import_edges(g, [edge], [g.shard_names[int(g.mirror("shard")[r])]])
        elif DEFAULT_SHARD in ShardsMap(g):
            import_edges(g, [edge], [DEFAULT_SHARD])

    def get_node(self, node_id: str) -> Optional[Node]:
        r = self._g.node_row(node_id)
        return NodeView.of(self._g, r) if r >= 0 else None

    def get_neighbors(self, node_id: str, min_weight: float = 0.3) -> List[str]:
        g = self._g
        r = g.node_row(node_id, include_super=False)
        return [g.ids[x] for x in g.neighbors(r, min_weight)] if r >= 0 else []

    def update_access(self, node_id: str) -> None:
        r = self._g.node_row(node_id)
        if r >= 0:
            self._g.touch([r])

    def apply_temporal_decay(self, decay_rate: float = 0.01) -> None:
        self._g.decay(decay_rate, None)

    def prune_weak_edges(self, threshold: float = 0.5) -> int:
        return self._g.prune(threshold)

    def get_connected_components(self) -> List[Set[str]]:
        ids = self._g.ids
        return [set(ids[r] for r in comp.tolist()) for comp in self._g.components()]

    def size(self) -> Tuple[int, int]:
        return self._g.num_nodes(), self._g.num_edges

    def get_all_nodes_summary(self) -> List[Dict]:
        g = self._g
        rows = g.ordered_node_rows()
        ts = g.mirror("ts")[rows]
        o = np.argsort(-ts, kind="stable")
        out = []
        for r in rows[o]:
            v = NodeView.of(g, int(r))
            c = v.content
            out.append({"id": v.id, "content": (c[:100] + "...") if len(c) > 100 else c, "type": v.type,
                        "salience": v.salience, "access_count": v.access_count, "shard": v.shard_key})
        return out
