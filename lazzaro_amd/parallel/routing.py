"""Tensor-native request routing for :class:`~.service.DistributedMemoryService`.

The JSON path of ``serve`` ships requests and results as serialized bytes and
builds a dict per hit; that is the general RPC for every per-tenant method.
Search -- the reference's ``search_memories`` (memory_system.py:1460-1472),
the hot serving call -- gets a columnar path here:

* :class:`TenantTable` -- per-rank device table of every resident tenant's
  column base addresses (fp32 rows, store bias, salience, access count, kind,
  super flag, shard) and row count, refreshed only for tenants whose graph
  version moved. A batch over thousands of tenants gathers its per-query
  pointers with one indexing op instead of Python lists per query.
* :func:`local_search` -- the owner's batched search over many of its
  tenants: big tenants through their store search (bf16 MFMA candidate scan
  + fp32 re-rank), the rest in ONE ``segment_topk`` launch over their fp32
  rows (exact -|q-x|^2). Rows the graph does not hold as nodes come back -1.
* :func:`search_routed` -- queries embedded by the front end that received
  them (replicated encoder, data-parallel embed: SURVEY.md §2.5 C2), routed
  to the tenants' owners in ONE ``all_to_all_single`` of packed
  ``[embedding | tenant key | limit]`` int32 rows, answered there, and sent
  back in ONE more as ``[score bits | row]`` (C3 over RCCL/xGMI). Only the
  (rank, tenant, row, score) come back; :func:`resolve` materialises node
  dicts for the hits a caller wants, in one more exchange.
* :func:`search_global_batch` -- every front end's queries against EVERY
  resident tenant of every rank: all-gather of the queries, local search,
  then ONE all-to-all that returns each rank's candidates to the queries'
  origin, merged there by (score desc, key asc) (C1 + K2).

Tenant names travel once: a front end announces a (tenant -> key) pair to an
owner the first time it routes to it (a 63-bit blake2b key; the announcement
rides an object exchange that only runs when some rank has one to send,
decided from the all-gathered count matrix, so steady state is two
all-to-alls and one tiny all-gather per batch).
"""
from __future__ import annotations

import hashlib
import os
from dataclasses import dataclass
from typing import Dict, List, Optional, Sequence, Tuple

import numpy as np
import torch

NODE = 1
# tenants with at least this many rows are searched through their own store
# search (MFMA candidate scan + fp32 re-rank); smaller ones share one fused
# segment_topk launch over their fp32 rows
BIG_ROWS = 1 << 18
_COLS = ("emb32", "bias", "sal", "acc", "kind", "sup", "shard", "emb16")


def tenant_key(name: str, _cache: Dict[str, int] = {}) -> int:
    """Stable 63-bit key of a tenant name (identical on every rank)."""
    k = _cache.get(name)
    if k is None:
        k = int.from_bytes(hashlib.blake2b(name.encode(), digest_size=8).digest(), "little") & ((1 << 63) - 1)
        _cache[name] = k
    return k


class TenantTable:
    """Device table of resident tenants' column base addresses (one column
    per slot) and row counts. A slot is refreshed when its graph object or
    graph version changed since it was written."""

    def __init__(self, device: torch.device):
        self.device = torch.device(device)
        self.slot: Dict[str, int] = {}
        self.state: List[Tuple[object, int, object]] = []
        self.names: List[str] = []
        self.free: List[int] = []
        self.cap = 0
        self.h_ptr = np.zeros((len(_COLS), 0), np.int64)
        self.h_n = np.zeros(0, np.int32)
        self.d_ptr = torch.zeros((len(_COLS), 0), dtype=torch.int64, device=self.device)
        self.d_n = torch.zeros(0, dtype=torch.int32, device=self.device)
        self.h_ld16 = np.zeros(0, np.int64)
        self._dirty = False
        self.gen = 0  # bumped whenever an entry changes (tile tables key on it)
        self._tiles = None

    def _grow(self, need: int) -> None:
        cap = max(need, 2 * self.cap, 64)
        hp = np.zeros((len(_COLS), cap), np.int64)
        hp[:, : self.cap] = self.h_ptr
        hn = np.zeros(cap, np.int32)
        hn[: self.cap] = self.h_n
        hl = np.zeros(cap, np.int64)
        hl[: self.cap] = self.h_ld16
        self.h_ld16 = hl
        # the new slots join the free list (smallest popped first)
        self.free = list(range(cap - 1, self.cap - 1, -1)) + self.free
        self.h_ptr, self.h_n, self.cap = hp, hn, cap
        self.state += [(None, -1, None)] * (cap - len(self.state))
        self.names += [""] * (cap - len(self.names))
        self._dirty = True

    def drop(self, user: str) -> None:
        s = self.slot.pop(user, None)
        if s is not None:
            self.state[s] = (None, -1, None)
            self.h_n[s] = 0
            self.free.append(s)
            self._dirty = True

    def slots(self, users: Sequence[str], systems: Dict[str, object]) -> torch.Tensor:
        """Slot per user (int64 device tensor), refreshing stale entries."""
        return _to_dev(torch.from_numpy(self.slots_host(users, systems)), self.device)

    def slots_host(self, users: Sequence[str], systems: Dict[str, object]) -> np.ndarray:
        """Slot per user (host int64 array), refreshing stale entries (the
        device copy of the table is re-uploaded when an entry changed)."""
        out = np.empty(len(users), np.int64)
        for j, u in enumerate(users):
            s = self.slot.get(u)
            g = systems[u].graph
            if s is None:
                if not self.free:
                    self._grow(len(self.slot) + 1)
                s = self.free.pop()
                self.slot[u] = s
                self.names[s] = u
            st = self.state[s]
            # the slot depends on the column allocations, the row count and
            # the stored-row mask (the bias column), not on row contents
            key = (getattr(g, "_alloc_gen", 0), g.n, g._store_version)
            if st[0] is not g or st[1] != key:
                ok = g.dim is not None and g.n > 0 and g.emb32 is not None
                b = None
                if ok:
                    b = g.store_bias("l2")
                    e, sal, acc, kind, sup, shard = g.column_ptrs()
                    e16 = getattr(g, "emb16", None)
                    self.h_ptr[:, s] = (e, b.data_ptr(), sal, acc, kind, sup, shard,
                                        e16.data_ptr() if e16 is not None else 0)
                    self.h_ld16[s] = e16.stride(0) if e16 is not None else 0
                    self.h_n[s] = g.n
                else:
                    self.h_ptr[:, s] = 0
                    self.h_n[s] = 0
                # the bias tensor is referenced here: a later store_bias() that
                # replaces the graph's cached one cannot free memory the table
                # still points at
                self.state[s] = (g, key, b)
                self._dirty = True
            out[j] = s
        if self._dirty:
            self.d_ptr = _to_dev(torch.from_numpy(self.h_ptr.copy()), self.device)
            self.d_n = _to_dev(torch.from_numpy(self.h_n.copy()), self.device)
            self._dirty = False
            self.gen += 1
        return out

    def tiles(self, slots: np.ndarray):
        """Tile table (ops/search.py MtTiles) of these slots' tenants, rebuilt
        only when an entry or the slot set changed."""
        from ..ops.search import MtTiles
        slots = np.asarray(slots, np.int64)
        key = (self.gen, slots.tobytes())
        if self._tiles is None or self._tiles[0] != key:
            ld = self.h_ld16[slots]
            if ld.size and (ld != ld[0]).any():
                raise ValueError("tile table: tenants with different bf16 row strides")
            t = MtTiles(slots, self.h_n[slots], self.h_ptr[7, slots], self.h_ptr[1, slots],
                        int(ld[0]) if ld.size else 0, self.device)
            self._tiles = (key, t)
        return self._tiles[1]


def _to_dev(t: torch.Tensor, device: torch.device) -> torch.Tensor:
    """Host tensor -> device (async through pinned memory on a GPU)."""
    if device.type == "cuda":
        return t.pin_memory().to(device, non_blocking=True)
    return t


def _fused_ok(ms, D: int, k: int) -> bool:
    g = ms.graph
    return (g.on_gpu and g.dim == D and D % 32 == 0 and k <= 16 and ms._store_binds_graph()
            and getattr(ms.store, "metric", "l2") == "l2" and g.n < BIG_ROWS)


def local_search(svc, users: Sequence[str], Q: torch.Tensor, limits: Sequence[int]):
    """Owner-side batched store search: query ``q`` against tenant
    ``users[q]`` (all owned by this rank), ``limits[q]`` results. Returns
    (scores fp32 [n, k], rows int64 [n, k]) on the device, k = max(limits);
    entries past a query's limit and rows that are not nodes are -1 / -inf
    (the reference skips ids the graph does not hold, :1467-1472)."""
    n = len(users)
    k = max(limits) if n else 1
    systems = {u: svc.system(u) for u in dict.fromkeys(users)}
    dev = next(iter(systems.values())).graph.device if systems else Q.device
    S = torch.full((n, k), float("-inf"), dtype=torch.float32, device=dev)
    R = torch.full((n, k), -1, dtype=torch.int64, device=dev)
    if n == 0:
        return S, R
    Q = Q.to(dev, torch.float32)
    D = Q.shape[1]
    groups: Dict[str, List[int]] = {}
    for j, u in enumerate(users):
        groups.setdefault(u, []).append(j)
    fused = [u for u in groups if _fused_ok(systems[u], D, k)]
    fs = set(fused)
    per = [u for u in groups if u not in fs]
    locks = [systems[u]._graph_lock for u in sorted(systems)]
    for lk in locks:
        lk.acquire()
    try:
        for u in per:
            ms = systems[u]
            g = ms.graph
            if g.dim != D or g.n == 0:
                continue
            whole = len(groups[u]) == n  # one tenant takes the whole batch: no gather / scatter
            idx = None if whole else torch.as_tensor(groups[u], dtype=torch.long).to(dev, non_blocking=True)
            s, r = g.store_search(Q if whole else Q[idx], k, getattr(ms.store, "metric", "l2"))
            with g.on_stream():
                bad = (r < 0) | (g.kind[r.clamp_min(0)] != NODE)
            s = torch.where(bad, torch.full_like(s, float("-inf")), s.float())
            r = torch.where(bad, torch.full_like(r, -1), r)
            if whole:
                S, R = s, r
            else:
                S[idx], R[idx] = s, r
        if fused:
            from ..ops.search import segment_topk_ptrs
            from ..ops.tenant_ops import gather_fields
            qi = [j for u in fused for j in groups[u]]
            qu = [users[j] for j in qi]
            table = svc.tenant_table(dev)
            slots = table.slots(qu, systems)
            ptrs = table.d_ptr[:, slots]
            nrows = table.d_n[slots]
            qt = _to_dev(torch.as_tensor(qi, dtype=torch.long), dev)
            Qs = Q[qt].contiguous()
            s, r = segment_topk_ptrs(ptrs[0].contiguous(), nrows.contiguous(), D, Qs, k,
                                     bptr=ptrs[1].contiguous(), alpha=2.0, qbias=-(Qs * Qs).sum(1))
            # kind of every result row: one gather over the per-query column pointers
            o = gather_fields(r, None, device_out=True, base=ptrs[2:7].contiguous())
            bad = (r < 0) | (o["kind"] != NODE)
            S[qt] = torch.where(bad, torch.full_like(s, float("-inf")), s)
            R[qt] = torch.where(bad, torch.full_like(r, -1), r)
        if dev.type == "cuda":
            # the fused launches above read the tenants' columns through raw
            # addresses asynchronously: order each graph's stream after them
            # before its lock goes, so a column reallocated (and its memory
            # reused in the graph stream's order) cannot be read stale
            cur = torch.cuda.current_stream(dev)
            for u in fused:
                gs = getattr(systems[u].graph, "stream", None)
                if gs is not None and gs.cuda_stream != cur.cuda_stream:
                    gs.wait_stream(cur)
        # a query's results past its own limit are dropped
        if min(limits) < k:  # decided on the host: no device sync on the serving path
            lim = torch.as_tensor(list(limits), dtype=torch.long).to(dev, non_blocking=True)
            cut = torch.arange(k, device=dev)[None, :] >= lim[:, None]
            S = torch.where(cut, torch.full_like(S, float("-inf")), S)
            R = torch.where(cut, torch.full_like(R, -1), R)
        # valid hits first, in score order (a filtered row leaves a hole)
        o = torch.sort(torch.where(R >= 0, S, torch.full_like(S, float("-inf"))), dim=1, descending=True,
                       stable=True).indices
        return torch.gather(S, 1, o), torch.gather(R, 1, o)
    finally:
        for lk in reversed(locks):
            lk.release()


@dataclass
class RoutedHits:
    """Result of :func:`search_routed`, in the caller's query order:
    ``scores`` fp32 [n, k] and ``rows`` int64 [n, k] (-1 = no hit) on the
    caller's device, ``owner`` the rank holding each query's tenant."""
    users: List[str]
    owner: List[int]
    scores: torch.Tensor
    rows: torch.Tensor

    def local_nodes(self, svc, q: int) -> list:
        """Lazy node views of query ``q``'s hits (its tenant must be local)."""
        from ..engine.views import NodeView
        g = svc.system(self.users[q]).graph
        return [NodeView.of(g, int(r)) for r in self.rows[q].tolist() if r >= 0]


def _pack_queries(Q: torch.Tensor, keys: Sequence[int], limits: Sequence[int]) -> torch.Tensor:
    """[n, D + 3] int32 rows: the fp32 embedding bits, the tenant key (lo,
    hi) and the limit -- one tensor, one all-to-all."""
    kk = np.asarray(keys, dtype=np.int64)
    meta = np.stack([(kk & 0xFFFFFFFF).astype(np.uint32).view(np.int32), (kk >> 32).astype(np.int32),
                     np.asarray(limits, np.int32)], 1)
    m = torch.from_numpy(meta)
    if Q.is_cuda:
        m = m.pin_memory().to(Q.device, non_blocking=True)
    return torch.cat([Q.float().contiguous().view(torch.int32), m], 1)


def _unpack_keys(meta: np.ndarray) -> List[int]:
    lo = meta[:, 0].astype(np.int64) & 0xFFFFFFFF
    hi = meta[:, 1].astype(np.int64)
    return ((hi << 32) | lo).tolist()


def search_routed(svc, users: Sequence[str], Q: torch.Tensor, limit=5) -> RoutedHits:
    """SPMD batched ``search_memories`` of queries already embedded by this
    rank's front end, each against its tenant ``users[q]`` wherever it is
    owned. Every rank must call it (possibly with no queries).

    Host metadata goes over the communicator's gloo group: one all-gather of
    a [W, 6] header (rows to send, announcements, width, k, the directory
    epoch this rank believes the destination has, its own epoch) gives every
    rank its all-to-all split sizes with no device-to-host read. The queries
    and the results cross in two RCCL all-to-alls. An owner whose every
    sender knew its current directory (all tenants they route to were
    announced to it and are pinned resident) maps the received tenant keys
    on the device (:func:`_owner_search_device`); otherwise it reads the keys
    back and serves by name (:func:`local_search`)."""
    comm = svc.comm
    W, me = comm.world, comm.rank
    n = len(users)
    limits = [int(limit)] * n if np.isscalar(limit) else [int(x) for x in limit]
    owner = [svc.owner(u) for u in users]
    if W == 1 and not svc.force_collectives:
        S, R = local_search(svc, list(users), Q, limits) if n else (
            torch.zeros((0, int(limit) if np.isscalar(limit) else 1)), torch.zeros((0, 1), dtype=torch.long))
        return RoutedHits(list(users), owner, S, R)
    dev = comm.device
    D = int(Q.shape[1]) if n else 0
    order = sorted(range(n), key=lambda j: owner[j])
    send_n = np.bincount(np.asarray(owner, np.int64), minlength=W) if n else np.zeros(W, np.int64)
    # first-time (tenant -> key) announcements per owner (this rank included:
    # an announced tenant is pinned resident by its owner)
    ann: List[List] = [[] for _ in range(W)]
    for u, r in zip(users, owner):
        if u not in svc._announced[r]:
            svc._announced[r].add(u)
            ann[r].append(u)
    for u in users:
        svc._key_names[tenant_key(u)] = u
    kmax = max(limits) if n else 0
    hdr = np.array([[int(send_n[r]), len(ann[r]), D, kmax, svc._owner_epoch.get(r, -1), svc._dir_epoch]
                    for r in range(W)], np.int64)
    allc = comm.host_all_gather(hdr)  # [src, dst, field]
    epoch0 = svc._dir_epoch
    for r in range(W):  # an owner whose directory changed hears every tenant again
        e = int(allc[r, 0, 5])
        prev = svc._owner_epoch.get(r)
        if prev != e:
            svc._owner_epoch[r] = e
            if prev is not None:
                svc._announced[r] = set()
    if allc[:, :, 1].sum():
        for part in comm.exchange_objects(ann):
            for u in part or []:
                svc._key_names[tenant_key(u)] = u
                if svc.is_local(u):
                    svc.pin(u)
    Dg = int(allc[:, :, 2].max())
    K = int(allc[:, :, 3].max())
    recv_n = allc[:, me, 0]
    if Dg == 0 or K == 0:
        return RoutedHits(list(users), owner, torch.zeros((n, 1)), torch.full((n, 1), -1, dtype=torch.long))
    senders_current = all(int(allc[s, me, 4]) == epoch0 for s in range(W) if allc[s, me, 0] > 0)
    ddir = svc.device_directory(Dg, K) if (senders_current and svc._dir_epoch == epoch0) else None
    on_device = ddir is not None
    # the permutations travel as pinned async copies: a pageable host -> device
    # copy would wait for every kernel already queued (the previous batch's
    # search), i.e. a host sync per routed batch
    order_h = np.asarray(order, np.int64)
    Qo = Q[_to_dev(torch.from_numpy(order_h), Q.device)] if n else torch.zeros((0, Dg), device=dev)
    pay = _pack_queries(Qo, [tenant_key(users[j]) for j in order], [limits[j] for j in order]) if n else \
        torch.zeros((0, Dg + 3), dtype=torch.int32)
    got = comm.all_to_all_v(pay.to(dev), send_n.tolist(), recv_n.tolist())
    m = got.shape[0]
    svc.route_stats["device" if (m and on_device) else "host"] += 1
    if m:
        if on_device:
            S, R = _owner_search_device(svc, got, Dg, K, ddir)
        else:
            meta = got[:, Dg:].cpu().numpy()
            rusers = [svc._key_names[x] for x in _unpack_keys(meta)]
            S, R = local_search(svc, rusers, got[:, :Dg].contiguous().view(torch.float32), meta[:, 2].tolist())
        if S.shape[1] < K:
            S = torch.cat([S, torch.full((m, K - S.shape[1]), float("-inf"), device=S.device)], 1)
            R = torch.cat([R, torch.full((m, K - R.shape[1]), -1, dtype=R.dtype, device=R.device)], 1)
        back = torch.cat([S.float().contiguous().view(torch.int32), R.to(torch.int32)], 1).to(dev)
    else:
        back = torch.zeros((0, 2 * K), dtype=torch.int32, device=dev)
    res = comm.all_to_all_v(back.contiguous(), recv_n.tolist(), send_n.tolist())
    inv = np.empty(n, np.int64)
    inv[order_h] = np.arange(n)
    res = res[_to_dev(torch.from_numpy(inv), res.device)]
    S = res[:, :K].contiguous().view(torch.float32)
    R = res[:, K:].to(torch.int64)
    return RoutedHits(list(users), owner, S, R)


def _owner_search_device(svc, got: torch.Tensor, Dg: int, K: int, ddir):
    """Owner side of :func:`search_routed` without reading the received
    rows back (:meth:`DistributedMemoryService.device_directory`): each
    row's tenant key is looked up on the device in the sorted keys of the
    pinned small tenants -- one segment_topk over their tenant-table rows
    serves every such row -- and matched against the pinned large tenants,
    each of which runs its store search over the batch (a row keeps the
    results of the tenant whose key it carries). Rows past a query's limit
    and rows that are not nodes come back -1 / -inf, valid hits first (as
    :func:`local_search`)."""
    m = got.shape[0]
    dev = got.device
    lo = got[:, Dg].long() & 0xFFFFFFFF
    keys = (got[:, Dg + 1].long() << 32) | lo
    lim = got[:, Dg + 2].long()
    Qr = got[:, :Dg].contiguous().view(torch.float32)
    S = torch.full((m, K), float("-inf"), dtype=torch.float32, device=dev)
    R = torch.full((m, K), -1, dtype=torch.int64, device=dev)
    dk = ddir["keys"]
    if dk.numel():
        from ..ops.search import segment_topk_ptrs
        from ..ops.tenant_ops import gather_fields
        table = ddir["table"]
        tdev = dk.device
        kk = keys.to(tdev)
        pos = torch.searchsorted(dk, kk).clamp_max(dk.numel() - 1)
        hit = dk[pos] == kk
        slot = ddir["slots"][pos]
        ptrs = table.d_ptr[:, slot]
        nrows = torch.where(hit, table.d_n[slot], torch.zeros_like(table.d_n[slot])).contiguous()
        Qs = Qr.to(tdev)
        cur = torch.cuda.current_stream(tdev) if tdev.type == "cuda" else None
        for st in ddir["streams"]:  # the tenants' pending column writes first
            if st.cuda_stream != cur.cuda_stream:
                cur.wait_stream(st)
        s, r = segment_topk_ptrs(ptrs[0].contiguous(), nrows, Dg, Qs, K, bptr=ptrs[1].contiguous(), alpha=2.0,
                                 qbias=-(Qs * Qs).sum(1))
        o = gather_fields(r, None, device_out=True, base=ptrs[2:7].contiguous())
        ok = hit[:, None] & (r >= 0) & (o["kind"] == NODE)
        S = torch.where(ok.to(dev), s.to(dev), S)
        R = torch.where(ok.to(dev), r.to(dev), R)
        # the fused scan read the tenants' columns through raw addresses: order
        # their streams after it before anything can move a column
        for st in ddir["streams"]:
            if st.cuda_stream != cur.cuda_stream:
                st.wait_stream(cur)
    for user in ddir["big"]:
        key = tenant_key(user)
        ms = svc.systems[user]
        g = ms.graph
        with ms._graph_lock:
            s, r = g.store_search(Qr.to(g.device), K, getattr(ms.store, "metric", "l2"))
            with g.on_stream():
                ok = (r >= 0) & (g.kind[r.clamp_min(0)] == NODE)
        ok = ok.to(dev) & (keys == key)[:, None]
        S = torch.where(ok, s.float().to(dev), S)
        R = torch.where(ok, r.to(dev), R)
    cut = torch.arange(K, device=dev)[None, :] >= lim[:, None]
    S = torch.where(cut, torch.full_like(S, float("-inf")), S)
    R = torch.where(cut, torch.full_like(R, -1), R)
    o = torch.sort(torch.where(R >= 0, S, torch.full_like(S, float("-inf"))), dim=1, descending=True,
                   stable=True).indices
    return torch.gather(S, 1, o), torch.gather(R, 1, o)


def resolve(svc, hits: RoutedHits) -> List[List[Dict]]:
    """SPMD: node dicts of every hit (one object exchange there and back)."""
    from .service import _view, node_dict
    comm = svc.comm
    rows = hits.rows.cpu().tolist()
    want: List[List] = [[] for _ in range(comm.world)]
    for q, (u, r) in enumerate(zip(hits.users, hits.owner)):
        want[r].append([q, u, [x for x in rows[q] if x >= 0]])
    inbox = svc._exchange(want)
    reply: List[List] = [[] for _ in range(comm.world)]
    for src, items in enumerate(inbox):
        for q, u, rr in items:
            ms = svc.system(u)
            with ms._graph_lock:
                reply[src].append([q, [node_dict(_view(ms.graph, x)) for x in rr]])
    out: List[List[Dict]] = [[] for _ in hits.users]
    for items in svc._exchange(reply):
        for q, nodes in items:
            out[q] = nodes
    return out


@dataclass
class GlobalHits:
    """:func:`search_global_batch` result: ``scores`` [b, k]; ``keys`` [b, k]
    int64 = rank << 56 | tenant slot << 32 | row (-1 = none) -- the merge's
    total order; a slot is only meaningful on its rank at search time (slots
    are recycled when tenants leave). ``tenant_keys`` [b, k] int64 is the
    stable 63-bit :func:`tenant_key` of each hit's tenant (-1 = none):
    :meth:`users` maps them to names."""
    scores: torch.Tensor
    keys: torch.Tensor
    tenant_keys: Optional[torch.Tensor] = None

    def split(self) -> Tuple[torch.Tensor, torch.Tensor, torch.Tensor]:
        k = self.keys
        return k >> 56, (k >> 32) & 0xFFFFFF, k & 0xFFFFFFFF

    def users(self, svc) -> List[List[Optional[str]]]:
        """Tenant name of every hit (None past the hits). Names this rank
        has not seen yet come from :meth:`DistributedMemoryService.get_all_users`
        (a collective: call it on every rank when a hit can name a tenant
        only another rank has served)."""
        names = svc._key_names
        return [[names.get(int(t)) if t >= 0 else None for t in row] for row in self.tenant_keys.tolist()]


def search_global_batch(svc, Q: torch.Tensor, limit: int = 5) -> GlobalHits:
    """SPMD global search: each rank's queries against every resident tenant
    of every rank (exact store scores). One all-gather of the queries, the
    local search over this rank's tenants, and ONE all-to-all returning each
    rank's top-``limit`` candidates to the queries' origin, merged there."""
    comm = svc.comm
    W, me = comm.world, comm.rank
    dev = comm.device
    b = int(Q.shape[0])
    force = W > 1 or svc.force_collectives
    counts = comm.host_all_gather(np.array([b, int(Q.shape[1]) if b else 0], np.int64))  # gloo: no GPU sync
    nb = counts[:, 0]
    D = int(counts[:, 1].max())
    B = int(nb.max()) if force else b
    Qp = torch.zeros((B, D), dtype=torch.float32, device=dev)
    if b:
        Qp[:b] = Q.to(dev, torch.float32)
    Qall = comm.all_gather_rows(Qp) if force else Qp  # [W * B, D]
    NQ = Qall.shape[0]
    best_s = torch.full((NQ, limit), float("-inf"), dtype=torch.float32, device=dev)
    best_k = torch.full((NQ, limit), -1, dtype=torch.int64, device=dev)
    best_t = torch.full((NQ, limit), -1, dtype=torch.int64, device=dev)
    gd = svc.global_directory(D, limit) if D else None
    redo = None
    if gd is not None and gd["small"] and NQ:
        if len(gd["small"]) >= MT_MIN_TENANTS and limit <= 16:  # (mt_topk's re-rank headroom: k <= 16)
            # the small tenants: ONE multi-tenant MFMA pass (ops/search.py mt_topk)
            s, key, tk, redo = _global_small(svc, gd, Qall, limit, me, dev)
            best_s, best_k, best_t = _merge(torch.cat([best_s, s], 1), torch.cat([best_k, key], 1), limit,
                                            torch.cat([best_t, tk], 1))
            per = [(u, int(sl), redo) for u, sl in zip(gd["small"], gd["slots"].tolist())] if redo is not None \
                else []
        else:
            per = [(u, int(sl), None) for u, sl in zip(gd["small"], gd["slots"].tolist())]
    else:
        per = []
    per += [(u, sl, None) for u, sl in (gd["big"] if gd is not None else [])]
    for u, slot, qsel in per:
        ms = svc.systems[u]
        g = ms.graph
        Qi = Qall if qsel is None else Qall[qsel]
        with ms._graph_lock:
            s, r = g.store_search(Qi.to(g.device), limit, getattr(ms.store, "metric", "l2"))
            with g.on_stream():
                ok = (r >= 0) & (g.kind[r.clamp_min(0)] == NODE)
        s = torch.where(ok, s.float(), torch.full_like(s, float("-inf"))).to(dev)
        key = torch.where(ok, (me << 56) | (int(slot) << 32) | r, torch.full_like(r, -1)).to(dev)
        tk = torch.where(ok, torch.full_like(r, tenant_key(u)), torch.full_like(r, -1)).to(dev)
        if qsel is None:
            best_s, best_k, best_t = _merge(torch.cat([best_s, s], 1), torch.cat([best_k, key], 1), limit,
                                            torch.cat([best_t, tk], 1))
        else:
            m_s, m_k, m_t = _merge(torch.cat([best_s[qsel], s], 1), torch.cat([best_k[qsel], key], 1), limit,
                                   torch.cat([best_t[qsel], tk], 1))
            best_s[qsel], best_k[qsel], best_t[qsel] = m_s, m_k, m_t
    if not force:
        return GlobalHits(best_s[:b], best_k[:b], best_t[:b])
    # candidates for rank j's queries go back to rank j
    pay = torch.cat([best_s.contiguous().view(torch.int32).reshape(NQ, limit),
                     best_k.view(torch.int32).reshape(NQ, 2 * limit),
                     best_t.view(torch.int32).reshape(NQ, 2 * limit)], 1)
    got = comm.all_to_all_v(pay, [B] * W, [B] * W)  # [W(src) * B, 5 * limit]
    gs = got[:, :limit].contiguous().view(torch.float32).reshape(W, B, limit)
    gk = got[:, limit:3 * limit].contiguous().view(torch.int64).reshape(W, B, limit)
    gt = got[:, 3 * limit:].contiguous().view(torch.int64).reshape(W, B, limit)
    gs = gs.permute(1, 0, 2).reshape(B, W * limit)
    gk = gk.permute(1, 0, 2).reshape(B, W * limit)
    gt = gt.permute(1, 0, 2).reshape(B, W * limit)
    s, k, t = _merge(gs, gk, limit, gt)
    return GlobalHits(s[:b], k[:b], t[:b])


# global search over >= MT_MIN_TENANTS small tenants: one multi-tenant pass
# (MT_GLOBAL = False: the per-tenant store searches)
MT_GLOBAL = True
MT_MIN_TENANTS = 2


def _global_small(svc, gd, Qall: torch.Tensor, limit: int, me: int, dev):
    """Every query against every small tenant of the global directory
    (:meth:`DistributedMemoryService.global_directory`) in one tile-table
    pass. Returns (scores, keys = rank << 56 | slot << 32 | row, tenant keys,
    the queries whose candidate list overflowed -- None when none did -- to be
    redone by the per-tenant path; those queries' rows here are empty)."""
    from ..ops.search import mt_topk
    table = gd["table"]
    locks = [svc.systems[u]._graph_lock for u in gd["small"]] if gd["lock"] else []
    for lk in locks:
        lk.acquire()
    try:
        gdev = table.device
        cur = torch.cuda.current_stream(gdev)
        for st in gd["streams"]:  # the tenants' pending column writes first
            if st.cuda_stream != cur.cuda_stream:
                cur.wait_stream(st)
        tiles = table.tiles(gd["slots"])
        s, key, ovf = mt_topk(tiles, Qall.to(gdev), limit, table.d_ptr[0], table.d_ptr[1], table.d_ptr[4])
        for st in gd["streams"]:  # no column freed / reused under the pass
            if st.cuda_stream != cur.cuda_stream:
                st.wait_stream(cur)
    finally:
        for lk in reversed(locks):
            lk.release()
    ok = key >= 0
    tk = torch.where(ok, gd["tkeys"][(key >> 32).clamp_min(0)], torch.full_like(key, -1))
    key = torch.where(ok, (me << 56) | key, torch.full_like(key, -1))
    redo = None
    if bool((ovf != 0).any()):  # rare: pathological score distributions
        redo = torch.nonzero(ovf != 0).flatten()
        s[redo] = float("-inf")
        key[redo] = -1
        tk[redo] = -1
    return s.to(dev), key.to(dev), tk.to(dev), redo if redo is None else redo.to(dev)


def _merge(s: torch.Tensor, key: torch.Tensor, k: int, extra: Optional[torch.Tensor] = None):
    """Top-k by (score desc, key asc; -1 keys last) -- the same total order on
    every rank, so the merge is independent of arrival order. ``extra`` (a
    per-candidate payload) follows its candidate."""
    kk = torch.where(key >= 0, key, torch.full_like(key, (1 << 63) - 1))
    o = torch.argsort(kk, dim=1, stable=True)
    s, key = torch.gather(s, 1, o), torch.gather(key, 1, o)
    if extra is not None:
        extra = torch.gather(extra, 1, o)
    o = torch.sort(s, dim=1, descending=True, stable=True).indices[:, :k]
    if extra is not None:
        return torch.gather(s, 1, o), torch.gather(key, 1, o), torch.gather(extra, 1, o)
    return torch.gather(s, 1, o), torch.gather(key, 1, o)
