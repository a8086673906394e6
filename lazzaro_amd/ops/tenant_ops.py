"""Tenant-graph maintenance ops (``csrc/kernels/tenant.hip``).

Device tensors go through the HIP kernels; CPU tensors through torch code that
computes the same thing (the CPU test tier, not a fallback: ``_lib.lib()``
raises on a GPU box without the kernel library).

Layout (see :mod:`lazzaro_amd.engine.tenant_graph`): nodes ``sal f32, acc
i32, last f64, kind u8, sup u8, shard i32, dirty u8``; edges ``src/dst i32,
w f32, co i32, lu f64, meta i32 (shard | type << 24)``.
"""
from __future__ import annotations

import ctypes as C
from typing import Dict, List, Optional, Sequence, Tuple

import numpy as np
import torch

from . import _lib

P, I, L, F = _lib.P, _lib.I, _lib.L, _lib.F
D_ = C.c_double

_lib.register("lzk_tg_decay", I, [P, L, F, F, P, P, P, P, P, L, I, I, P])
_lib.register("lzk_tg_write_emb", I, [P, L, P, I, I, P, L, P, L, P, L, P, L, P, P, P, P, P, P, P])
_lib.register("lzk_tg_set_rows", I, [P, L, I, P, I, P, P, P, P, P, P, P, P, P, P, P, I, I, P])
_lib.register("lzk_store_rerank", I, [P, L, P, L, I, P, P, P, I, I, I, I, P, P, P, P, P])
_lib.register("lzk_tg_flag_remove", I, [P, P, P, L, P, P, P, L, P, P, P])
_lib.register("lzk_tg_compact", I, [P, P, L, P, P, P, P, P, P, P, P, P, P, P, P, P, P, P, P])
_lib.register("lzk_tg_boost", I, [P, P, P, P, P, I, P, P, F, D_, D_, P, P, P, P, I, P, P])
_lib.register("lzk_tg_touch", I, [P, I, P, P, P, P, D_, D_, P])
_lib.register("lzk_tg_importance", I, [P, P, P, P, P, L, D_, P, P])
_lib.register("lzk_tg_evict_verify", I, [P, P, P, P, P, P, P, L, D_, F, I, P, P, P, P, P, P, P, D_, I, D_, I, L])
_lib.register("lzk_scan_blocks", I, [P, I, P, P])
_lib.register("lzk_pack_bits", I, [P, L, P, P])
_lib.register("lzk_tg_gather_fields", I, [P, I, I, P, P, P, P, P, P, P])
_lib.register("lzk_dg_stats", I, [P, P, P, L, P, L, P, P, P, I, D_, I, P, P, P, P, P, P, P, P, P, P])
_lib.register("lzk_dg_select", I, [P, L, P, P, P, P, P, P, I, P, I, P, P, P, P, P, I, P, P, L, P])
_lib.register("lzk_tg_first_rows", I, [P, P, P, L, P, P, P, I, P, P])
_lib.register("lzk_num_rows", I, [P, L, L, P, P, L, P, P, L, P, P, L, P, P])
_lib.register("lzk_row_cent_cos", I, [P, L, I, P, P, P, L, P, L, P, P])
_lib.register("lzk_dg_small_ws", L, [I])
_lib.register("lzk_tg_append_edges", I, [P, I, L, I, D_, P, P, P, P, P, P, P])
_lib.register("lzk_tg_seg_end", I, [P, I, P, P, P, P, I, P, P, P, P, L, P, L, P, P, P, P])
_lib.register("lzk_dg_small_max_edges", I, [])
_lib.register("lzk_dg_small", I, [P, P, P, I, P, P, P, L, I, D_, I, P, P, I, P, P])

SALIENCE_FLOOR = 0.2
EDGE_COLS = ("src", "dst", "w", "co", "lu", "meta")
NTB = 256


def _st(t: torch.Tensor) -> int:
    return _lib.stream_ptr(t.device)


def to_dev_packed(cols: Sequence, dev) -> List[torch.Tensor]:
    """Equal-length host columns -> device float64 rows through ONE pinned,
    non-blocking copy (exact for int32 / fp32 / fp64 and integers below 2^53).
    Callers cast each row to its dtype on the device. A pageable ``.to(dev)``
    per column blocks the host once each."""
    m = len(cols[0]) if cols else 0
    blk = torch.empty((len(cols), m), dtype=torch.float64)
    if dev.type == "cuda":
        blk = blk.pin_memory()
    bn = blk.numpy()
    for j, c in enumerate(cols):
        bn[j] = np.asarray(c, dtype=np.float64).reshape(-1)
    d = blk.to(dev, non_blocking=True) if dev.type == "cuda" else blk
    return [d[j] for j in range(len(cols))]


def _compact(e: Dict[str, torch.Tensor], flag: torch.Tensor, bc: torch.Tensor, ne: int, extra: int = 0,
             total: Optional[torch.Tensor] = None, n_out: Optional[int] = None, dropped: bool = False):
    """Stable device compaction of the flagged edges (scan + scatter). With
    ``extra`` each output column is a view of a buffer ``extra`` rows longer
    (room for appends without a copy, :meth:`TenantGraph._edge_append`).
    ``total`` / ``n_out``: the block counts were already scanned and the
    survivor count read by the caller. ``dropped``: also return (src, dst,
    meta) of the removed edges in order, written by the same pass."""
    L_ = _lib.lib()
    dev = e["src"].device
    if n_out is None:
        total = torch.zeros(1, dtype=torch.int32, device=dev)
        _lib.check(L_.lzk_scan_blocks(bc.data_ptr(), bc.numel(), total.data_ptr(), _st(bc)), "scan_blocks")
        n_out = int(total.item())
    if n_out == ne:
        return (e, 0, None) if dropped else (e, 0)
    out = {k: torch.empty(n_out + extra, dtype=e[k].dtype, device=dev)[:n_out] for k in EDGE_COLS}
    dr = [torch.empty(ne - n_out, dtype=torch.int32, device=dev) for _ in range(3)] if dropped else None
    _lib.check(L_.lzk_tg_compact(flag.data_ptr(), bc.data_ptr(), ne, *(e[k].data_ptr() for k in EDGE_COLS),
                                 *(out[k].data_ptr() for k in EDGE_COLS),
                                 *((d.data_ptr() for d in dr) if dr else (None, None, None)), _st(flag)), "tg_compact")
    return (out, ne - n_out, tuple(dr) if dr else None) if dropped else (out, ne - n_out)


def decay_prune(e: Dict[str, torch.Tensor], sal, kind, sup, rate: float, threshold: Optional[float],
                decay_nodes: bool = True, want_dropped: bool = False, steps: int = 1):
    """Temporal decay of every edge and shard-node salience (reference
    memory_shard.py:64-77), ``steps`` rounds (each rounded to fp32, as
    ``steps`` end_conversation calls), then, if ``threshold`` is not None,
    removal of edges with ``w < threshold`` (:79-84) with stable compaction.

    Returns (edges, n_pruned, dropped) where ``dropped`` is (src, dst, meta)
    of the pruned edges when ``want_dropped`` (for incremental persistence)."""
    ne = int(e["src"].numel())
    keep = 1.0 - rate
    nn = int(sal.numel()) if sal is not None else 0
    dropped = None
    if not e["src"].is_cuda:
        for _ in range(steps):
            if rate:
                e["w"].mul_(keep)
            if decay_nodes and nn:
                m = (kind == 1) & (sup == 0)
                dec = torch.where(sal > SALIENCE_FLOOR, SALIENCE_FLOOR + (sal - SALIENCE_FLOOR) * keep,
                                  torch.full_like(sal, SALIENCE_FLOOR))
                sal.copy_(torch.where(m, dec, sal))
        if threshold is None or ne == 0:
            return e, 0, dropped
        f = e["w"] >= threshold
        if want_dropped:
            dropped = (e["src"][~f], e["dst"][~f], e["meta"][~f])
        n_keep = int(f.sum())
        if n_keep == ne:
            return e, 0, dropped
        return {k: v[f] for k, v in e.items()}, ne - n_keep, dropped
    dev = e["src"].device
    nb = max(1, (ne + NTB - 1) // NTB)
    flag = torch.empty(max(ne, 1), dtype=torch.uint8, device=dev) if threshold is not None else None
    bc = torch.empty(nb, dtype=torch.int32, device=dev) if threshold is not None else None
    thr = float(threshold) if threshold is not None else float("-inf")
    _lib.check(_lib.lib().lzk_tg_decay(e["w"].data_ptr(), ne, float(keep), thr, _lib.ptr(flag), _lib.ptr(bc),
                                       _lib.ptr(sal), _lib.ptr(kind), _lib.ptr(sup), nn,
                                       1 if (decay_nodes and nn) else 0, int(steps), _st(e["w"])), "tg_decay")
    if threshold is None or ne == 0:
        return e, 0, dropped
    out, n = _compact(e, flag, bc, ne)
    if want_dropped:  # only when something went (one nonzero, three gathers)
        dropped = _dropped(e, flag, ne, n)
    return out, n, dropped


def _bits(rm: torch.Tensor) -> torch.Tensor:
    """u8 row flags (device) -> int32 bitmap words (bit r of word r >> 5)."""
    n = int(rm.numel())
    bits = torch.empty(max(1, (n + 31) // 32), dtype=torch.int32, device=rm.device)
    _lib.check(_lib.lib().lzk_pack_bits(rm.data_ptr(), n, bits.data_ptr(), _st(rm)), "pack_bits")
    return bits


def _dropped(e: Dict[str, torch.Tensor], flag: torch.Tensor, ne: int, n: int):
    """(src, dst, meta) of the edges whose keep flag is 0 (``n`` of them)."""
    if n == 0:
        z = e["src"][:0]
        return z, e["dst"][:0], e["meta"][:0]
    # the count is known: a fixed-size nonzero, no host synchronisation
    idx = torch.nonzero_static(flag[:ne] == 0, size=n).flatten()
    return e["src"][idx], e["dst"][idx], e["meta"][idx]


def remove_edges_of(e: Dict[str, torch.Tensor], rm: torch.Tensor, shard: torch.Tensor, want_dropped: bool = False):
    """Drop the edges that a removed node's shard stores (reference
    memory_system.py:558-569): edge dropped iff an endpoint has ``rm`` set and
    the edge's shard equals that endpoint's shard. Returns (edges, n, dropped)."""
    ne = int(e["src"].numel())
    if ne == 0:
        return e, 0, None
    es = e["meta"] & 0xFFFFFF
    if not e["src"].is_cuda:
        s, d = e["src"].long(), e["dst"].long()
        drop = (rm[s].bool() & (shard[s] == es)) | (rm[d].bool() & (shard[d] == es))
        dropped = (e["src"][drop], e["dst"][drop], e["meta"][drop]) if want_dropped else None
        n = int(drop.sum())
        if n == 0:
            return e, 0, dropped
        keep = ~drop
        return {k: v[keep] for k, v in e.items()}, n, dropped
    dev = e["src"].device
    nb = max(1, (ne + NTB - 1) // NTB)
    flag = torch.empty(ne, dtype=torch.uint8, device=dev)
    bc = torch.empty(nb, dtype=torch.int32, device=dev)
    rmb = _bits(rm.to(torch.uint8).contiguous())
    _lib.check(_lib.lib().lzk_tg_flag_remove(e["src"].data_ptr(), e["dst"].data_ptr(), e["meta"].data_ptr(), ne,
                                             rmb.data_ptr(), shard.data_ptr(), None, 0, flag.data_ptr(),
                                             bc.data_ptr(), _st(flag)), "tg_flag_remove")
    out, n = _compact(e, flag, bc, ne)
    dropped = _dropped(e, flag, ne, n) if want_dropped else None
    return out, n, dropped


def decay_flags(e: Dict[str, torch.Tensor], sal, kind, sup, rate: float, threshold: Optional[float], steps: int):
    """The decay half of :func:`decay_prune` on the device with the prune
    deferred: ``steps`` decay rounds of every edge and shard-node salience in
    place, and (``threshold`` not None) the keep flag ``w >= threshold`` of
    each current edge, returned for :func:`flag_finish`. No host sync."""
    ne = int(e["src"].numel())
    dev = e["src"].device
    nn = int(sal.numel())
    flag = bc = None
    if threshold is not None and ne:
        flag = torch.empty(ne, dtype=torch.uint8, device=dev)
        bc = torch.empty(max(1, (ne + NTB - 1) // NTB), dtype=torch.int32, device=dev)
    thr = float(threshold) if threshold is not None else float("-inf")
    _lib.check(_lib.lib().lzk_tg_decay(e["w"].data_ptr(), ne, float(1.0 - rate), thr, _lib.ptr(flag), _lib.ptr(bc),
                                       _lib.ptr(sal), _lib.ptr(kind), _lib.ptr(sup), nn, 1 if nn else 0, int(steps),
                                       _st(e["w"])), "tg_decay")
    return flag


def flag_finish(e: Dict[str, torch.Tensor], rm: Optional[torch.Tensor], shard: torch.Tensor,
                prev: Optional[torch.Tensor]):
    """Keep flags of every current edge: ``prev`` (a :func:`decay_flags`
    result over the first ``prev.numel()`` edges; later edges were appended
    since) AND not dropped by the removal of the ``rm`` rows (same rule as
    :func:`remove_edges_of`). Returns (flag, block counts, total) -- the
    survivor count stays on the device until the caller's one sync."""
    ne = int(e["src"].numel())
    dev = e["src"].device
    flag = torch.empty(ne, dtype=torch.uint8, device=dev)
    bc = torch.empty(max(1, (ne + NTB - 1) // NTB), dtype=torch.int32, device=dev)
    total = torch.zeros(1, dtype=torch.int32, device=dev)
    L_ = _lib.lib()
    rmb = _bits(rm) if rm is not None else None
    _lib.check(L_.lzk_tg_flag_remove(e["src"].data_ptr(), e["dst"].data_ptr(), e["meta"].data_ptr(), ne,
                                     _lib.ptr(rmb), shard.data_ptr(), _lib.ptr(prev),
                                     int(prev.numel()) if prev is not None else 0, flag.data_ptr(), bc.data_ptr(),
                                     _st(flag)), "tg_flag_remove")
    _lib.check(L_.lzk_scan_blocks(bc.data_ptr(), bc.numel(), total.data_ptr(), _st(bc)), "scan_blocks")
    return flag, bc, total


def seg_end(vrows: Optional[torch.Tensor], nv: int, kind, sup, shard, stored, unstore: bool, rmb: torch.Tensor,
            e: Dict[str, torch.Tensor], prev: Optional[torch.Tensor], flag: Optional[torch.Tensor],
            bc: Optional[torch.Tensor], info: torch.Tensor) -> None:
    """tenant.hip lzk_tg_seg_end: one segment end of consolidate_batch (see
    TenantGraph.segment_end) -- victims ghosted and their (kind, sup, shard)
    in info[:3 nv], the keep flags of every edge (decay prune AND victim
    removal) with scanned block offsets in flag / bc, info[3 nv] = survivors,
    info[3 nv + 1] = pruned by the decay. ``rmb``: persistent zero bitmap."""
    ne = int(e["src"].numel())
    _lib.check(_lib.lib().lzk_tg_seg_end(_lib.ptr(vrows), int(nv), kind.data_ptr(), sup.data_ptr(), shard.data_ptr(),
                                         stored.data_ptr(), 1 if unstore else 0, rmb.data_ptr(), e["src"].data_ptr(),
                                         e["dst"].data_ptr(), e["meta"].data_ptr(), ne, _lib.ptr(prev),
                                         int(prev.numel()) if prev is not None else 0, _lib.ptr(flag), _lib.ptr(bc),
                                         info.data_ptr(), _st(info)), "tg_seg_end")


def build_visible_csr(e: Dict[str, torch.Tensor], shard: torch.Tensor, n: int):
    """CSR of visible arcs: a->b for an edge (a, b) or (b, a) stored in a's
    shard, ordered per source by edge index (the reference's dict order), built
    on the tensors' device. Returns (off int64 [n+1], adj int32, eid int32)."""
    dev = e["src"].device
    ne = int(e["src"].numel())
    if ne == 0:
        return (torch.zeros(n + 1, dtype=torch.int64, device=dev), torch.zeros(0, dtype=torch.int32, device=dev),
                torch.zeros(0, dtype=torch.int32, device=dev))
    s, d = e["src"].long(), e["dst"].long()
    es = e["meta"] & 0xFFFFFF
    fwd = shard[s] == es
    bwd = (shard[d] == es) & (s != d)
    frm = torch.stack([s, d], 1).reshape(-1)
    to = torch.stack([d, s], 1).reshape(-1)
    ok = torch.stack([fwd, bwd], 1).reshape(-1)
    eid = torch.arange(ne, device=dev).repeat_interleave(2)
    frm, to, eid = frm[ok], to[ok], eid[ok]
    order = torch.sort(frm, stable=True).indices
    frm, to, eid = frm[order], to[order], eid[order]
    off = torch.zeros(n + 1, dtype=torch.int64, device=dev)
    off[1:] = torch.cumsum(torch.bincount(frm, minlength=n)[:n], 0)
    return off, to.to(torch.int32), eid.to(torch.int32)


class BoostState:
    """Per-graph epoch stamps so a boost never clears an N-sized array."""

    def __init__(self):
        self.stamp: Optional[torch.Tensor] = None
        self.epoch = 0

    def next(self, n: int, dev) -> Tuple[torch.Tensor, int]:
        if self.stamp is None or self.stamp.numel() < n or self.stamp.device != torch.device(dev) \
                or self.epoch >= (1 << 30):
            self.stamp = torch.zeros(max(n, 1024) * 3 // 2, dtype=torch.int32, device=dev)
            self.epoch = 0
        self.epoch += 1
        return self.stamp, self.epoch


def neighbor_boost(csr, w, seeds: torch.Tensor, kind, sup, sal, last, dirty, now: float, state: BoostState,
                   min_w: float = 0.3, delta: float = 0.02) -> int:
    """Reference ``_boost_neighbors`` (memory_system.py:242-260): neighbours
    (visible, w >= min_w, live nodes, not seeds) of the seeds get
    last_accessed = now and salience + delta (capped at 1), once each."""
    if seeds.numel() == 0:
        return 0
    off, adj, eid = csr
    if not sal.is_cuda:
        seen = set()
        ss = set(int(x) for x in seeds.tolist())
        for s in seeds.tolist():
            if s < 0 or int(sup[s]):
                continue
            for p in range(int(off[s]), int(off[s + 1])):
                nb = int(adj[p])
                if float(w[int(eid[p])]) < min_w or nb in ss or nb in seen or int(kind[nb]) != 1:
                    continue
                seen.add(nb)
                sal[nb] = min(1.0, float(sal[nb]) + delta)
                last[nb] = now
                dirty[nb] = 1
        return len(seen)
    stamp, ep = state.next(int(sal.numel()), sal.device)
    cnt = torch.zeros(1, dtype=torch.int32, device=sal.device)
    seeds = seeds.to(torch.int32).contiguous()
    _lib.check(_lib.lib().lzk_tg_boost(off.data_ptr(), adj.data_ptr(), eid.data_ptr(), w.data_ptr(),
                                       seeds.data_ptr(), seeds.numel(), kind.data_ptr(), sup.data_ptr(), float(min_w),
                                       float(now), float(delta), sal.data_ptr(), last.data_ptr(), dirty.data_ptr(),
                                       stamp.data_ptr(), ep, cnt.data_ptr(), _st(sal)), "tg_boost")
    return int(cnt.item())


def touch(rows: torch.Tensor, acc, last, sal, dirty, now: float, delta: float = 0.05) -> None:
    """``BufferGraph.update_access`` for each row (buffer_graph.py:79-85)."""
    if rows.numel() == 0:
        return
    if not sal.is_cuda:
        for r in rows.tolist():
            acc[r] += 1
            last[r] = now
            sal[r] = min(1.0, float(sal[r]) + delta)
            dirty[r] = 1
        return
    rows = rows.to(torch.int64).contiguous()
    _lib.check(_lib.lib().lzk_tg_touch(rows.data_ptr(), rows.numel(), acc.data_ptr(), last.data_ptr(),
                                       sal.data_ptr(), dirty.data_ptr(), float(now), float(delta), _st(sal)),
               "tg_touch")


def importance(sal, acc, last, kind, sup, now: float) -> torch.Tensor:
    """Eviction score (memory_system.py:541-549) in float64; +inf for rows that
    are not evictable (not a live shard node, or a super-node)."""
    if not sal.is_cuda:
        days = (now - last) / 86400.0
        v = sal.double() * 0.5 + torch.clamp(acc.double() / 10.0, max=1.0) * 0.3 + (1.0 / (1.0 + days)) * 0.2
        bad = (kind != 1) | (sup != 0)
        return torch.where(bad, torch.full_like(v, float("inf")), v)
    out = torch.empty(sal.numel(), dtype=torch.float64, device=sal.device)
    _lib.check(_lib.lib().lzk_tg_importance(sal.data_ptr(), acc.data_ptr(), last.data_ptr(), kind.data_ptr(),
                                            sup.data_ptr(), sal.numel(), float(now), out.data_ptr(), _st(sal)),
               "tg_importance")
    return out


def evict_verify(sal, acc, last, kind, sup, shard, pool: torch.Tensor, now: float, keep: float,
                 events: Sequence[Tuple[int, float, int, int]], rowkey: Optional[torch.Tensor] = None) -> bool:
    """True when no row outside ``pool`` (uint8 mask) that nothing touched
    would have been evicted before the planned victims: ``events`` =
    (decays before the eviction, importance, shard, row) of each eviction's
    last victim, in order (core/batch_plan.py). ``rowkey`` (int64 [n]): the
    order key of each row in place of its index (a row-sharded tenant's
    global row number)."""
    if not events:
        return True
    n = int(sal.numel())
    if not sal.is_cuda:
        import numpy as np
        m = ((kind == 1) & (sup == 0) & (pool == 0)).numpy()
        idx = np.nonzero(m)[0]
        if idx.size == 0:
            return True
        s = sal.numpy()[idx].astype(np.float32)
        a = np.minimum(1.0, acc.numpy()[idx].astype(np.float64) / 10.0) * 0.3
        d = (1.0 / (1.0 + (np.float64(now) - last.numpy()[idx]) / 86400.0)) * 0.2
        code = shard.numpy()[idx].astype(np.int64)
        kf, fl = np.float32(keep), np.float32(SALIENCE_FLOOR)
        t = 0
        for st, vi, vc, vr in events:
            while t < st:
                s = np.where(s > fl, fl + (s - fl) * kf, fl).astype(np.float32)
                t += 1
            imp = s.astype(np.float64) * 0.5 + a + d
            key = idx if rowkey is None else rowkey.numpy()[idx]
            if ((imp < vi) | ((imp == vi) & ((code < vc) | ((code == vc) & (key < vr))))).any():
                return False
        return True
    dev = sal.device
    ev = list(events)
    steps = torch.tensor([e[0] for e in ev], dtype=torch.int32).to(dev)
    imp = torch.tensor([e[1] for e in ev], dtype=torch.float64).to(dev)
    code = torch.tensor([e[2] for e in ev], dtype=torch.int32).to(dev)
    row = torch.tensor([e[3] for e in ev], dtype=torch.int64).to(dev)
    bad = torch.zeros(1, dtype=torch.int32, device=dev)
    # the kernel's shortcuts: the largest event importance, the last event's
    # decay count (steps ascend), keep^that in double, the largest event key
    import numpy as np
    st_last = max(int(e[0]) for e in ev)
    vmax = max(float(e[1]) for e in ev)
    mc, mk = max((int(e[2]), int(e[3])) for e in ev)
    kt = float(np.float32(keep)) ** st_last
    _lib.check(_lib.lib().lzk_tg_evict_verify(sal.data_ptr(), acc.data_ptr(), last.data_ptr(), kind.data_ptr(),
                                              sup.data_ptr(), shard.data_ptr(), pool.data_ptr(), n, float(now),
                                              float(keep), len(ev), steps.data_ptr(), imp.data_ptr(),
                                              code.data_ptr(), row.data_ptr(), bad.data_ptr(), _st(sal),
                                              None if rowkey is None else rowkey.contiguous().data_ptr(),
                                              vmax, st_last, kt, mc, mk),
               "tg_evict_verify")
    return int(bad.item()) == 0


DIGEST_WINDOW = 1 << 16  # rows of the first selection pass (component_digest)


def component_digest(src: torch.Tensor, dst: torch.Tensor, w: torch.Tensor, kind: torch.Tensor, sup: torch.Tensor,
                     shard: torch.Tensor, n: int, min_size: int, min_avg_w: float,
                     take: int, lab: Optional[torch.Tensor] = None) -> Tuple[torch.Tensor, torch.Tensor]:
    """Device component digest (``csrc/kernels/digest.hip``): (order key,
    row) of the first ``take`` live shard-node rows of every component with
    >= ``min_size`` members and mean edge weight > ``min_avg_w``, sorted by
    (key, row). Union-find labels, then keyed reductions and selection rounds
    -- no sort over the graph (see the kernel file). One host synchronisation
    sizes the output. GPU tensors only (TenantGraph.component_digest has the
    sort-based CPU formulation); ``min_size`` >= 2, ``take`` >= 1. ``lab``:
    the components' labels when the caller has them (int32 [n], smallest row
    per component: TenantGraph's incremental labels within a batch)."""
    assert src.is_cuda and min_size >= 2 and take >= 1
    dev = src.device
    if lab is None:
        lab = components(src, dst, n)
    ne = int(src.numel())
    touched = torch.zeros(n, dtype=torch.uint8, device=dev)
    gsum = torch.zeros(n, dtype=torch.float64, device=dev)
    gi = torch.zeros((3, n), dtype=torch.int32, device=dev)  # edge count, member count, candidate count
    gfirst = torch.full((n,), 1 << 62, dtype=torch.int64, device=dev)
    cls = torch.empty(n, dtype=torch.uint8, device=dev)
    biglist = torch.empty(n // (take + 1) + 1, dtype=torch.int32, device=dev)
    counters = torch.zeros(4, dtype=torch.int32, device=dev)
    src, dst = src.to(torch.int32).contiguous(), dst.to(torch.int32).contiguous()
    w = w.to(torch.float32).contiguous()
    L_ = _lib.lib()
    _lib.check(L_.lzk_dg_stats(src.data_ptr(), dst.data_ptr(), w.data_ptr(), ne, lab.data_ptr(), n, kind.data_ptr(),
                               sup.data_ptr(), shard.data_ptr(), int(min_size), float(min_avg_w), int(take),
                               touched.data_ptr(), gsum.data_ptr(), gi[0].data_ptr(), gi[1].data_ptr(),
                               gi[2].data_ptr(), gfirst.data_ptr(), cls.data_ptr(), biglist.data_ptr(),
                               counters.data_ptr(), _st(src)), "dg_stats")
    direct, nbig = (int(v) for v in counters[:2].cpu().tolist())
    cap = direct + take * nbig
    keys = torch.empty(cap, dtype=torch.int64, device=dev)
    rows = torch.empty(cap, dtype=torch.int32, device=dev)
    if cap == 0:
        return keys, rows.long()
    if nbig:
        cur = torch.full((n,), 0x7FFFFFFF, dtype=torch.int32, device=dev)
        last = torch.full((n,), -1, dtype=torch.int32, device=dev)
        cnt = torch.zeros(n, dtype=torch.int32, device=dev)
    else:
        cur = last = cnt = torch.empty(1, dtype=torch.int32, device=dev)
    rem = torch.zeros(1, dtype=torch.int32, device=dev)
    _lib.check(L_.lzk_dg_select(lab.data_ptr(), n, touched.data_ptr(), kind.data_ptr(), sup.data_ptr(),
                                cls.data_ptr(), gfirst.data_ptr(), biglist.data_ptr(), nbig, None, int(take),
                                cur.data_ptr(), last.data_ptr(), cnt.data_ptr(), keys.data_ptr(), rows.data_ptr(),
                                cap, counters[3:].data_ptr(), rem.data_ptr(), int(DIGEST_WINDOW), _st(src)),
               "dg_select")
    m = int(counters[3].item())
    if m > cap:
        raise RuntimeError(f"component digest overflow: {m} selected rows for capacity {cap}")
    keys, rows = keys[:m], rows[:m].long()
    if m and int(keys.max()) < (1 << 62) // max(n, 1):
        o = torch.argsort(keys * n + rows)
    else:  # (key, row) by two stable sorts
        o = torch.argsort(rows, stable=True)
        o = o[torch.argsort(keys[o], stable=True)]
    return keys[o], rows[o]


def component_digest_local(src: torch.Tensor, dst: torch.Tensor, w: torch.Tensor, kind: torch.Tensor,
                           sup: torch.Tensor, shard: torch.Tensor, min_size: int, min_avg_w: float,
                           take: int) -> torch.Tensor:
    """:func:`component_digest` in O(edges) and without a host
    synchronisation, for graphs whose edges touch few of the tenant's rows
    (the consolidation buffer at the reference's prune threshold keeps a few
    thousand edges over 10M rows): the edge endpoints are renumbered 0 .. U-1
    in row order (one sort of the 2E endpoints; the index space is padded to
    2E, the padding rows FREE and untouched), the digest kernels run over that
    space -- the renumbering is monotone, so the row order and the order of
    the components' first-member keys are the tenant's -- and the result
    stays on the device, sized by the bound instead of a read-back count:
    int64 [2, 2E] = (order key, tenant row) sorted by (key, row), the unused
    tail (key 1 << 62, row -1) last. The caller copies it to the host when
    it needs the rows (:class:`TenantGraph.DigestCapture`)."""
    assert src.is_cuda and min_size >= 2 and take >= 1
    dev = src.device
    E = int(src.numel())
    nl = 2 * E
    BIG = 1 << 62
    if E == 0:
        return torch.stack([torch.full((0,), BIG, dtype=torch.int64, device=dev),
                            torch.full((0,), -1, dtype=torch.int64, device=dev)])
    ep = torch.cat([src, dst]).long()
    srt, perm = torch.sort(ep)
    newf = torch.ones(nl, dtype=torch.bool, device=dev)
    newf[1:] = srt[1:] != srt[:-1]
    uid = torch.cumsum(newf, 0, dtype=torch.int64) - 1
    local = torch.empty(nl, dtype=torch.int32, device=dev)
    local[perm] = uid.to(torch.int32)
    rowmap = torch.full((nl,), -1, dtype=torch.int64, device=dev)
    rowmap[uid] = srt
    valid = rowmap >= 0
    rc = rowmap.clamp_min(0)
    kind_l = torch.where(valid, kind[rc], torch.zeros((), dtype=kind.dtype, device=dev)).contiguous()
    sup_l, shard_l = sup[rc].contiguous(), shard[rc].contiguous()
    lsrc, ldst = local[:E].contiguous(), local[E:].contiguous()
    lab = components(lsrc, ldst, nl)
    touched = torch.zeros(nl, dtype=torch.uint8, device=dev)
    gsum = torch.zeros(nl, dtype=torch.float64, device=dev)
    gi = torch.zeros((3, nl), dtype=torch.int32, device=dev)
    gfirst = torch.full((nl,), BIG, dtype=torch.int64, device=dev)
    cls = torch.empty(nl, dtype=torch.uint8, device=dev)
    nbig_max = nl // (take + 1) + 1
    biglist = torch.empty(nbig_max, dtype=torch.int32, device=dev)
    counters = torch.zeros(4, dtype=torch.int32, device=dev)
    w = w.to(torch.float32).contiguous()
    L_ = _lib.lib()
    _lib.check(L_.lzk_dg_stats(lsrc.data_ptr(), ldst.data_ptr(), w.data_ptr(), E, lab.data_ptr(), nl,
                               kind_l.data_ptr(), sup_l.data_ptr(), shard_l.data_ptr(), int(min_size),
                               float(min_avg_w), int(take), touched.data_ptr(), gsum.data_ptr(), gi[0].data_ptr(),
                               gi[1].data_ptr(), gi[2].data_ptr(), gfirst.data_ptr(), cls.data_ptr(),
                               biglist.data_ptr(), counters.data_ptr(), _st(lsrc)), "dg_stats")
    # selection by one sort over the (small) index space instead of the
    # rounds of dg_select: candidates of qualifying components (cls 1 / 2)
    # grouped by label in row order, the first `take` of each group kept
    MAXI = torch.iinfo(torch.int64).max
    idx = torch.arange(nl, device=dev)
    labl = lab.long()
    cand = (touched != 0) & (kind_l == 1) & (sup_l == 0) & (cls[labl] != 0)  # cls is per label
    o1 = torch.sort(torch.where(cand, labl * (nl + 1) + idx, torch.full_like(idx, MAXI))).indices
    lab_s, cand_s = labl[o1], cand[o1]
    newg = torch.ones(nl, dtype=torch.bool, device=dev)
    newg[1:] = lab_s[1:] != lab_s[:-1]
    gstart = torch.cummax(torch.where(newg, idx, torch.zeros_like(idx)), 0).values
    sel = cand_s & ((idx - gstart) < take)
    key_s = gfirst[lab_s]
    # (key, row): keys are < (shard codes + 2) * nl, so key * (nl + 1) + row fits
    comb = torch.where(sel, key_s * (nl + 1) + o1, torch.full_like(o1, MAXI))
    c2, o2 = torch.sort(comb)
    ok = c2 != MAXI
    ks = torch.where(ok, key_s[o2], torch.full_like(c2, BIG))
    grow = torch.where(ok, rowmap[o1[o2]], torch.full_like(c2, -1))
    return torch.stack([ks, grow])


def num_rows(nums: torch.Tensor, add: int, base_k: torch.Tensor, base_o: torch.Tensor, delta_k: torch.Tensor,
             delta_o: torch.Tensor, holder: Optional[torch.Tensor] = None, kind: Optional[torch.Tensor] = None,
             rank: int = -1) -> torch.Tensor:
    """tenant.hip num_rows_kernel: the local row of each number ``nums + add``
    in a sorted number index (base, then delta; int64, -1 if absent); with
    ``rank`` >= 0 only rows that rank holds live (holder == rank, kind
    NODE). One launch, no host synchronisation."""
    nums = nums.to(torch.int64).contiguous()
    out = torch.empty_like(nums)
    m = int(nums.numel())
    if m == 0:
        return out
    _lib.check(_lib.lib().lzk_num_rows(nums.data_ptr(), int(add), m, base_k.data_ptr(), base_o.data_ptr(),
                                       int(base_k.numel()), delta_k.data_ptr(), delta_o.data_ptr(),
                                       int(delta_k.numel()), holder.data_ptr() if holder is not None else None,
                                       kind.data_ptr() if kind is not None else None, int(rank), out.data_ptr(),
                                       _st(nums)), "num_rows")
    return out


def row_centroid_cos(X: torch.Tensor, D: int, sqn: torch.Tensor, rows: torch.Tensor, lab: torch.Tensor,
                     C: torch.Tensor) -> torch.Tensor:
    """tenant.hip row_cent_cos_kernel: fp32 cos of each row ``X[rows[i], :D]``
    with its centroid ``C[lab[i]]`` (unit rows), -1 for rows without a vector
    (``sqn`` 0). One read of the rows; no [rows, K] product."""
    rows = rows.to(torch.int64).contiguous()
    lab = lab.to(torch.int64).contiguous()
    C = C.float().contiguous()
    out = torch.empty(rows.numel(), dtype=torch.float32, device=rows.device)
    if rows.numel() == 0:
        return out
    assert X.dtype == torch.float32 and X.stride(1) == 1 and sqn.dtype == torch.float32
    _lib.check(_lib.lib().lzk_row_cent_cos(X.data_ptr(), X.stride(0), int(D), sqn.data_ptr(), rows.data_ptr(),
                                           lab.data_ptr(), int(rows.numel()), C.data_ptr(), C.stride(0),
                                           out.data_ptr(), _st(rows)), "row_cent_cos")
    return out


def first_rows(kind: torch.Tensor, sup: torch.Tensor, shard: torch.Tensor, n: int, tgt: np.ndarray,
               out: torch.Tensor) -> None:
    """tenant.hip tg_first_rows_kernel: ``tgt`` host int32 [3, nt] (shard
    code, rows wanted, output offset) per target shard in code order, passed
    to the kernel by value; ``out`` int64 [sum wanted] receives each target's
    first live shard-node rows in row order (-1 where a target falls short)."""
    nt = int(tgt.shape[1])
    if nt == 0:
        return
    tgt = np.ascontiguousarray(tgt, dtype=np.int32)
    _lib.check(_lib.lib().lzk_tg_first_rows(kind.data_ptr(), sup.data_ptr(), shard.data_ptr(), int(n),
                                            tgt[0].ctypes.data, tgt[1].ctypes.data, tgt[2].ctypes.data, nt,
                                            out.data_ptr(), _st(out)), "tg_first_rows")


def dg_small_max_edges() -> int:
    return int(_lib.lib().lzk_dg_small_max_edges())


def component_digest_small(src: torch.Tensor, dst: torch.Tensor, w: torch.Tensor, kind: torch.Tensor,
                           sup: torch.Tensor, shard: torch.Tensor, n: int, min_size: int, min_avg_w: float,
                           take: int) -> torch.Tensor:
    """:func:`component_digest` of a graph with at most
    :func:`dg_small_max_edges` edges in ONE kernel launch (digest.hip
    dg_small_kernel: sort + renumber the endpoints, union-find, reductions
    and selection in one block), no host synchronisation: int64 [2, 2E] =
    (order key, row) sorted, unused entries (1 << 62, -1) last."""
    dev = src.device
    E = int(src.numel())
    out = torch.empty((2, 2 * E), dtype=torch.int64, device=dev)
    cnt = torch.empty(1, dtype=torch.int32, device=dev)
    ws = torch.empty(int(_lib.lib().lzk_dg_small_ws(E)), dtype=torch.uint8, device=dev)
    src, dst = src.to(torch.int32).contiguous(), dst.to(torch.int32).contiguous()
    w = w.to(torch.float32).contiguous()
    _lib.check(_lib.lib().lzk_dg_small(src.data_ptr(), dst.data_ptr(), w.data_ptr(), E, kind.data_ptr(),
                                       sup.data_ptr(), shard.data_ptr(), int(n), int(min_size), float(min_avg_w),
                                       int(take), ws.data_ptr(), out.data_ptr(), 2 * E, cnt.data_ptr(), _st(src)),
               "dg_small")
    return out


def digest_lists(kr: np.ndarray) -> List[np.ndarray]:
    """Host form of a digest: int64 [2, m] (key, row) sorted by (key, row),
    unused entries (row -1) last -> one row array per component."""
    ok = kr[1] >= 0
    key_h, rows_h = kr[0][ok], kr[1][ok]
    if rows_h.size == 0:
        return []
    return np.split(rows_h, np.nonzero(np.diff(key_h))[0] + 1)


def components(src: torch.Tensor, dst: torch.Tensor, n: int) -> torch.Tensor:
    """Undirected connected components (label = smallest row of the
    component): device hook/compress kernels (graph.hip) or host union-find."""
    from .graph_ops import connected_components
    return connected_components(src, dst, n)


def gather_fields(rows: torch.Tensor, graphs: Optional[Sequence], device_out: bool = False,
                  base: Optional[torch.Tensor] = None) -> Dict:
    """(salience, access count, kind, super flag, shard) of result rows
    [nq, k] where query q's rows belong to ``graphs[q]`` (a TenantGraph per
    query): one device gather over per-query base pointers, one host copy
    (``device_out``: the device tensors, for an asynchronous copy). ``base``:
    the int64 [5, nq] device table of those column pointers when the caller
    already has it (``routing.TenantTable``); ``graphs`` is then unused."""
    nq, k = rows.shape
    dev = rows.device
    if not rows.is_cuda:
        out = {n: np.zeros((nq, k), dt) for n, dt in (("sal", np.float32), ("acc", np.int32), ("kind", np.uint8),
                                                      ("sup", np.uint8), ("shard", np.int32))}
        out["shard"][:] = -1
        rh = rows.numpy()
        for q, g in enumerate(graphs):
            for j, r in enumerate(rh[q]):
                if r >= 0:
                    for n in out:
                        out[n][q, j] = getattr(g, n)[int(r)]
        return out
    if base is None:
        base = torch.tensor([[getattr(g, c).data_ptr() for g in graphs] for c in ("sal", "acc", "kind", "sup",
                                                                                  "shard")],
                            dtype=torch.int64).pin_memory().to(dev, non_blocking=True)
    if base.device != dev or base.dtype != torch.int64 or tuple(base.shape) != (5, nq) or not base.is_contiguous():
        raise ValueError(f"gather_fields: base must be a contiguous int64 [5, {nq}] tensor on {dev}, "
                         f"got {base.dtype} {tuple(base.shape)} on {base.device}")
    o = {"sal": torch.empty((nq, k), dtype=torch.float32, device=dev),
         "acc": torch.empty((nq, k), dtype=torch.int32, device=dev),
         "kind": torch.empty((nq, k), dtype=torch.uint8, device=dev),
         "sup": torch.empty((nq, k), dtype=torch.uint8, device=dev),
         "shard": torch.empty((nq, k), dtype=torch.int32, device=dev)}
    rows = rows.to(torch.int64).contiguous()
    _lib.check(_lib.lib().lzk_tg_gather_fields(rows.data_ptr(), nq, k, base.data_ptr(), o["sal"].data_ptr(),
                                                o["acc"].data_ptr(), o["kind"].data_ptr(), o["sup"].data_ptr(),
                                                o["shard"].data_ptr(), _st(rows)), "tg_gather_fields")
    if device_out:
        return o
    return {n: t.cpu().numpy() for n, t in o.items()}


_METRIC_CODE = {"l2": 0, "ip": 1, "dot": 1, "cosine": 2}


def store_rerank(Qf: torch.Tensor, X: torch.Tensor, sqn: torch.Tensor, bias: torch.Tensor, cand: torch.Tensor,
                 k: int, metric: str, kind: Optional[torch.Tensor] = None):
    """Exact fp32 re-rank of store-search candidates in one launch
    (tenant.hip store_rerank_kernel): scores of the rows ``cand`` [M, C]
    (C <= 64, -1 = empty) against ``Qf`` [M, D], top-k by (score desc, row
    asc). Returns (scores [M, k], rows int64 [M, k]; -inf / -1 padding);
    with ``kind`` (the graph's kind column) the rows that are not graph
    nodes come back as -1 (the search_memories view), in the same launch."""
    M, C = cand.shape
    D = Qf.shape[1]
    Qc = Qf.contiguous()
    cc = cand.contiguous()
    assert X.stride(1) == 1 and X.shape[1] == D and C <= 64 and Qc.dtype == torch.float32
    os_ = torch.empty((M, k), dtype=torch.float32, device=Qf.device)
    oi = torch.empty((M, k), dtype=torch.long, device=Qf.device)
    if M == 0:
        return os_, oi
    oin = torch.empty((M, k), dtype=torch.long, device=Qf.device) if kind is not None else None
    _lib.check(_lib.lib().lzk_store_rerank(Qc.data_ptr(), Qc.stride(0), X.data_ptr(), X.stride(0), D, sqn.data_ptr(),
                                           bias.data_ptr(), cc.data_ptr(), C, M, int(k), _METRIC_CODE[metric],
                                           os_.data_ptr(), oi.data_ptr(), _lib.ptr(kind), _lib.ptr(oin),
                                           _lib.stream_ptr(Qf.device)),
               "lzk_store_rerank")
    return (os_, oin) if kind is not None else (os_, oi)


SET_ROWS_COLS = ("sal", "acc", "last", "ts", "shard", "sup", "parent")


def set_rows(g, rows: Optional[torch.Tensor], block: torch.Tensor, present: int, kind_v: int, stored_v: int,
             m: Optional[int] = None, row0: Optional[int] = None) -> None:
    """Node columns of ``rows`` in one launch (tenant.hip tg_set_rows_kernel):
    ``block`` is a device float64 vector = 7 constants (one per
    SET_ROWS_COLS column) followed by [ncols, m] per-row values of the
    columns whose bit is set in ``present``. ``rows`` None: bit 15 of
    ``present``, the rows are the block's first m per-row values; bits 8-14
    leave columns unwritten, ``kind_v`` / ``stored_v`` < 0 leave kind /
    stored; ``row0``: the contiguous rows row0 .. row0 + m - 1 (no row
    list)."""
    m = int(rows.numel()) if rows is not None else int(m)
    if rows is None and row0 is None:
        present |= 1 << 15
    b = block.data_ptr()
    _lib.check(_lib.lib().lzk_tg_set_rows(
        _lib.ptr(rows), int(row0 or 0), m, b + 7 * 8, int(present), b, g.sal.data_ptr(), g.acc.data_ptr(), g.last.data_ptr(),
        g.ts.data_ptr(), g.shard.data_ptr(), g.sup.data_ptr(), g.parent.data_ptr(), g.kind.data_ptr(),
        g.stored.data_ptr(), g.dirty.data_ptr(), int(kind_v), int(stored_v), _lib.stream_ptr(block.device)),
        "lzk_tg_set_rows")


def write_emb(g, e32: torch.Tensor, has: Optional[torch.Tensor], rows: Optional[torch.Tensor], dv_max: torch.Tensor,
              row0: int = 0, has_emb: bool = False) -> None:
    """Embedding columns of ``rows`` from fp32 ``e32`` [m, dim] in one launch
    (tenant.hip tg_write_emb_kernel): emb32, emb16, the int8 copy + row
    scale, sqn, the per-dimension fp64 sums of squares, and device maxima of
    the row scale (``g._rs8_max``) and of | |x| - 1 | (``dv_max`` [1]).
    ``rows`` None: the contiguous rows row0 ..; ``has_emb``: the has_emb
    column too."""
    m, D = e32.shape
    x = e32.contiguous() if e32.dtype == torch.float32 else e32.float().contiguous()
    r = rows.to(torch.long).contiguous() if rows is not None else None
    h = has.to(torch.uint8).contiguous() if has is not None else None
    i8 = g.emb8 is not None and g.emb8.dtype == torch.int8
    _lib.check(_lib.lib().lzk_tg_write_emb(
        x.data_ptr(), x.stride(0), _lib.ptr(h), m, D, _lib.ptr(r), int(row0), g.emb32.data_ptr(), g.emb32.stride(0),
        _lib.ptr(g.emb16), g.emb16.stride(0) if g.emb16 is not None else 0,
        g.emb8.data_ptr() if i8 else None, g.emb8.stride(0) if i8 else 0, g.rs8.data_ptr() if i8 else None,
        g.sqn.data_ptr(), g.sumsq.data_ptr(), g._rs8_max.data_ptr() if i8 else None, dv_max.data_ptr(),
        g.has_emb.data_ptr() if has_emb else None, _lib.stream_ptr(x.device)), "lzk_tg_write_emb")
    if g.emb8 is not None and not i8:  # fp8 copy: the torch quantiser
        g._write_lowp(r, x * h[:, None].to(x.dtype) if h is not None else x)
