"""Graph-maintenance ops: device kernels in
``csrc/kernels/graph.hip`` for HIP tensors, torch references for CPU tensors.

All functions take/return torch tensors in the DeviceGraph SoA layout:
nodes ``sal f32, acc i32, last f64, alive u8``; edges ``src/dst i32, w f32,
co i32, lu f64``.
"""
from __future__ import annotations

from typing import Dict, Optional, Tuple

import torch

from . import _lib

P, I, L, F = _lib.P, _lib.I, _lib.L, _lib.F
import ctypes as _C  # noqa: E402

D_ = _C.c_double
_lib.register("lzk_decay_flag", I, [P, P, P, L, P, F, F, P, P, P, L, F, P])
_lib.register("lzk_flag_alive", I, [P, P, L, P, P, P, P])
_lib.register("lzk_scan_blocks", I, [P, I, P, P])
_lib.register("lzk_compact_edges", I, [P, P, L, P, P, P, P, P, P, P, P, P, P, P])
_lib.register("lzk_importance", I, [P, P, P, P, P, L, D_, P, P])
_lib.register("lzk_mark_dead", I, [P, L, P, P])
_lib.register("lzk_cc_hook", I, [P, P, L, P, F, P, P, P])
_lib.register("lzk_cc_compress", I, [P, L, P])
_lib.register("lzk_uf_union", I, [P, P, L, P, F, P, P])
_lib.register("lzk_neighbor_boost", I, [P, P, P, P, P, I, F, D_, F, P, P, P, P, P])
_lib.register("lzk_pairs_above", I, [P, L, I, I, F, P, I, P, P])
_lib.register("lzk_seg_sum", I, [P, L, L, I, P, P, P, P])
_lib.register("lzk_centroids", I, [P, P, I, I, I, P, P, I, P])
_lib.register("lzk_seg_sum_sorted", I, [P, L, I, P, P, I, P, P, P])

SALIENCE_FLOOR = 0.2


def _st(t):
    return _lib.stream_ptr(t.device)


def _compact(edges: Dict[str, torch.Tensor], flag, block_cnt, ne: int) -> Dict[str, torch.Tensor]:
    L_ = _lib.lib()
    dev = edges["src"].device
    total = torch.zeros(1, dtype=torch.int32, device=dev)
    _lib.check(L_.lzk_scan_blocks(block_cnt.data_ptr(), block_cnt.numel(), total.data_ptr(), _st(block_cnt)),
               "scan")
    n_out = int(total.item())
    out = {k: torch.empty(n_out, dtype=v.dtype, device=dev) for k, v in edges.items()}
    if n_out:
        _lib.check(L_.lzk_compact_edges(flag.data_ptr(), block_cnt.data_ptr(), ne, edges["src"].data_ptr(),
                                        edges["dst"].data_ptr(), edges["w"].data_ptr(),
                                        _lib.ptr(edges.get("co")), _lib.ptr(edges.get("lu")),
                                        out["src"].data_ptr(), out["dst"].data_ptr(), out["w"].data_ptr(),
                                        _lib.ptr(out.get("co")), _lib.ptr(out.get("lu")), _st(flag)), "compact")
    return out


def decay_prune(edges: Dict[str, torch.Tensor], sal: Optional[torch.Tensor], alive: Optional[torch.Tensor],
                rate: float, threshold: float) -> Tuple[Dict[str, torch.Tensor], int]:
    """K10: w *= 1-rate; salience floor-decay; drop edges with w < threshold or
    a dead endpoint. Returns (compacted edges, n_pruned). Edge order kept."""
    ne = edges["src"].numel()
    keep = 1.0 - rate
    if not edges["src"].is_cuda:
        edges["w"].mul_(keep)
        if sal is not None:
            sal.copy_(torch.where(sal > SALIENCE_FLOOR, SALIENCE_FLOOR + (sal - SALIENCE_FLOOR) * keep,
                                  torch.full_like(sal, SALIENCE_FLOOR)))
        m = edges["w"] >= threshold
        if alive is not None and ne:
            m &= alive[edges["src"].long()].bool() & alive[edges["dst"].long()].bool()
        return {k: v[m] for k, v in edges.items()}, int(ne - int(m.sum()))
    dev = edges["src"].device
    nb = max(1, (ne + 255) // 256)
    flag = torch.empty(max(ne, 1), dtype=torch.uint8, device=dev)
    bc = torch.empty(nb, dtype=torch.int32, device=dev)
    _lib.check(_lib.lib().lzk_decay_flag(edges["w"].data_ptr(), edges["src"].data_ptr(), edges["dst"].data_ptr(),
                                         ne, _lib.ptr(alive), float(rate), float(threshold), flag.data_ptr(),
                                         bc.data_ptr(), _lib.ptr(sal), sal.numel() if sal is not None else 0,
                                         SALIENCE_FLOOR, _st(flag)), "decay_flag")
    out = _compact(edges, flag, bc, ne)
    return out, ne - out["src"].numel()


def drop_dead_edges(edges: Dict[str, torch.Tensor], alive: torch.Tensor) -> Dict[str, torch.Tensor]:
    ne = edges["src"].numel()
    if not edges["src"].is_cuda:
        m = alive[edges["src"].long()].bool() & alive[edges["dst"].long()].bool() if ne else torch.zeros(0, dtype=torch.bool)
        return {k: v[m] for k, v in edges.items()}
    dev = edges["src"].device
    nb = max(1, (ne + 255) // 256)
    flag = torch.empty(max(ne, 1), dtype=torch.uint8, device=dev)
    bc = torch.empty(nb, dtype=torch.int32, device=dev)
    _lib.check(_lib.lib().lzk_flag_alive(edges["src"].data_ptr(), edges["dst"].data_ptr(), ne, alive.data_ptr(),
                                         flag.data_ptr(), bc.data_ptr(), _st(flag)), "flag_alive")
    return _compact(edges, flag, bc, ne)


def importance(sal, acc, last, alive, protect, now: float) -> torch.Tensor:
    """K11 score (lower = evicted first); dead/protected -> +inf."""
    if not sal.is_cuda:
        days = (now - last.double()) / 86400.0
        v = 0.5 * sal.double() + 0.3 * torch.clamp(acc.double() / 10.0, max=1.0) + 0.2 / (1.0 + days)
        v = v.float()
        bad = torch.zeros_like(v, dtype=torch.bool)
        if alive is not None:
            bad |= ~alive.bool()
        if protect is not None:
            bad |= protect.bool()
        return torch.where(bad, torch.full_like(v, float("inf")), v)
    out = torch.empty_like(sal)
    _lib.check(_lib.lib().lzk_importance(sal.data_ptr(), acc.data_ptr(), last.data_ptr(), _lib.ptr(alive),
                                         _lib.ptr(protect), sal.numel(), float(now), out.data_ptr(), _st(sal)),
               "importance")
    return out


def select_lowest(score: torch.Tensor, k: int) -> torch.Tensor:
    """Indices of the k lowest scores (ties -> lower index), excluding +inf."""
    if k <= 0:
        return torch.zeros(0, dtype=torch.long, device=score.device)
    o = torch.argsort(score, stable=True)[:k]
    return o[torch.isfinite(score[o])]


def mark_dead(alive: torch.Tensor, idx: torch.Tensor) -> None:
    if idx.numel() == 0:
        return
    if not alive.is_cuda:
        alive[idx] = 0
        return
    idx = idx.to(torch.long).contiguous()
    _lib.check(_lib.lib().lzk_mark_dead(idx.data_ptr(), idx.numel(), alive.data_ptr(), _st(alive)), "mark_dead")


def connected_components(src: torch.Tensor, dst: torch.Tensor, n: int, w: Optional[torch.Tensor] = None,
                         min_w: float = 0.0, max_iter: int = 64, method: str = "uf") -> torch.Tensor:
    """K9: undirected components; label = smallest node index in the component.

    GPU ``method="uf"`` (default): one lock-free union-find pass over the
    edges (``uf_union_kernel``) + one compress pass -- two launches, no host
    synchronisation. ``method="hook"``: the iterative min-label hooking +
    pointer jumping, one host-checked round trip per iteration."""
    if not src.is_cuda:
        from ..store.colstore import _rt
        s, d = src, dst
        if w is not None:
            m = w >= min_w
            s, d = s[m], d[m]
        lab = _rt().union_find_components(s.numpy().astype("int32"), d.numpy().astype("int32"), n)
        return torch.from_numpy(lab)
    parent = torch.arange(n, dtype=torch.int32, device=src.device)
    L_ = _lib.lib()
    if method == "uf":
        src, dst = src.to(torch.int32).contiguous(), dst.to(torch.int32).contiguous()
        _lib.check(L_.lzk_uf_union(src.data_ptr(), dst.data_ptr(), src.numel(), _lib.ptr(w), float(min_w),
                                   parent.data_ptr(), _st(src)), "uf_union")
        _lib.check(L_.lzk_cc_compress(parent.data_ptr(), n, _st(src)), "cc_compress")
        return parent
    changed = torch.zeros(1, dtype=torch.int32, device=src.device)
    for _ in range(max_iter):
        changed.zero_()
        _lib.check(L_.lzk_cc_hook(src.data_ptr(), dst.data_ptr(), src.numel(), _lib.ptr(w), float(min_w),
                                  parent.data_ptr(), changed.data_ptr(), _st(src)), "cc_hook")
        _lib.check(L_.lzk_cc_compress(parent.data_ptr(), n, _st(src)), "cc_compress")
        if int(changed.item()) == 0:
            break
    return parent


def neighbor_boost(off, adj, eid, w, seeds: torch.Tensor, sal, last, now: float, min_w: float = 0.3,
                   delta: float = 0.02) -> int:
    """K12 over an undirected CSR (off int64 [n+1], adj/eid int32)."""
    if seeds.numel() == 0:
        return 0
    if not sal.is_cuda:
        seen = set()
        ss = set(seeds.tolist())
        for s in seeds.tolist():
            for p in range(int(off[s]), int(off[s + 1])):
                nb = int(adj[p])
                if float(w[int(eid[p])]) < min_w or nb in ss or nb in seen:
                    continue
                seen.add(nb)
                sal[nb] = min(1.0, float(sal[nb]) + delta)
                last[nb] = now
        return len(seen)
    flag = torch.zeros(sal.numel(), dtype=torch.int32, device=sal.device)
    nb = torch.zeros(1, dtype=torch.int32, device=sal.device)
    seeds = seeds.to(torch.int32).contiguous()
    _lib.check(_lib.lib().lzk_neighbor_boost(off.data_ptr(), adj.data_ptr(), eid.data_ptr(), w.data_ptr(),
                                             seeds.data_ptr(), seeds.numel(), float(min_w), float(now), float(delta),
                                             sal.data_ptr(), last.data_ptr(), flag.data_ptr(), nb.data_ptr(),
                                             _st(sal)), "neighbor_boost")
    return int(nb.item())


def pairs_above(X: torch.Tensor, tau: float, max_pairs: int = 1 << 22) -> torch.Tensor:
    """K7: all (i<j) with <x_i,x_j> > tau, sorted by (i, j). X bf16 [n, D%64==0] on GPU."""
    n = X.shape[0]
    if not X.is_cuda:
        S = X.float() @ X.float().T
        iu = torch.triu_indices(n, n, 1)
        m = S[iu[0], iu[1]] > tau
        return torch.stack([iu[0][m], iu[1][m]], 1).to(torch.int32)
    cnt = torch.zeros(1, dtype=torch.int32, device=X.device)
    out = torch.empty((max_pairs, 2), dtype=torch.int32, device=X.device)
    _lib.check(_lib.lib().lzk_pairs_above(X.data_ptr(), X.stride(0), n, X.shape[1], float(tau), cnt.data_ptr(),
                                          max_pairs, out.data_ptr(), _st(X)), "pairs_above")
    k = min(int(cnt.item()), max_pairs)
    p = out[:k].long()
    o = torch.argsort(p[:, 0] * n + p[:, 1])
    return p[o].to(torch.int32)


SEG_SUM_ATOMIC = False  # True: per-element fp32 atomics (the original K8 kernel) instead of sort + segment


def _seg_sum_sorted(X: torch.Tensor, label: torch.Tensor, C: int):
    """Per-cluster row sums without atomics: stable sort of the labels (rows
    with label < 0 go to a sentinel segment past the last cluster), then one
    workgroup per cluster streams its rows (lzk_seg_sum_sorted)."""
    n, D = X.shape
    key = torch.where(label >= 0, label, torch.full_like(label, C))
    # the radix sort's passes scale with the key width: 16-bit keys (C < 32767,
    # e.g. 4096 k-means clusters) take half the passes of int32 ones; a
    # stable sort of equal key values gives the same order either way
    order = torch.argsort(key.to(torch.int16) if C < 32767 else key, stable=True).contiguous()
    off = torch.zeros(C + 2, dtype=torch.int64, device=X.device)
    off[1:] = torch.cumsum(torch.bincount(key.long(), minlength=C + 1)[: C + 1], 0)
    sums = torch.empty((C, D), dtype=torch.float32, device=X.device)
    cnt = torch.empty(C, dtype=torch.int32, device=X.device)
    _lib.check(_lib.lib().lzk_seg_sum_sorted(X.data_ptr(), X.stride(0), D, order.data_ptr(), off.data_ptr(), C,
                                             sums.data_ptr(), cnt.data_ptr(), _st(X)), "seg_sum_sorted")
    return sums, cnt


def centroids(X: torch.Tensor, label: torch.Tensor, C: int, normalize: bool = True, pad_to: int = 0):
    """K8: per-cluster mean of rows (optionally L2-normalised). Returns
    (fp32 [C, D], bf16 [C, pad_to] or None, counts [C])."""
    n, D = X.shape
    if not X.is_cuda:
        sums = torch.zeros((C, D), dtype=torch.float32)
        cnt = torch.zeros(C, dtype=torch.int32)
        m = label >= 0
        sums.index_add_(0, label[m].long(), X[m].float())
        cnt.index_add_(0, label[m].long(), torch.ones(int(m.sum()), dtype=torch.int32))
        c32 = sums / cnt.clamp_min(1)[:, None].float()
        if normalize:
            c32 = c32 / c32.norm(dim=1, keepdim=True).clamp_min(1e-30)
        c16 = None
        if pad_to:
            c16 = torch.zeros((C, pad_to), dtype=torch.bfloat16)
            c16[:, :D] = c32.to(torch.bfloat16)
        return c32, c16, cnt
    if X.dtype != torch.bfloat16 or X.stride(1) != 1 or label.numel() != n:
        raise ValueError("centroids: GPU rows must be a bf16 [n, D] view with unit column stride and n labels")
    label = label.to(torch.int32).contiguous()
    if D <= 2048 and not SEG_SUM_ATOMIC:
        sums, cnt = _seg_sum_sorted(X, label, C)
    else:
        sums = torch.zeros((C, D), dtype=torch.float32, device=X.device)
        cnt = torch.zeros(C, dtype=torch.int32, device=X.device)
        _lib.check(_lib.lib().lzk_seg_sum(X.data_ptr(), X.stride(0), n, D, label.data_ptr(), sums.data_ptr(),
                                          cnt.data_ptr(), _st(X)), "seg_sum")
    c32 = torch.empty((C, D), dtype=torch.float32, device=X.device)
    c16 = torch.empty((C, pad_to), dtype=torch.bfloat16, device=X.device) if pad_to else None
    _lib.check(_lib.lib().lzk_centroids(sums.data_ptr(), cnt.data_ptr(), C, D, int(normalize), c32.data_ptr(),
                                        _lib.ptr(c16), pad_to, _st(X)), "centroids")
    return c32, c16, cnt
