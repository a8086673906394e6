"""Whole-graph ops: device kernels in
``csrc/kernels/graph.hip`` for HIP tensors, torch references for CPU tensors.
Connected components over COO edges (``src/dst`` int32, optional weight
filter), the all-pairs threshold join of the pairwise merge, and segmented
sums / centroids for the k-means hierarchy. The per-edge / per-node
maintenance of a tenant (decay + prune, eviction, boost, touch) is
``ops.tenant_ops`` on the TenantGraph columns.
"""
from __future__ import annotations

import os

from typing import Dict, Optional, Tuple

import torch

from . import _lib

P, I, L, F = _lib.P, _lib.I, _lib.L, _lib.F
_lib.register("lzk_cc_hook", I, [P, P, L, P, F, P, P, P])
_lib.register("lzk_cc_compress", I, [P, L, P])
_lib.register("lzk_uf_union", I, [P, P, L, P, F, P, P])
_lib.register("lzk_uf_union_plain", I, [P, P, L, P, F, P, P])
# Union-find pass switches: cached parent loads (default; UF_PLAIN = False =
# agent-scope atomic loads, 2.8 -> 2.05 ms on 10M rows / 20M edges,
# profiles/r4/uf_plain_loads.txt), and the number of union stages (0 = by
# edge count).
UF_PLAIN = True
UF_STAGES = 0
_lib.register("lzk_uf_union_sel", I, [P, P, L, P, F, P, I, I, P, P])
_lib.register("lzk_pairs_above", I, [P, L, I, I, F, P, I, P, P])
_lib.register("lzk_seg_sum", I, [P, L, L, I, P, P, P, P])
_lib.register("lzk_centroids", I, [P, P, I, I, I, P, P, I, P])
_lib.register("lzk_seg_sum_sorted", I, [P, L, I, P, P, I, P, P, P])


def _st(t):
    return _lib.stream_ptr(t.device)


def connected_components(src: torch.Tensor, dst: torch.Tensor, n: int, w: Optional[torch.Tensor] = None,
                         min_w: float = 0.0, max_iter: int = 64, method: str = "uf") -> torch.Tensor:
    """K9: undirected components; label = smallest node index in the component.

    GPU ``method="uf"`` (default): lock-free union-find passes over edge
    chunks (``uf_union_kernel``), each followed by a compress pass -- no host
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
        if w is not None:
            w = w.to(torch.float32).contiguous()
        ne = int(src.numel())
        # Staged: the union pass over >= 2M-edge chunks, each followed by a
        # compress pass, so later chunks find flat trees (1-2 hops) instead of
        # the long chains a single pass can leave behind. At most 4 stages:
        # on the 20M-edge persistent consolidation graph 4 stages run 894-904
        # turns/s against 742-747 with 8 and 815 with 3
        # (profiles/r4/uf_stages_ab.txt).
        stages = UF_STAGES or max(1, min(4, ne // (2 << 20)))
        step = -(-ne // stages) if ne else 1
        st = _st(src)
        for c0 in range(0, max(ne, 1), step):
            c1 = min(ne, c0 + step)
            _lib.check((L_.lzk_uf_union_plain if UF_PLAIN else L_.lzk_uf_union)(src[c0:].data_ptr(), dst[c0:].data_ptr(), c1 - c0,
                                       w[c0:].data_ptr() if w is not None else None, float(min_w),
                                       parent.data_ptr(), st), "uf_union")
            _lib.check(L_.lzk_cc_compress(parent.data_ptr(), n, st), "cc_compress")
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


def components_sel(src: torch.Tensor, dst: torch.Tensor, n: int, w: Optional[torch.Tensor], wthr: float,
                   vmark: torch.Tensor, n0: int, sel: int, parent: Optional[torch.Tensor] = None) -> torch.Tensor:
    """Union-find labels over one side of an edge selection (graph.hip
    uf_union_sel_kernel): an edge is volatile when an endpoint is a row >= n0
    or marked in ``vmark`` (uint8 [n0]), or its weight is below ``wthr``.
    ``sel`` 0: the stable edges, from singletons (``parent`` None) -- a
    batch's base labels; 1: the volatile edges on top of ``parent`` (int32
    [n], a compressed labelling of the base, extended by singletons).
    Returns the compressed labels (smallest row per component), GPU only."""
    assert src.is_cuda and vmark.dtype == torch.uint8 and vmark.numel() >= n0
    if parent is None:
        parent = torch.arange(n, dtype=torch.int32, device=src.device)
    src, dst = src.to(torch.int32).contiguous(), dst.to(torch.int32).contiguous()
    if w is not None:
        w = w.to(torch.float32).contiguous()
    ne = int(src.numel())
    L_ = _lib.lib()
    st = _st(src)
    # the stable side holds nearly every edge: staged like connected_components;
    # the volatile side is a few thousand edges found by one filtering pass
    stages = 1 if sel else (UF_STAGES or max(1, min(4, ne // (2 << 20))))
    step = -(-ne // stages) if ne else 1
    for c0 in range(0, max(ne, 1), step):
        c1 = min(ne, c0 + step)
        _lib.check(L_.lzk_uf_union_sel(src[c0:].data_ptr(), dst[c0:].data_ptr(), c1 - c0,
                                       w[c0:].data_ptr() if w is not None else None, float(wthr), vmark.data_ptr(),
                                       int(n0), int(sel), parent.data_ptr(), st), "uf_union_sel")
        _lib.check(L_.lzk_cc_compress(parent.data_ptr(), n, st), "cc_compress")
    return parent


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
