"""Spherical k-means on the device -- the scalable form of the reference's
super-node hierarchy (one mean super-node per shard, memory_system.py:893-933;
SURVEY.md §2.4 K16/K8) and the coarse quantiser of the IVF-PQ index.

assign: fused MFMA top-1 over the centroid matrix (``flat_topk`` with the
        centroids as the arena and the data as queries)
update: segmented mean + L2 renormalisation (``graph_ops.centroids``)
Distributed: with a :class:`~lazzaro_amd.parallel.Communicator`, per-rank partial sums/counts are combined
with one all-reduce per iteration so every rank holds the
same global centroids.
"""
from __future__ import annotations

import os
from typing import Optional, Tuple

import numpy as np
import torch

from ..ops import graph_ops as G
from ..ops.search import flat_top1, flat_topk
from ..utils.tracing import tracer


# "top1": the 256x256 argmax kernel (flat_top1); "lane": flat_topk(k=1) on the 128x128 per-lane kernel
ASSIGN = 'top1'


def assign(X: torch.Tensor, C16: torch.Tensor, chunk: int = 1 << 20) -> Tuple[torch.Tensor, torch.Tensor]:
    """Nearest (max inner product) centroid per row of X. Returns (label, score)."""
    if ASSIGN == "top1" and X.is_cuda:
        s, i = flat_top1(C16, X.contiguous() if X.stride(1) != 1 else X)
        return i, s
    labs, scs = [], []
    for r0 in range(0, X.shape[0], chunk):
        s, i = flat_topk(C16, X[r0:r0 + chunk], 1)
        labs.append(i[:, 0])
        scs.append(s[:, 0])
    return torch.cat(labs).to(torch.int32), torch.cat(scs)


# two-level assign in one grouped launch (flat_top1_grouped_kernel) instead of
# a gather + flat_top1 per topic group; GROUPED = False for the loop
GROUPED = True
GROUP_TILE = 256  # the 256x256 pipeline's tile edge (lzk_g256.h BM = BN)


def _assign_grouped(X: torch.Tensor, C16: torch.Tensor, tl: torch.Tensor, top_of: torch.Tensor,
                    t: int) -> Tuple[torch.Tensor, torch.Tensor]:
    """Rows sorted by topic (positions), fine centroids sorted by topic; one
    block per (centroid tile, query tile) of every topic group. The kernel
    reads each row straight from X by index (no gather) and returns, per
    position, the best sorted-centroid index with flat_top1's tie order."""
    import numpy as np

    from ..ops import _lib

    if X.dim() != 2 or X.stride(1) != 1:  # the kernel reads rows by index at stride ldx, unit column stride
        X = X.contiguous()
    n = X.shape[0]
    dev = X.device
    fo = torch.argsort(top_of, stable=True)
    fcnt = np.asarray(torch.bincount(top_of, minlength=t)[:t].tolist(), dtype=np.int64)
    ro = torch.argsort(tl, stable=True)
    rcnt = np.asarray(torch.bincount(tl, minlength=t)[:t].tolist(), dtype=np.int64)
    fstart = np.concatenate([[0], np.cumsum(fcnt)[:-1]])
    rstart = np.concatenate([[0], np.cumsum(rcnt)[:-1]])
    T = GROUP_TILE
    parts = []
    for c in np.nonzero((fcnt > 0) & (rcnt > 0))[0]:
        nf, nr = int(fcnt[c]), int(rcnt[c])
        rt = np.arange(0, nf, T)
        qt = np.arange(0, nr, T)
        q, r = np.meshgrid(qt, rt, indexing="ij")  # centroid tile fastest: a query tile's blocks are adjacent
        q, r = q.ravel(), r.ravel()
        parts.append(np.stack([fstart[c] + r, nf - r, rstart[c] + q, nr - q], 1))
    Cs = C16[fo].contiguous()
    qidx = ro.to(torch.int32).contiguous()
    score = torch.full((n,), float("-inf"), dtype=torch.float32, device=dev)
    pos = torch.full((n,), -1, dtype=torch.int32, device=dev)
    if parts:
        blk = np.concatenate(parts).astype(np.int32)
        # the kernel reads centroid rows [c0, c0+min(nc,T)) and qidx[p0, p0+min(np,T)):
        # checked here, not by assert (python -O must not remove a bounds check)
        if blk[:, 1].min() < 1 or blk[:, 3].min() < 1:
            raise ValueError("grouped assign: empty block in the block table")
        if int((blk[:, 0] + np.minimum(blk[:, 1], T)).max()) > Cs.shape[0]:
            raise ValueError("grouped assign: centroid range past the centroid matrix")
        if int((blk[:, 2] + np.minimum(blk[:, 3], T)).max()) > n:
            raise ValueError("grouped assign: query range past the row index")
        blocks = torch.from_numpy(blk).to(dev)
        ws = torch.empty(n, dtype=torch.int64, device=dev)
        _lib.check(_lib.lib().lzk_flat_top1_grouped(Cs.data_ptr(), Cs.stride(0), X.data_ptr(), X.stride(0),
                                                     qidx.data_ptr(), n, blocks.data_ptr(), int(blk.shape[0]),
                                                     X.shape[1], ws.data_ptr(), score.data_ptr(), pos.data_ptr(),
                                                     _lib.stream_ptr(dev)), "lzk_flat_top1_grouped")
    lab = torch.empty(n, dtype=torch.int32, device=dev)
    sc = torch.empty(n, dtype=torch.float32, device=dev)
    lab[ro] = fo[pos.long().clamp_min(0)].to(torch.int32)
    sc[ro] = score
    lone = np.nonzero((fcnt == 0) & (rcnt > 0))[0]
    if lone.size:  # rows whose topic has no fine centroid: the full search
        lone_t = torch.as_tensor(lone, device=dev)
        rr = torch.nonzero(torch.isin(tl, lone_t)).flatten()
        li, si = assign(X[rr].contiguous(), C16)
        lab[rr], sc[rr] = li.to(torch.int32), si.float()
    return lab, sc


def assign_two_level(X: torch.Tensor, C16: torch.Tensor, T16: torch.Tensor, top_of: torch.Tensor,
                     chunk: int = 1 << 22) -> Tuple[torch.Tensor, torch.Tensor]:
    """Nearest fine centroid per row, searched only under the row's nearest
    top centroid: ``T16`` [t, Dp] top centroids, ``top_of`` [k] the top
    cluster of each fine centroid (``C16`` [k, Dp]). Cost n x (t + k/t) dot
    products instead of n x k -- at 10M rows, 64 tops and 4096 fine
    centroids ~2 TFLOP instead of 63. Returns (label, score) like
    :func:`assign`; a row whose top cluster has no fine centroid falls back
    to the full search."""
    n = X.shape[0]
    dev = X.device
    tl, _ = assign(X, T16)
    tl = tl.long()
    t = T16.shape[0]
    if GROUPED and X.is_cuda and X.dtype == torch.bfloat16 and n > 0:
        return _assign_grouped(X, C16, tl, top_of.long(), t)
    fo = torch.argsort(top_of.long(), stable=True)
    fcnt = torch.bincount(top_of.long(), minlength=t).tolist()
    ro = torch.argsort(tl, stable=True)
    rcnt = torch.bincount(tl, minlength=t).tolist()
    lab = torch.empty(n, dtype=torch.int32, device=dev)
    score = torch.empty(n, dtype=torch.float32, device=dev)
    r0 = f0 = 0
    for c in range(t):
        nr, nf = rcnt[c], fcnt[c]
        rows = ro[r0:r0 + nr]
        fines = fo[f0:f0 + nf]
        r0 += nr
        f0 += nf
        if nr == 0:
            continue
        for a in range(0, nr, chunk):
            rr = rows[a:a + chunk]
            if nf == 0:
                li, si = assign(X[rr], C16)
                lab[rr], score[rr] = li.to(torch.int32), si.float()
                continue
            # the fused argmax kernel (fp32 accumulate, exact ties) on the group
            j, si = assign(X[rr].contiguous(), C16[fines].contiguous())
            lab[rr] = fines[j.long()].to(torch.int32)
            score[rr] = si.float()
    return lab, score


# farthest-first seeding as one fused kernel per pick (csrc/kernels/kmeans.hip); 0 = torch GEMV chain
FF_KERNEL = True


FF_SAMPLE = 32768


def _farthest_first(X: torch.Tensor, k: int, seed: int, max_sample: Optional[int] = None,
                    rows: Optional[torch.Tensor] = None) -> torch.Tensor:
    """Deterministic farthest-first seeding on a subsample (k-means++ without
    the sampling): avoids two seeds landing in one cluster. ``rows``: the
    eligible row indices (default all). ``max_sample`` (default
    ``FF_SAMPLE`` = 32k rows, 8 per seed at k = 4096): every pick is one pass
    over the sample, so the 4096 picks cost 4096 sample reads -- 64k rows
    took 27 us per pick (111 ms per seeding, profiles/r4/bench_kernel_summary.txt)."""
    if max_sample is None:
        max_sample = FF_SAMPLE
    with tracer.stage("ff_seed", X.device):
        return _ff(X, k, seed, max_sample, rows)


def _ff(X, k, seed, max_sample, rows):
    n = X.shape[0] if rows is None else rows.numel()
    g = torch.Generator(device="cpu").manual_seed(seed)
    m0 = min(n, max_sample)
    if n > 4 * m0:
        # a sample without a permutation of all n rows (a host randperm of
        # 10M rows took ~300 ms, most of the seeding)
        pick = np.random.default_rng(seed).choice(n, size=m0, replace=False, shuffle=True)
        sub = torch.from_numpy(pick.astype(np.int64)).to(X.device)
    else:
        sub = torch.randperm(n, generator=g)[:m0].to(X.device)
    if rows is not None:
        sub = rows[sub]
    if FF_KERNEL and X.is_cuda and X.dtype == torch.bfloat16 and X.shape[1] % 8 == 0 and X.shape[1] <= 2048 \
            and sub.numel():
        # one fused HIP kernel per pick, enqueued from C++ (csrc/kernels/kmeans.hip)
        from ..ops import _lib
        Sb = X[sub].contiguous()
        m = min(k, Sb.shape[0])
        L = _lib.lib()
        picks = torch.empty(m, dtype=torch.int32, device=X.device)
        ws = torch.empty(int(L.lzk_farthest_first_ws(Sb.shape[0], m)), dtype=torch.uint8, device=X.device)
        _lib.check(L.lzk_farthest_first(Sb.data_ptr(), Sb.stride(0), Sb.shape[0], Sb.shape[1], m, picks.data_ptr(),
                                        ws.data_ptr(), _lib.stream_ptr(X.device)), "lzk_farthest_first")
        c = Sb[picks.long()].float()
        if c.shape[0] < k:
            c = torch.cat([c, Sb[torch.randint(0, Sb.shape[0], (k - c.shape[0],), generator=g).to(X.device)].float()])
        return c
    S = X[sub].float()
    m = min(k, S.shape[0])
    picks = torch.zeros(m, dtype=torch.long, device=S.device)
    best = torch.mv(S, S[0])
    for t in range(1, m):  # picks stay on the device: no host sync per seed
        j = torch.argmin(best).view(1)
        picks[t:t + 1] = j
        best = torch.maximum(best, torch.mv(S, S.index_select(0, j)[0]))
    c = S[picks]
    if c.shape[0] < k:
        c = torch.cat([c, S[torch.randint(0, S.shape[0], (k - c.shape[0],), generator=g).to(X.device)]])
    return c


def kmeans(X: torch.Tensor, k: int, iters: int = 10, seed: int = 0, comm=None,
           init: Optional[torch.Tensor] = None, mask: Optional[torch.Tensor] = None,
           sample: int = 0, full_assign=None,
           sample_assign=None) -> Tuple[torch.Tensor, torch.Tensor, torch.Tensor]:
    """X: unit rows [n, Dp] (bf16 on GPU). Returns (centroids fp32 [k, Dp],
    centroids bf16 [k, Dp], labels int32 [n]). ``mask`` (bool [n]): rows
    that take part (others get label -1 and do not move the centroids) --
    an arena with tombstones is clustered in place, without a gather.
    ``sample`` > 0 and fewer than the participating rows: every iteration but
    the last refines the centroids on a fresh random ``sample``-row subset
    (mini-batch Lloyd steps); the last one assigns and updates over all rows,
    so every row's label is exact for the returned centroids' predecessors as
    in the full algorithm -- at 10M rows x 4096 centroids a full assign is
    63 TFLOP, a 1M-row one 6.3. ``full_assign(X, C16)``: replaces the
    assign of the full-data steps (e.g. :func:`assign_two_level`);
    ``sample_assign(Xs, C16)`` the same for the mini-batch steps."""
    n, Dp = X.shape
    dev = X.device
    if init is None and k <= 4096:
        c32 = _farthest_first(X, k, seed, rows=None if mask is None else torch.nonzero(mask).flatten())
    elif init is None:
        g = torch.Generator(device="cpu").manual_seed(seed)
        c32 = X[torch.randperm(n, generator=g)[:k].to(dev)].float()
    distributed = comm is not None and comm.world > 1
    if init is None:
        if distributed:
            comm.broadcast(c32, src=0)
    else:
        c32 = init.float().to(dev)
    c32 = c32 / c32.norm(dim=1, keepdim=True).clamp_min(1e-30)
    c16 = c32.to(X.dtype)
    lab = None
    rows_all = torch.nonzero(mask).flatten() if (sample and mask is not None) else None
    n_part = int(rows_all.numel()) if rows_all is not None else n
    for it in range(iters):
        if sample and n_part > sample and it < iters - 1:
            # uniform draws on the device (a host randperm of 10M rows costs
            # more than the sampled assign saves); repeats are harmless here
            g = torch.Generator(device=dev).manual_seed(seed * 7919 + it + 1)
            pick = torch.randint(0, n_part, (sample,), device=dev, generator=g)
            Xs = X[rows_all[pick] if rows_all is not None else pick]
            ls, _ = (sample_assign or assign)(Xs, c16)
            c32n, c16n, cnt = G.centroids(Xs, ls, k, normalize=not distributed, pad_to=Dp if X.is_cuda else 0)
            if distributed:
                sums = c32n * cnt.clamp_min(1)[:, None].float()
                comm.all_reduce(sums)
                comm.all_reduce(cnt)
                c32n = sums / cnt.clamp_min(1)[:, None].float()
                c32n = c32n / c32n.norm(dim=1, keepdim=True).clamp_min(1e-30)
                c16n = None
            empty = cnt == 0
            c32 = torch.where(empty[:, None], c32, c32n)
            c16 = c32.to(X.dtype) if c16n is None else torch.where(empty[:, None], c16, c16n)
            continue
        lab, _ = (full_assign or assign)(X, c16)
        if mask is not None:
            lab = torch.where(mask, lab, torch.full_like(lab, -1))
        if not distributed:
            c32, c16n, cnt = G.centroids(X, lab, k, normalize=True, pad_to=Dp if X.is_cuda else 0)
        else:
            c32u, _, cnt = G.centroids(X, lab, k, normalize=False)
            sums = c32u * cnt.clamp_min(1)[:, None].float()
            comm.all_reduce(sums)
            comm.all_reduce(cnt)
            c32 = sums / cnt.clamp_min(1)[:, None].float()
            c32 = c32 / c32.norm(dim=1, keepdim=True).clamp_min(1e-30)
            c16n = None
        # empty clusters keep their previous centroid
        empty = cnt == 0
        if bool(empty.any()):
            c32[empty] = c16[empty].float()
        c16 = c32.to(X.dtype) if c16n is None else torch.where(empty[:, None], c16, c16n)
    return c32, c16, lab
