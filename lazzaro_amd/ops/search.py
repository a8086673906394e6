"""Similarity top-k over a vector arena.

``flat_topk`` is the single entry point used by the store's vector search
(reference ``vector_store.py:132-140``), super-node scoring
(``memory_system.py:464-472``), consolidation dedupe (``:719-733``) and
associative linking (``:797-889``).

Scores are ``alpha * <q, x> + bias[row]`` (fp32 accumulate over bf16 operands),
which expresses all three metrics of the framework:

* ``ip``      alpha=1, no bias
* ``cosine``  rows and queries pre-normalised, alpha=1
* ``l2``      alpha=2, bias=-|x|^2  (monotone in -|q-x|^2; LanceDB's default)

Dead rows (tombstones) carry ``bias=-inf``; ``row_label``/``q_label`` restrict
a query to rows with an equal label (tenant / shard filter; label<0 = any).
Results are ordered by (score desc, row asc); missing slots are (-inf, -1).
"""
from __future__ import annotations

import os

import numpy as np
import torch

from . import _lib

TARGET_WGS = 512  # 2 resident 256-thread workgroups per CU on 256 CUs


def _ref_topk(X, Q, k, bias=None, row_label=None, q_label=None, alpha=1.0, idx_offset=0,
              chunk=1 << 16):
    """fp32 torch reference with the same (score desc, index asc) order."""
    nq = Q.shape[0]
    n = X.shape[0]
    dev = X.device
    best_s = torch.full((nq, 0), float("-inf"), device=dev)
    best_i = torch.zeros((nq, 0), dtype=torch.long, device=dev)
    Qf = Q.float()
    for c0 in range(0, n, chunk):
        c1 = min(n, c0 + chunk)
        s = alpha * (Qf @ X[c0:c1].float().T)
        if bias is not None:
            s = s + bias[c0:c1].float()[None, :]
        if row_label is not None and q_label is not None:
            ok = (row_label[c0:c1][None, :] == q_label[:, None]) | (q_label[:, None] < 0)
            s = s.masked_fill(~ok, float("-inf"))
        idx = torch.arange(c0, c1, device=dev).expand(nq, -1)
        cs = torch.cat([best_s, s], 1)
        ci = torch.cat([best_i, idx], 1)
        # stable sort on index first, then on score -> ties keep ascending index
        o = torch.argsort(ci, dim=1, stable=True)
        cs = torch.gather(cs, 1, o)
        ci = torch.gather(ci, 1, o)
        o = torch.argsort(-cs, dim=1, stable=True)[:, :k]
        best_s = torch.gather(cs, 1, o)
        best_i = torch.gather(ci, 1, o)
    if best_s.shape[1] < k:
        pad = k - best_s.shape[1]
        best_s = torch.cat([best_s, torch.full((nq, pad), float("-inf"), device=dev)], 1)
        best_i = torch.cat([best_i, torch.full((nq, pad), -1, dtype=torch.long, device=dev)], 1)
    best_i = torch.where(torch.isinf(best_s) & (best_s < 0), torch.full_like(best_i, -1),
                         best_i + idx_offset)
    return best_s, best_i


class _Workspace:
    """Scratch for partial / candidate lists (grown, never shrunk), one buffer
    per (device, stream): kernels on one stream reuse it in stream order, and
    two streams searching at once (e.g. background consolidation on its side
    stream beside retrieval on the main stream) never share one."""

    def __init__(self):
        self.buf = {}

    def get(self, dev, nbytes):
        dev = torch.device(dev)
        key = (dev, torch.cuda.current_stream(dev).cuda_stream) if dev.type == "cuda" else (dev, 0)
        b = self.buf.get(key)
        if b is None or b.numel() < nbytes:
            b = torch.empty(max(nbytes, 1 << 20), dtype=torch.uint8, device=dev)
            self.buf[key] = b
        return b


_ws = _Workspace()
_ws_cand = _Workspace()
_ws_cand2 = _Workspace()
_ws_fallback = _Workspace()
_ws_blk = _Workspace()


def _blk_records(dev, grid: int, nq: int, kslot: int, S: int, lists: int):
    """Block-private candidate records of one persistent pass (search256.hip
    BlkCands): int4 [grid, cap] + int32 counts [grid]; cap ~8x the expected
    records per block (a block that overflows marks its queries for the
    exact fallback)."""
    cap = max(8192, 8 * lists * nq * kslot * S // max(grid, 1))
    ws = _ws_blk.get(dev, grid * cap * 16 + grid * 4)
    buf = ws[: grid * cap * 16]
    cnt = ws[grid * cap * 16: grid * cap * 16 + grid * 4].view(torch.int32)
    return buf, cap, cnt

# Large-batch candidate path (csrc/kernels/search256.hip): used when the batch
# fills whole 256-query tiles and the arena is large enough that the strided
# threshold sample is cheap (SEARCH_MODE "lane" / "cand" force one path: tests).
CAND_MIN_ROWS = 1 << 20
CAND_MIN_Q = 256
CAND_STRIDE = 64
# narrow int8 store searches: the sample stride of the threshold. 1/256
# halves the sample pass (~45 us of a single-query search) but its threshold
# sits ~4x more rows down, and the longer lists cost more in the gather and
# the two selects than the pass saved (+27 us; tools/narrow_margins.py: the
# worst-case margin, 0.055 at d = 768, keeps 2-5k rows per query at 1/64 and
# 7-16k at 1/256)
CAND_STRIDE_NARROW = 64


SEARCH_MODE = "auto"


def _use_cand(N, nq, kslot):
    mode = SEARCH_MODE
    if mode == "lane":
        return False
    if mode == "cand":
        return True
    return N >= CAND_MIN_ROWS and nq >= CAND_MIN_Q and kslot <= 16


def flat_topk(X: torch.Tensor, Q: torch.Tensor, k: int, *, bias=None, row_label=None,
              q_label=None, alpha: float = 1.0, idx_offset: int = 0, n_chunks: int = None):
    """Exact top-k of ``alpha*Q@X.T + bias`` per query row.

    X: [N, D] bf16 (row stride may exceed D), Q: [nq, D] bf16, D % 64 == 0 on GPU.
    Returns (scores fp32 [nq, k], rows int64 [nq, k]) with rows offset by idx_offset.
    """
    if Q.dim() == 1:
        Q = Q[None, :]
    nq, D = Q.shape
    N = X.shape[0]
    if not X.is_cuda:
        return _ref_topk(X, Q, k, bias, row_label, q_label, alpha, idx_offset)
    L = _lib.lib()
    kslot = L.lzk_flat_topk_kslot(int(k))
    if kslot < 0:
        raise ValueError(f"flat_topk supports k <= 16 per pass (got {k}); use search.topk_large")
    assert X.dtype == torch.bfloat16 and Q.dtype == torch.bfloat16
    assert X.shape[1] == D and D % 64 == 0, "D must be a multiple of 64 (pad the arena)"
    assert X.stride(1) == 1 and Q.stride(1) == 1
    if N == 0 or nq == 0:
        dev = X.device
        return (torch.full((nq, k), float("-inf"), device=dev),
                torch.full((nq, k), -1, dtype=torch.long, device=dev))
    if bias is not None:
        assert bias.dtype == torch.float32 and bias.is_contiguous() and bias.shape[0] >= N
    if row_label is not None:
        assert row_label.dtype == torch.int32 and q_label is not None
        assert q_label.dtype == torch.int32 and q_label.shape[0] == nq
    if n_chunks is None and _use_cand(N, nq, kslot):
        return _flat_topk_cand(X, Q, k, kslot, bias, row_label, q_label, alpha, idx_offset)
    return _flat_topk_lane(X, Q, k, kslot, bias, row_label, q_label, alpha, idx_offset, n_chunks)


def flat_top1(X: torch.Tensor, Q: torch.Tensor):
    """Exact argmax of ``Q @ X.T`` per query: (score fp32 [nq], row int32 [nq]).

    The k-means assign shape (millions of queries, a few thousand rows) on the
    256x256 MFMA pipeline with a packed 64-bit atomicMax merge across row
    tiles (search256.hip flat_top1_kernel); ties go to the smaller row.
    """
    nq, D = Q.shape
    N = X.shape[0]
    if not X.is_cuda:
        s, i = _ref_topk(X, Q, 1, None, None, None, 1.0, 0)
        return s[:, 0], i[:, 0].to(torch.int32)
    assert X.dtype == torch.bfloat16 and Q.dtype == torch.bfloat16
    assert X.shape[1] == D and D % 64 == 0 and X.stride(1) == 1 and Q.stride(1) == 1
    dev = X.device
    if N == 0 or nq == 0:
        return torch.full((nq,), float("-inf"), device=dev), torch.full((nq,), -1, dtype=torch.int32, device=dev)
    ws = torch.empty(nq, dtype=torch.int64, device=dev)
    score = torch.empty(nq, dtype=torch.float32, device=dev)
    row = torch.empty(nq, dtype=torch.int32, device=dev)
    _lib.check(_lib.lib().lzk_flat_top1(X.data_ptr(), X.stride(0), N, Q.data_ptr(), Q.stride(0), nq, D, ws.data_ptr(),
                                        score.data_ptr(), row.data_ptr(), _lib.stream_ptr(dev)), "lzk_flat_top1")
    return score, row


def _flat_topk_lane(X, Q, k, kslot, bias, row_label, q_label, alpha, idx_offset, n_chunks):
    """Per-lane running top-K kernel (search.hip) + partial-list merge."""
    L = _lib.lib()
    nq, D = Q.shape
    N = X.shape[0]
    if n_chunks:
        # same normalisation as the C launcher: chunks are whole 128-row tiles
        rpc = -(-(-(-N // n_chunks)) // 128) * 128
        nch = -(-N // rpc)
    else:
        nch = L.lzk_flat_topk_chunks(N, nq, TARGET_WGS)
    dev = X.device
    part = nq * nch * kslot
    ws = _ws.get(dev, part * 8)
    ps = ws[: part * 4].view(torch.float32)
    pi = ws[part * 4: part * 8].view(torch.int32)
    st = _lib.stream_ptr(dev)
    rc = L.lzk_flat_topk_partial(X.data_ptr(), X.stride(0), N, Q.data_ptr(), Q.stride(0), nq,
                                 _lib.ptr(bias), _lib.ptr(row_label), _lib.ptr(q_label),
                                 float(alpha), D, kslot, nch, ps.data_ptr(), pi.data_ptr(), st)
    _lib.check(rc, "lzk_flat_topk_partial")
    ncand = nch * kslot
    G = _merge_groups(nq, nch)
    if G > 1:
        # few queries, many partial lists (the 1/S sample of a narrow batch:
        # 512 chunks x 16 = 8192 candidates on ONE wave took 163 us): merge
        # G groups per query on G waves, then their G x kslot survivors
        os1 = torch.empty((nq * G, kslot), dtype=torch.float32, device=dev)
        oi1 = torch.empty((nq * G, kslot), dtype=torch.long, device=dev)
        _lib.check(L.lzk_topk_merge(ps.data_ptr(), pi.data_ptr(), ncand // G, nq * G, kslot, kslot, 0,
                                    os1.data_ptr(), oi1.data_ptr(), st), "lzk_topk_merge")
        ps, pi, ncand = os1, oi1.to(torch.int32), G * kslot
    os_ = torch.empty((nq, k), dtype=torch.float32, device=dev)
    oi = torch.empty((nq, k), dtype=torch.long, device=dev)
    rc = L.lzk_topk_merge(ps.data_ptr(), pi.data_ptr(), ncand, nq, kslot, int(k),
                          int(idx_offset), os_.data_ptr(), oi.data_ptr(), st)
    _lib.check(rc, "lzk_topk_merge")
    return os_, oi


def _merge_groups(nq: int, nch: int) -> int:
    """Groups per query of the two-level partial-list merge: only when the
    queries alone leave the chip mostly idle (< 64 merge waves); the largest
    divisor G <= 64 of nch that keeps >= 8 chunks per group and <= 512
    first-level waves."""
    if nq >= 64 or nch < 16:
        return 1
    for G in range(min(64, nch // 8, 512 // max(nq, 1)), 1, -1):
        if nch % G == 0:
            return G
    return 1


def _sample_threshold(X, Q, k, kslot, bias, row_label, q_label, alpha, S):
    """Lower bound of each query's k-th score: exact top-k over the strided
    sample X[::S] (lane kernel), lowered by a margin covering the fp32
    accumulation-order difference between the two kernels."""
    N = X.shape[0]
    bs = bias[:N:S].contiguous() if bias is not None else None
    ls = row_label[:N:S].contiguous() if row_label is not None else None
    ts, _ = _flat_topk_lane(X[::S], Q, kslot, kslot, bs, ls, q_label, alpha, 0, None)
    thr = ts[:, k - 1].contiguous()
    thr = thr - 2e-4 * (1.0 + thr.abs())
    return torch.nan_to_num(thr, nan=float("-inf"))


def _cand_lists(dev, nq, cap, slot, zero=True):
    ws = (_ws_cand if slot == 0 else _ws_cand2).get(dev, nq * (4 + 8 * cap))
    cnt = ws[: nq * 4].view(torch.int32)
    cs = ws[nq * 4: nq * 4 + nq * cap * 4].view(torch.float32)
    ci = ws[nq * 4 + nq * cap * 4: nq * 4 + nq * cap * 8].view(torch.int32)
    if zero:  # (zero=False: the caller's first launch zeroes the counts)
        cnt.zero_()
    return cnt, cs, ci


def _select_with_fallback(X, Q, k, kslot, bias, row_label, q_label, alpha, idx_offset, cnt, cs, ci, cap,
                          need=None, ovf_sink=None):
    """Exact per-query select from a candidate list; queries whose list
    overflowed -- or, with ``need``, holds fewer than need[q] entries (a
    speculative threshold that turned out too high) -- are recomputed by the
    lane kernel ON DEVICE (the masked launch skips every query tile without
    such a query -- a few us when none did), so the path never synchronises
    with the host."""
    L = _lib.lib()
    nq, D = Q.shape
    N = X.shape[0]
    dev = X.device
    st = _lib.stream_ptr(dev)
    os_ = torch.empty((nq, k), dtype=torch.float32, device=dev)
    oi = torch.empty((nq, k), dtype=torch.long, device=dev)
    ovf = torch.empty((nq,), dtype=torch.int32, device=dev)
    rc = L.lzk_cand_select(cnt.data_ptr(), cs.data_ptr(), ci.data_ptr(), cap, nq, kslot, int(k),
                           int(idx_offset), os_.data_ptr(), oi.data_ptr(), ovf.data_ptr(), _lib.ptr(need), st)
    _lib.check(rc, "lzk_cand_select")
    if ovf_sink is not None:  # the caller's view of the lists: (overflowed query flags, list lengths)
        ovf_sink.append((ovf, cnt))
    if SPEC_STATS is not None and need is not None:  # LZK_SPEC_STATS=1: queries sent to the exact fallback
        SPEC_STATS.append((need != 0).sum())
    if isinstance(X, LeanRows):
        _lean_fallback(X, Q, k, bias, row_label, q_label, alpha, idx_offset, os_, oi, ovf)
        return os_, oi
    nch = L.lzk_flat_topk_chunks(N, nq, TARGET_WGS)
    part = nq * nch * kslot
    wsf = _ws_fallback.get(dev, part * 8)
    ps = wsf[: part * 4].view(torch.float32)
    pi = wsf[part * 4: part * 8].view(torch.int32)
    rc = L.lzk_flat_topk_partial_masked(X.data_ptr(), X.stride(0), N, Q.data_ptr(), Q.stride(0), nq,
                                        _lib.ptr(bias), _lib.ptr(row_label), _lib.ptr(q_label), float(alpha), D,
                                        kslot, nch, ps.data_ptr(), pi.data_ptr(), ovf.data_ptr(), st)
    _lib.check(rc, "lzk_flat_topk_partial_masked")
    rc = L.lzk_topk_merge_masked(ps.data_ptr(), pi.data_ptr(), nch * kslot, nq, kslot, int(k), int(idx_offset),
                                 os_.data_ptr(), oi.data_ptr(), ovf.data_ptr(), st)
    _lib.check(rc, "lzk_topk_merge_masked")
    return os_, oi


def _lean_fallback(X: LeanRows, Q, k, bias, row_label, q_label, alpha, idx_offset, os_, oi, ovf):
    """Overflowed queries of a lean tenant's candidate select, recomputed
    exactly over the rows converted to bf16 one block at a time (one host
    read of the overflow flags; a block is converted only when some query
    overflowed -- pathological score distributions)."""
    bad = torch.nonzero(ovf).flatten()
    if bad.numel() == 0:
        return
    N = X.shape[0]
    Qb = Q[bad].contiguous()
    ql = q_label[bad].contiguous() if q_label is not None else None
    best_s = best_i = None
    for c0 in range(0, N, X.CHUNK):
        c1 = min(N, c0 + X.CHUNK)
        s, i = flat_topk(X[c0:c1], Qb, k, bias=bias[c0:c1].contiguous() if bias is not None else None,
                         row_label=row_label[c0:c1].contiguous() if row_label is not None else None, q_label=ql,
                         alpha=alpha, idx_offset=c0 + idx_offset)
        if best_s is None:
            best_s, best_i = s, i
            continue
        s, i = torch.cat([best_s, s], 1), torch.cat([best_i, i], 1)
        key = torch.where(i >= 0, i, torch.full_like(i, 1 << 62))
        o = torch.argsort(key, dim=1, stable=True)
        s, i = torch.gather(s, 1, o), torch.gather(i, 1, o)
        o = torch.sort(s, dim=1, descending=True, stable=True).indices[:, :k]
        best_s, best_i = torch.gather(s, 1, o), torch.gather(i, 1, o)
    os_[bad], oi[bad] = best_s, best_i


def _flat_topk_cand(X, Q, k, kslot, bias, row_label, q_label, alpha, idx_offset):
    """Threshold-filtered candidates on the 256x256 pipeline (search256.hip).

    1. thr[q] = lower bound of the k-th score (:func:`_sample_threshold`), so
       every true top-k row passes ``score >= thr``;
    2. candidate pass over all rows; 3. exact select per query with the
       on-device overflow fallback (:func:`_select_with_fallback`).
    """
    L = _lib.lib()
    nq, D = Q.shape
    N = X.shape[0]
    dev = X.device
    S = max(1, min(CAND_STRIDE, N // max(16 * kslot, 1)))
    thr = _sample_threshold(X, Q, k, kslot, bias, row_label, q_label, alpha, S)
    cap = max(1024, 8 * kslot * S)
    cnt, cs, ci = _cand_lists(dev, nq, cap, 0)
    grid = L.lzk_cand_grid(N, nq, 0)
    st = _lib.stream_ptr(dev)
    if grid > 0:
        bbuf, bcap, bcnt = _blk_records(dev, grid, nq, kslot, S, 1)
        bargs = (bbuf.data_ptr(), bcap, bcnt.data_ptr())
    else:
        bargs = (None, 0, None)
    rc = L.lzk_flat_cand(X.data_ptr(), X.stride(0), N, Q.data_ptr(), Q.stride(0), nq, D,
                         _lib.ptr(bias), _lib.ptr(row_label), _lib.ptr(q_label), float(alpha),
                         thr.data_ptr(), cap, cnt.data_ptr(), cs.data_ptr(), ci.data_ptr(), *bargs, st)
    _lib.check(rc, "lzk_flat_cand")
    if grid > 0:
        _lib.check(L.lzk_cand_gather(bargs[0], bcap, bargs[2], grid, cap, nq, cnt.data_ptr(), cs.data_ptr(),
                                     ci.data_ptr(), None, None, None, st), "lzk_cand_gather")
    return _select_with_fallback(X, Q, k, kslot, bias, row_label, q_label, alpha, idx_offset, cnt, cs, ci, cap)


_lib.register("lzk_flat_cand_f8", _lib.I, [_lib.P, _lib.L, _lib.I, _lib.P, _lib.L, _lib.I, _lib.I, _lib.P, _lib.F,
                                           _lib.P, _lib.I, _lib.P, _lib.P, _lib.P, _lib.P, _lib.I, _lib.P, _lib.P])
_lib.register("lzk_cand_grid_f8", _lib.I, [_lib.I, _lib.I])
_lib.register("lzk_set_cu_budget", None, [_lib.I])

# A consolidation batch's candidate scan prefetched under the previous batch's
# apply (TenantGraph.cos_topk_prefetch) runs its persistent blocks on this
# fraction of the CUs: the apply's small kernels need free CUs to make progress
# while the scan (whose waves fill a CU's registers) runs.
PREFETCH_GRID_FRAC = 0.75


class grid_cap:
    """Context: persistent scans launched inside, by THIS thread, use at most
    ``frac`` of the device's CUs (search256.hip g_cu_budget is thread-local:
    the grid-sizing call and the launch of one scan read the same budget, and
    a search on another thread keeps the whole device; restored on exit)."""

    def __init__(self, frac: float):
        self.frac = float(frac)

    def __enter__(self):
        n = torch.cuda.get_device_properties(torch.cuda.current_device()).multi_processor_count
        _lib.lib().lzk_set_cu_budget(max(8, int(n * self.frac)))
        return self

    def __exit__(self, *exc):
        _lib.lib().lzk_set_cu_budget(0)
        return False
_lib.register("lzk_thr_prep", _lib.I, [_lib.P, _lib.L, _lib.I, _lib.P, _lib.P, _lib.I, _lib.P, _lib.P, _lib.P, _lib.P])
_lib.register("lzk_cand_rescore", _lib.I, [_lib.P, _lib.L, _lib.P, _lib.L, _lib.I, _lib.I, _lib.P, _lib.F, _lib.P,
                                           _lib.I, _lib.P, _lib.P, _lib.P, _lib.F, _lib.P, _lib.I, _lib.I, _lib.P,
                                           _lib.P])
_lib.register("lzk_cand_cut", _lib.I, [_lib.P, _lib.L, _lib.L, _lib.P, _lib.L, _lib.I, _lib.I, _lib.I, _lib.P,
                                       _lib.F, _lib.P, _lib.I, _lib.I, _lib.P, _lib.F, _lib.I, _lib.P, _lib.P])
_lib.register("lzk_cand_rescore32", _lib.I, [_lib.P, _lib.L, _lib.P, _lib.L, _lib.I, _lib.I, _lib.P, _lib.F, _lib.P,
                                             _lib.I, _lib.P, _lib.P, _lib.P, _lib.F, _lib.P, _lib.I, _lib.I, _lib.P,
                                             _lib.P])


def bf16_rows(X32: torch.Tensor, Dp: int) -> torch.Tensor:
    """bf16 copy of fp32 rows, zero-padded to Dp columns (the scan layout)."""
    out = torch.zeros((X32.shape[0], Dp), dtype=torch.bfloat16, device=X32.device)
    out[:, : X32.shape[1]] = X32
    return out


class LeanRows:
    """The fp32 rows of a lean tenant (no bf16 copy kept in HBM) standing in
    for the bf16 operand of the int8 search paths: a slice converts on the fly
    (bf16, zero-padded to Dp -- the 1/S threshold sample and the rare overflow
    fallback); the re-score above the error cut reads the fp32 rows and the
    fp32 queries ``Q32`` directly (lzk_cand_rescore32)."""
    dtype = torch.bfloat16
    CHUNK = 1 << 20  # rows per converted block of the overflow fallback

    def __init__(self, X32: torch.Tensor, Dp: int, Q32: torch.Tensor):
        self.X32, self.Dp = X32, int(Dp)
        self.Q32 = Q32.float().contiguous()
        self.device = X32.device
        self.shape = (X32.shape[0], self.Dp)

    def __getitem__(self, sl):
        return bf16_rows(self.X32[sl], self.Dp)
_lib.register("lzk_flat_cand_dual_i8", _lib.I, [_lib.P, _lib.L, _lib.I, _lib.P, _lib.L, _lib.I, _lib.I, _lib.P,
                                                _lib.P, _lib.P, _lib.P, _lib.P, _lib.F, _lib.P, _lib.P, _lib.I,
                                                _lib.P, _lib.P, _lib.P, _lib.P, _lib.P, _lib.P, _lib.P, _lib.I,
                                                _lib.P, _lib.P])
_lib.register("lzk_flat_cand_i8", _lib.I, [_lib.P, _lib.L, _lib.I, _lib.P, _lib.L, _lib.I, _lib.I, _lib.P, _lib.P,
                                           _lib.P, _lib.F, _lib.P, _lib.I, _lib.P, _lib.P, _lib.P, _lib.P, _lib.I,
                                           _lib.P, _lib.P])

_lib.register("lzk_scan8_narrow_grid", _lib.I, [_lib.I])
_lib.register("lzk_scan8_narrow", _lib.I, [_lib.P, _lib.L, _lib.I, _lib.P, _lib.L, _lib.I, _lib.I, _lib.P, _lib.P,
                                           _lib.P, _lib.F, _lib.P, _lib.P, _lib.I, _lib.P, _lib.P])
_lib.register("lzk_farthest_first_ws", _lib.L, [_lib.I, _lib.I])
_lib.register("lzk_farthest_first", _lib.I, [_lib.P, _lib.L, _lib.I, _lib.I, _lib.I, _lib.P, _lib.P, _lib.P])
_lib.register("lzk_cos_rerank64", _lib.I, [_lib.P, _lib.L, _lib.P, _lib.L, _lib.I, _lib.P, _lib.P, _lib.I, _lib.I,
                                           _lib.I, _lib.P, _lib.P, _lib.P])
NARROW_MAX_Q = 128  # below this many queries the int8 scan is the HBM-bound narrow kernel
_lib.register("lzk_i8_query", _lib.I, [_lib.P, _lib.L, _lib.I, _lib.I, _lib.I, _lib.P, _lib.D, _lib.P, _lib.F,
                                       _lib.F, _lib.F, _lib.P, _lib.L, _lib.P, _lib.P, _lib.P, _lib.P])

# the narrow kernel for batches under 128 queries (scan8.hip) is on
# (SCAN8_NARROW = False disables it)
SCAN8_NARROW = True


def _wave_records(dev, grid: int, nq: int, kslot: int, S: int, lists: int):
    """Per-wave candidate record regions of the int8 scan (scan8.hip: 8
    regions per block, each filled by one wave without atomics): int4
    [grid * 8, capw] + int32 counts [grid * 8]; capw ~8x the expected records
    per wave (a region that overflows marks every query for the fallback)."""
    regions = grid * 8
    capw = max(1024, lists * nq * kslot * S // max(grid, 1))
    ws = _ws_blk.get(dev, regions * capw * 16 + regions * 4)
    buf = ws[: regions * capw * 16]
    cnt = ws[regions * capw * 16: regions * capw * 16 + regions * 4].view(torch.int32)
    return buf, capw, cnt, regions


def _scan8_narrow(X8, rscale, Q8, qscale, bias, alpha, thr, kslot, S, cap, ca):
    """Narrow-batch int8 candidate pass (scan8.hip scan8_narrow_kernel,
    nq < 128: 16-row blocks streamed into registers against the queries in
    LDS) + gather into the per-query lists ``ca``."""
    L = _lib.lib()
    nq, Dp = Q8.shape
    N = X8.shape[0]
    dev = Q8.device
    st = _lib.stream_ptr(dev)
    grid = L.lzk_scan8_narrow_grid(N)
    bbuf, bcap, bcnt, regions = _wave_records(dev, grid, nq, kslot, S, 1)
    _lib.check(L.lzk_scan8_narrow(X8.data_ptr(), X8.stride(0), N, Q8.data_ptr(), Q8.stride(0), nq, Dp,
                                  _lib.ptr(bias), rscale.data_ptr(), qscale.data_ptr(), float(alpha), thr.data_ptr(),
                                  bbuf.data_ptr(), bcap, bcnt.data_ptr(), st), "lzk_scan8_narrow")
    _lib.check(L.lzk_cand_gather(bbuf.data_ptr(), bcap, bcnt.data_ptr(), regions, cap, nq, ca[0].data_ptr(),
                                 ca[1].data_ptr(), ca[2].data_ptr(), None, None, None, st), "lzk_cand_gather")


FP8_MAX = 448.0


def quantize_e4m3(x: torch.Tensor, scale: float, out: torch.Tensor = None) -> torch.Tensor:
    """x * scale as OCP e4m3 bytes (uint8), saturated to +-448."""
    q = (x.float() * scale).clamp_(-FP8_MAX, FP8_MAX).to(torch.float8_e4m3fn).view(torch.uint8)
    if out is not None:
        out.copy_(q)
        return out
    return q


def flat_topk_fp8(X8: torch.Tensor, Q8: torch.Tensor, scale2: float, X16: torch.Tensor, Q16: torch.Tensor, k: int,
                  *, bias=None, alpha: float = 1.0, margin=None):
    """Top-k of ``alpha * <Q, X> + bias`` with the candidate scan on the fp8
    MFMA (twice the bf16 rate, half the bytes) and exact bf16 scores for the
    candidates.

    X8 / Q8: e4m3 bytes [N, Dp] / [nq, Dp] of X16 / Q16 times per-tensor
    scales with product ``scale2`` (Dp % 128 == 0); X16 / Q16 the bf16 rows
    and queries. ``margin`` [nq] (fp32, >= 0): the fp8 error allowance -- the
    sampled threshold (exact bf16 k-th best of a 1/S row sample, a lower bound
    of the true k-th score) is lowered by it, so a row whose exact score clears
    the true k-th best stays a candidate unless its fp8 error exceeds the
    margin. Candidates are re-scored from the bf16 rows (``cand_rescore``) and
    selected exactly; overflowed lists go to the exact bf16 fallback.
    Returns (scores fp32 [nq, k], rows int64 [nq, k]) like :func:`flat_topk`."""
    L = _lib.lib()
    nq, Dp = Q16.shape
    N = X16.shape[0]
    kslot = L.lzk_flat_topk_kslot(int(k))
    assert kslot > 0 and X8.dtype == torch.uint8 and Q8.dtype == torch.uint8 and Dp % 128 == 0
    assert X8.shape[1] == Dp and X8.stride(1) == 1 and Q8.stride(1) == 1 and X8.shape[0] >= N
    dev = X16.device
    S = max(1, min(CAND_STRIDE, N // max(16 * kslot, 1)))
    thr = _sample_threshold(X16, Q16, k, kslot, bias, None, None, alpha, S)
    if margin is not None:
        thr = (thr - margin).contiguous()
    cap = max(2048, 32 * kslot * S)
    cnt, cs, ci = _cand_lists(dev, nq, cap, 0)
    grid = L.lzk_cand_grid_f8(N, nq)
    bbuf, bcap, bcnt = _blk_records(dev, grid, nq, kslot, 4 * S, 1)
    st = _lib.stream_ptr(dev)
    _lib.check(L.lzk_flat_cand_f8(X8.data_ptr(), X8.stride(0), N, Q8.data_ptr(), Q8.stride(0), nq, Dp, _lib.ptr(bias),
                                  float(alpha / scale2), thr.data_ptr(), cap, cnt.data_ptr(), cs.data_ptr(),
                                  ci.data_ptr(), bbuf.data_ptr(), bcap, bcnt.data_ptr(), st), "lzk_flat_cand_f8")
    _lib.check(L.lzk_cand_gather(bbuf.data_ptr(), bcap, bcnt.data_ptr(), grid, cap, nq, cnt.data_ptr(), cs.data_ptr(),
                                 ci.data_ptr(), None, None, None, st), "lzk_cand_gather")
    _lib.check(L.lzk_cand_rescore(X16.data_ptr(), X16.stride(0), Q16.data_ptr(), Q16.stride(0), nq, Dp,
                                  _lib.ptr(bias), float(alpha), cnt.data_ptr(), cap, cs.data_ptr(), ci.data_ptr(), None,
                                  float("-inf"), None, 0, 0, None, st), "lzk_cand_rescore")
    return _select_with_fallback(X16, Q16, k, kslot, bias, None, None, alpha, 0, cnt, cs, ci, cap)


def quantize_i8_rows(x: torch.Tensor, out: torch.Tensor = None, scale_out: torch.Tensor = None):
    """Symmetric per-row int8: q = round(x / s), s = max|x_row| / 127 (0 for
    an all-zero row, which quantises exactly and so must not widen any error
    bound), so x ~= q * s with |error| <= s / 2 per element.
    Returns (q int8 [n, D] (or ``out`` filled in its first D columns), s fp32 [n])."""
    xf = x.float()
    amax = xf.abs().amax(1)
    s = torch.where(amax > 0, amax / 127.0, torch.zeros_like(amax))
    den = torch.where(amax > 0, s, torch.ones_like(amax))
    q = torch.round(xf / den[:, None]).clamp_(-127, 127).to(torch.int8)
    if out is not None:
        out[:, : q.shape[1]] = q
        q = out
    if scale_out is not None:
        scale_out.copy_(s)
        s = scale_out
    return q, s


def i8_query(q16: torch.Tensor, d: int, sumsq: torch.Tensor, n_sumsq: int, smax: torch.Tensor, alpha: float,
             z: float, xn: float = 1.0):
    """int8 queries, scales and both error margins of the int8 store search
    in one launch (search256.hip i8_query_kernel): the same quantisation as
    :func:`quantize_i8_rows`, the statistical margin (scan threshold) and the
    worst-case one (re-score cut + certificate) of TenantGraph._i8_query.
    Returns (q8 int8 [nq, Dp], qs fp32 [nq], margin fp32 [nq], margin_rig fp32 [nq])."""
    nq, Dp = q16.shape
    dev = q16.device
    q8 = torch.empty((nq, Dp), dtype=torch.int8, device=dev)
    qs = torch.empty(nq, dtype=torch.float32, device=dev)
    margin = torch.empty(nq, dtype=torch.float32, device=dev)
    margin_rig = torch.empty(nq, dtype=torch.float32, device=dev)
    q16 = q16.contiguous()
    _lib.check(_lib.lib().lzk_i8_query(q16.data_ptr(), q16.stride(0), nq, Dp, int(d), sumsq.data_ptr(),
                                       1.0 / max(int(n_sumsq), 1), smax.data_ptr(), abs(float(alpha)), float(z),
                                       float(xn), q8.data_ptr(), q8.stride(0), qs.data_ptr(), margin.data_ptr(),
                                       margin_rig.data_ptr(), _lib.stream_ptr(dev)), "lzk_i8_query")
    return q8, qs, margin, margin_rig


def flat_topk_i8(X8: torch.Tensor, rscale: torch.Tensor, Q8: torch.Tensor, qscale: torch.Tensor,
                 X16: torch.Tensor, Q16: torch.Tensor, k: int, *, bias=None, alpha: float = 1.0, margin=None,
                 margin_rig=None):
    """Top-k of ``alpha * <Q16, X16> + bias`` with the candidate scan on the
    int8 MFMA (v_mfma_i32_16x16x64_i8: twice the bf16 rate, half the bytes).

    X8 / Q8: per-row symmetric int8 of X16 / Q16 (:func:`quantize_i8_rows`,
    Dp % 128 == 0, Dp <= 1024) with fp32 scales ``rscale`` [N] / ``qscale``
    [nq]. Two per-query allowances for |int8 score - bf16 score|: ``margin``
    (fp32 [nq]) only sets how many candidates the scan keeps -- TenantGraph
    passes its statistical estimate -- and ``margin_rig`` must BOUND the
    difference for every row (TenantGraph: the worst case of every term; when
    omitted, ``margin`` is taken as the bound). The result always equals the
    bf16 scan's:
      1. thr = bf16 sample bound - margin: tau = the 1/S sample's SPEC_J-th best
         (speculative) or k-th best; the int8 scan keeps every row whose int8
         score clears thr;
      2. cut = (k-th best int8 score of the list) - 2 * margin_rig: a row of
         the true top-k has int8 score >= T - m >= that cut (T the true k-th
         score, itself >= the list's k-th int8 score - m), so only entries
         above the cut are re-scored from the bf16 rows;
      3. certificate (in the re-score kernel): every row the scan dropped has
         bf16 score < thr + margin_rig, so a query whose k re-scored entries
         reach thr + margin_rig has its exact top-k in the list; any other
         query -- a statistical margin or a speculative threshold that was too
         optimistic -- is recomputed by the exact bf16 fallback, as is a list
         that overflowed;
      4. exact select.
    Returns (scores fp32 [nq, k], rows int64 [nq, k]) like :func:`flat_topk`."""
    L = _lib.lib()
    nq, Dp = Q16.shape
    N = X16.shape[0]
    kslot = L.lzk_flat_topk_kslot(int(k))
    assert kslot > 0 and X8.dtype == torch.int8 and Q8.dtype == torch.int8 and Dp % 128 == 0 and Dp <= 1024
    assert X8.shape[1] == Dp and X8.stride(1) == 1 and Q8.stride(1) == 1 and X8.shape[0] >= N
    assert rscale.dtype == torch.float32 and qscale.dtype == torch.float32 and rscale.shape[0] >= N
    assert alpha > 0
    dev = X16.device
    if margin_rig is None:
        margin_rig = margin  # (None: no bound known -- every list entry is re-scored)
    narrow = nq < NARROW_MAX_Q and SCAN8_NARROW and Dp % 64 == 0
    S = max(1, min(CAND_STRIDE_NARROW if narrow else CAND_STRIDE, N // max(16 * kslot, 1)))
    J = SPEC_J_NARROW if narrow else SPEC_J
    spec = 0 < J < k and S >= SPEC_MIN_STRIDE
    # the 1/S sample's top-kslot (lane kernel); speculative threshold: its
    # J-th best (~J * S-th overall) instead of its k-th -- lists ~k / J times
    # shorter; the certificate sends a query whose threshold was too high to
    # the exact fallback
    bs = bias[:N:S].contiguous() if bias is not None else None
    ts, _ = _flat_topk_lane(X16[::S], Q16, kslot, kslot, bs, None, None, alpha, 0, None)
    # narrow batches scan at HBM speed with a worst-case margin by default:
    # longer lists (a few thousand rows per query) cost next to nothing there
    cap = max(NARROW_CAP if narrow else 2048, 16 * kslot * S)
    cnt, cs, ci = _cand_lists(dev, nq, cap, 0, zero=False)
    # tau (sample bound - slack), thr = tau - margin, the certificate level
    # thr + margin_rig and the zeroed list counts: one launch (thr_prep_kernel)
    thr = torch.empty(nq, dtype=torch.float32, device=dev)
    cert = torch.empty(nq, dtype=torch.float32, device=dev)
    mg = margin.float().contiguous() if margin is not None else None
    mr = margin_rig.float().contiguous() if margin_rig is not None else None
    _lib.check(L.lzk_thr_prep(ts.data_ptr(), ts.stride(0), (J if spec else k) - 1, _lib.ptr(mg), _lib.ptr(mr), nq,
                              thr.data_ptr(), cert.data_ptr(), cnt.data_ptr(), _lib.stream_ptr(dev)), "lzk_thr_prep")
    qs = qscale.contiguous()
    need = torch.empty(nq, dtype=torch.int32, device=dev)
    chk = (cert, k, cap + 1, need)
    if narrow:
        _scan8_narrow(X8[:N], rscale[:N], Q8, qs, bias, alpha, thr, kslot, 2 * S, cap, (cnt, cs, ci))
    else:
        grid = L.lzk_cand_grid_f8(N, nq)
        bbuf, bcap, bcnt = _blk_records(dev, grid, nq, kslot, 2 * S, 1)
        st = _lib.stream_ptr(dev)
        _lib.check(L.lzk_flat_cand_i8(X8.data_ptr(), X8.stride(0), N, Q8.data_ptr(), Q8.stride(0), nq, Dp,
                                      _lib.ptr(bias), rscale.data_ptr(), qs.data_ptr(), float(alpha), thr.data_ptr(),
                                      cap, cnt.data_ptr(), cs.data_ptr(), ci.data_ptr(), bbuf.data_ptr(), bcap,
                                      bcnt.data_ptr(), st), "lzk_flat_cand_i8")
        _lib.check(L.lzk_cand_gather(bbuf.data_ptr(), bcap, bcnt.data_ptr(), grid, cap, nq, cnt.data_ptr(),
                                     cs.data_ptr(), ci.data_ptr(), None, None, None, st), "lzk_cand_gather")
    _rescore_above_cut(X16, Q16, k, kslot, bias, alpha, margin_rig, cnt, cs, ci, cap, chk=chk)
    return _select_with_fallback(X16, Q16, k, kslot, bias, None, None, alpha, 0, cnt, cs, ci, cap, need=need)


def _cert_tau(thr: torch.Tensor, margin_rig: torch.Tensor, floor: float = None,
              floor_tol: float = 0.0) -> torch.Tensor:
    """The certificate level of a low-precision scan list: thr + margin_rig
    (+ relative slack) -- no row the scan dropped can reach it. With a caller
    floor that the level does not exceed (by more than ``floor_tol``), every
    row at or above floor + floor_tol is in the list already: -inf, certified
    without a count. The floor test comes BEFORE the relative slack: a
    threshold clamped to floor - margin_rig gives thr + margin_rig = floor up
    to fp32 rounding, which the slack (1e-6 (1 + |t|)) would always push
    above the floor, so the floor certificate never fired and every
    floor-clamped query went to the exact fallback."""
    t = thr + margin_rig if margin_rig is not None else thr
    fl_ok = (t <= float(floor) + float(floor_tol)) if floor is not None else None
    t = t + 1e-6 * (1.0 + t.abs())
    if fl_ok is not None:
        t = torch.where(fl_ok, torch.full_like(t, float("-inf")), t)
    # (neginf= too: nan_to_num's default maps -inf to -FLT_MAX, which the
    # re-score kernel's "tau == -inf: certified" test does not recognise)
    return torch.nan_to_num(t, nan=float("-inf"), neginf=float("-inf")).contiguous()


# Speculative store-search threshold (flat_topk_i8, wide batches): the 1/S
# sample's SPEC_J-th best score; SPEC_J = 0 restores the sample's k-th best.
SPEC_J = 5
# narrow batches: the sample's 3rd best (~192nd row overall at S = 64): a query
# is sent to the fallback only when 3 of its top-10 rows are in the 1/S sample
SPEC_J_NARROW = 3
NARROW_CAP = 16384
SPEC_MIN_STRIDE = 32
SPEC_STATS = [] if os.environ.get("LZK_SPEC_STATS") == "1" else None  # diagnostic: fallback queries per search


def _rescore_above_cut(X16, Q16, k, kslot, bias, alpha, margin, cnt, cs, ci, cap, floor=None, chk=None):
    """int8 candidate lists -> exact bf16 scores for the entries that can
    still reach the query's top-k; the others become -inf without a row read.
    ``margin`` bounds |int8 score - bf16 score| (see :func:`flat_topk_i8`).
    The cut: the list's k best entries by int8 score are scored exactly
    first; the smallest of those k exact scores, L, is a lower bound of the
    true k-th score, so a row of the true top-k has int8 score >= L - margin
    (tighter than (k-th int8 score) - 2 margin: a few hundred re-scored rows
    instead of thousands under a worst-case margin). ``chk`` = (tau [nq], k,
    need_val, need [nq] int32): need[q] = 0 when k re-scored entries reach
    tau[q] (or tau[q] is -inf), else need_val (the per-query certificate)."""
    tau_p, k_need, need_val, need_p = (None, 0, 0, None) if chk is None else (
        chk[0].data_ptr(), int(chk[1]), int(chk[2]), chk[3].data_ptr())
    L = _lib.lib()
    nq, Dp = Q16.shape
    dev = Q16.device
    st = _lib.stream_ptr(dev)
    cut = None
    if margin is not None:
        s8 = torch.empty((nq, kslot), dtype=torch.float32, device=dev)
        i8 = torch.empty((nq, kslot), dtype=torch.long, device=dev)
        ovf = torch.empty((nq,), dtype=torch.int32, device=dev)
        _lib.check(L.lzk_cand_select(cnt.data_ptr(), cs.data_ptr(), ci.data_ptr(), cap, nq, kslot, kslot, 0,
                                     s8.data_ptr(), i8.data_ptr(), ovf.data_ptr(), None, st), "lzk_cand_select")
        # the k best entries scored exactly, their minimum L -> the cut
        # L - margin (- fp32 slack), raised to floor - margin: ONE launch
        # (search256.hip cand_cut_kernel; rows outside the scanned ones, e.g.
        # an overflowed list's, count as missing)
        cut = torch.empty(nq, dtype=torch.float32, device=dev)
        mg = margin.float().contiguous()
        if isinstance(X16, LeanRows):
            Xc, Qc, f32 = X16.X32, X16.Q32, 1
        else:
            Xc, Qc, f32 = X16, Q16, 0
        _lib.check(L.lzk_cand_cut(Xc.data_ptr(), Xc.stride(0), int(X16.shape[0]), Qc.data_ptr(), Qc.stride(0),
                                  int(Xc.shape[1]) if f32 else Dp, nq, f32, _lib.ptr(bias), float(alpha),
                                  i8.data_ptr(), kslot, int(k), mg.data_ptr(),
                                  float(floor) if floor is not None else 0.0, int(floor is not None),
                                  cut.data_ptr(), st), "lzk_cand_cut")
    fl = float("-inf") if floor is None else float(floor)
    if isinstance(X16, LeanRows):
        X32, Q32 = X16.X32, X16.Q32
        _lib.check(L.lzk_cand_rescore32(X32.data_ptr(), X32.stride(0), Q32.data_ptr(), Q32.stride(0), nq,
                                        X32.shape[1], _lib.ptr(bias), float(alpha), cnt.data_ptr(), cap,
                                        cs.data_ptr(), ci.data_ptr(), _lib.ptr(cut), fl, tau_p, k_need, need_val,
                                        need_p, st), "lzk_cand_rescore32")
        return
    _lib.check(L.lzk_cand_rescore(X16.data_ptr(), X16.stride(0), Q16.data_ptr(), Q16.stride(0), nq, Dp,
                                  _lib.ptr(bias), float(alpha), cnt.data_ptr(), cap, cs.data_ptr(), ci.data_ptr(),
                                  _lib.ptr(cut), fl, tau_p, k_need, need_val, need_p, st), "lzk_cand_rescore")


def flat_topk_dual_i8(X8: torch.Tensor, rscale: torch.Tensor, Q8: torch.Tensor, qscale: torch.Tensor,
                      X16: torch.Tensor, Q16: torch.Tensor, k: int, *, row_label, q_label, bias=None,
                      alpha: float = 1.0, margin=None, margin_rig=None, floor: float = None,
                      floor_tol: float = None, stats: Optional[list] = None):
    """:func:`flat_topk_dual` with the candidate scan on the int8 MFMA (the
    rows' int8 copy, see :func:`flat_topk_i8` for the two margins): each list's
    threshold is max(sampled bf16 k-th best - margin, floor - margin_rig), both
    lists are re-scored from the bf16 rows above their worst-case cut and
    certified per query (k entries at thr + margin_rig, or a threshold that
    sits margin_rig below the floor), uncertified queries recomputed exactly --
    the same lists as the bf16 dual scan for every entry >= floor + floor_tol
    (``floor_tol``: how far above the floor the caller's decisions start;
    default fp32 rounding, 1e-6 (1 + |floor|)). ``stats``:
    receives the (fallback flags, list lengths) device tensors of both lists.
    Returns ((scores, rows) unfiltered, (scores, rows) filtered)."""
    L = _lib.lib()
    nq, Dp = Q16.shape
    N = X16.shape[0]
    kslot = L.lzk_flat_topk_kslot(int(k))
    assert kslot > 0 and X8.dtype == torch.int8 and Q8.dtype == torch.int8 and Dp % 128 == 0 and Dp <= 1024
    assert row_label.dtype == torch.int32 and q_label.dtype == torch.int32 and alpha > 0
    dev = X16.device
    if margin_rig is None:
        margin_rig = margin  # (None: no bound known -- every list entry is re-scored)
    S = max(1, min(CAND_STRIDE, N // max(16 * kslot, 1)))
    thr_b = _sample_threshold(X16, Q16, k, kslot, bias, row_label, q_label, alpha, S)
    thr_a = _sample_threshold(X16, Q16, k, kslot, bias, None, None, alpha, S)
    if margin is not None:
        thr_a, thr_b = thr_a - margin, thr_b - margin
    if floor is not None:
        fl = float(floor) - (margin_rig if margin_rig is not None else 0.0)
        fl = torch.as_tensor(fl, dtype=thr_a.dtype, device=dev)
        thr_a, thr_b = torch.maximum(thr_a, fl), torch.maximum(thr_b, fl)
    thr_a, thr_b = thr_a.contiguous(), thr_b.contiguous()
    cap = max(2048, 16 * kslot * S)
    ca = _cand_lists(dev, nq, cap, 0)
    cb = _cand_lists(dev, nq, cap, 1)
    qs = qscale.contiguous()
    _dual_i8_template(X8, rscale, Q8, qs, X16, bias, alpha, thr_a, thr_b, row_label, q_label, kslot, S, cap, ca, cb)
    need_a = torch.empty(nq, dtype=torch.int32, device=dev)
    need_b = torch.empty(nq, dtype=torch.int32, device=dev)
    if floor is not None and floor_tol is None:
        floor_tol = 1e-6 * (1.0 + abs(float(floor)))
    _rescore_above_cut(X16, Q16, k, kslot, bias, alpha, margin_rig, *ca, cap, floor=floor,
                       chk=(_cert_tau(thr_a, margin_rig, floor, floor_tol or 0.0), k, cap + 1, need_a))
    _rescore_above_cut(X16, Q16, k, kslot, bias, alpha, margin_rig, *cb, cap, floor=floor,
                       chk=(_cert_tau(thr_b, margin_rig, floor, floor_tol or 0.0), k, cap + 1, need_b))
    ra = _select_with_fallback(X16, Q16, k, kslot, bias, None, None, alpha, 0, *ca, cap, need=need_a,
                               ovf_sink=stats)
    rb = _select_with_fallback(X16, Q16, k, kslot, bias, row_label, q_label, alpha, 0, *cb, cap, need=need_b,
                               ovf_sink=stats)
    if stats is not None:
        stats.append(cap)
    return ra, rb


def _dual_i8_template(X8, rscale, Q8, qs, X16, bias, alpha, thr_a, thr_b, row_label, q_label, kslot, S, cap, ca, cb):
    """The dual int8 pass on the shared 256^2 template."""
    L = _lib.lib()
    nq, Dp = Q8.shape
    N = X16.shape[0]
    dev = Q8.device
    grid = L.lzk_cand_grid_f8(N, nq)
    bbuf, bcap, bcnt = _blk_records(dev, grid, nq, kslot, 2 * S, 2)
    st = _lib.stream_ptr(dev)
    _lib.check(L.lzk_flat_cand_dual_i8(X8.data_ptr(), X8.stride(0), N, Q8.data_ptr(), Q8.stride(0), nq, Dp,
                                       _lib.ptr(bias), rscale.data_ptr(), qs.data_ptr(), row_label.data_ptr(),
                                       q_label.data_ptr(), float(alpha), thr_a.data_ptr(), thr_b.data_ptr(), cap,
                                       ca[0].data_ptr(), ca[1].data_ptr(), ca[2].data_ptr(), cb[0].data_ptr(),
                                       cb[1].data_ptr(), cb[2].data_ptr(), bbuf.data_ptr(), bcap, bcnt.data_ptr(), st),
               "lzk_flat_cand_dual_i8")
    _lib.check(L.lzk_cand_gather(bbuf.data_ptr(), bcap, bcnt.data_ptr(), grid, cap, nq, ca[0].data_ptr(),
                                 ca[1].data_ptr(), ca[2].data_ptr(), cb[0].data_ptr(), cb[1].data_ptr(),
                                 cb[2].data_ptr(), st), "lzk_cand_gather")


# Speculative list-B threshold of flat_topk_dual (DUAL_SPEC = True): aim for
# this many expected label rows above it. Off by default: on the 10M x 1024
# consolidation shape it cuts the scan 13.93 -> 12.90 ms (a round-1 probe:
# list-B candidates 198 -> 16 per query), but the top-16 sample pass it needs
# costs ~1.1 ms more than the top-4 one, so the whole call ties (15.07 vs
# 15.13 ms, bench/ab_dual_spec.py, profiles/ab_dual_spec_r1.json).
DUAL_SPEC = False
DUAL_SPEC_E = 16.0
SPEC_SLOTS = 16


def _margin(t):
    t = t - 2e-4 * (1.0 + t.abs())
    return torch.nan_to_num(t, nan=float("-inf"))


def _spec_threshold_b(ts, thr_b, row_label, q_label, n_labels, N, S, k):
    """Speculative list-B thresholds from the global sample's top-16 ``ts``.

    The safe bound ``thr_b`` (k-th best of the label-filtered 1/S sample)
    sits around the label's top k*S rows, so ~k*S*n_labels rows of ALL labels
    clear it and each costs the scan's per-score label test. The global
    sample's j-th best leaves about E = j*S*n_l/N rows of a label with n_l
    rows above it; j is chosen per query for E ~ DUAL_SPEC_E. The list stays
    exact: a query whose list ends up with fewer than k entries is recomputed
    by the select's fallback (need[q] = k), so only speed depends on the
    estimate. Returns (thr, need)."""
    dev = ts.device
    lab = row_label.to(torch.float32)
    hist = torch.histc(lab, bins=n_labels, min=0, max=n_labels)  # rows per label (no host sync)
    ql = q_label.long()
    n_l = torch.where(ql >= 0, hist[ql.clamp(0, n_labels - 1)], torch.full_like(ql, N, dtype=torch.float32))
    n_l = torch.where((ql >= n_labels), torch.zeros_like(n_l), n_l)
    j = torch.ceil(DUAL_SPEC_E * N / (S * n_l.clamp_min(1.0))).long()
    ok = j <= ts.shape[1]
    cand = _margin(ts.gather(1, (j.clamp(1, ts.shape[1]) - 1)[:, None])[:, 0])
    spec = ok & (cand > thr_b)
    thr = torch.where(spec, cand, thr_b).contiguous()
    need = torch.where(spec, torch.full_like(ql, k), torch.zeros_like(ql)).to(torch.int32).contiguous()
    return thr, need


def flat_topk_dual(X: torch.Tensor, Q: torch.Tensor, k: int, *, row_label, q_label, bias=None,
                   alpha: float = 1.0, idx_offset: int = 0, n_labels: int = None, floor: float = None):
    """Two searches of the same queries from ONE scan: the unfiltered top-k and
    the label-filtered top-k (label < 0 = any). Consolidation needs both --
    global dedupe/links and within-shard links (reference memory_system.py:
    719-733, 816-836, 853-889) -- and the large-batch scan is MFMA-bound, so
    the candidate path computes each score once and files it into two lists.
    ``n_labels`` (row labels in [0, n_labels)) enables the speculative
    list-B threshold (:func:`_spec_threshold_b`); results are exact either way.
    ``floor``: the caller only needs entries scoring >= floor (consolidation
    acts on cos > 0.5 only): both candidate thresholds are raised to it, so
    the lists stay short and list B's label test almost never runs; slots
    with no such entry come back as (-inf, -1). The caller lowers ``floor``
    by its bf16 error allowance.
    Returns ((scores, rows) unfiltered, (scores, rows) filtered)."""
    if Q.dim() == 1:
        Q = Q[None, :]
    nq, D = Q.shape
    N = X.shape[0]
    if not X.is_cuda:
        return (_ref_topk(X, Q, k, bias, None, None, alpha, idx_offset),
                _ref_topk(X, Q, k, bias, row_label, q_label, alpha, idx_offset))
    L = _lib.lib()
    kslot = L.lzk_flat_topk_kslot(int(k))
    if kslot < 0 or N == 0 or nq == 0 or not _use_cand(N, nq, kslot):
        return (flat_topk(X, Q, k, bias=bias, alpha=alpha, idx_offset=idx_offset),
                flat_topk(X, Q, k, bias=bias, row_label=row_label, q_label=q_label, alpha=alpha,
                          idx_offset=idx_offset))
    assert X.dtype == torch.bfloat16 and Q.dtype == torch.bfloat16 and D % 64 == 0
    assert row_label.dtype == torch.int32 and q_label.dtype == torch.int32
    dev = X.device
    S = max(1, min(CAND_STRIDE, N // max(16 * kslot, 1)))
    thr_b = _sample_threshold(X, Q, k, kslot, bias, row_label, q_label, alpha, S)
    need_b = None
    if DUAL_SPEC and n_labels and S > 1 and kslot < SPEC_SLOTS:
        bs = bias[:N:S].contiguous() if bias is not None else None
        ts, _ = _flat_topk_lane(X[::S], Q, SPEC_SLOTS, SPEC_SLOTS, bs, None, None, alpha, 0, None)
        thr_a = _margin(ts[:, k - 1]).contiguous()
        thr_b, need_b = _spec_threshold_b(ts, thr_b, row_label, q_label, int(n_labels), N, S, k)
    else:
        thr_a = _sample_threshold(X, Q, k, kslot, bias, None, None, alpha, S)
    if floor is not None:
        thr_a = thr_a.clamp_min(float(floor)).contiguous()
        thr_b = thr_b.clamp_min(float(floor)).contiguous()
        need_b = None
    cap = max(1024, 8 * kslot * S)
    ca = _cand_lists(dev, nq, cap, 0)
    cb = _cand_lists(dev, nq, cap, 1)
    grid = L.lzk_cand_grid(N, nq, 1)
    bbuf, bcap, bcnt = _blk_records(dev, grid, nq, kslot, S, 2)
    st = _lib.stream_ptr(dev)
    rc = L.lzk_flat_cand_dual(X.data_ptr(), X.stride(0), N, Q.data_ptr(), Q.stride(0), nq, D, _lib.ptr(bias),
                              row_label.data_ptr(), q_label.data_ptr(), float(alpha), thr_a.data_ptr(),
                              thr_b.data_ptr(), cap, ca[0].data_ptr(), ca[1].data_ptr(), ca[2].data_ptr(),
                              cb[0].data_ptr(), cb[1].data_ptr(), cb[2].data_ptr(), bbuf.data_ptr(), bcap,
                              bcnt.data_ptr(), st)
    _lib.check(rc, "lzk_flat_cand_dual")
    _lib.check(L.lzk_cand_gather(bbuf.data_ptr(), bcap, bcnt.data_ptr(), grid, cap, nq, ca[0].data_ptr(),
                                 ca[1].data_ptr(), ca[2].data_ptr(), cb[0].data_ptr(), cb[1].data_ptr(),
                                 cb[2].data_ptr(), st), "lzk_cand_gather")
    ra = _select_with_fallback(X, Q, k, kslot, bias, None, None, alpha, idx_offset, *ca, cap)
    rb = _select_with_fallback(X, Q, k, kslot, bias, row_label, q_label, alpha, idx_offset, *cb, cap, need=need_b)
    return ra, rb


def segment_topk(xs, Q: torch.Tensor, k: int, *, biases=None, scales=None, alpha: float = 1.0, qbias=None):
    """Multi-tenant batch: query ``q`` scans only the rows ``xs[q]`` (its tenant's
    arena or a slice of a shared arena) -- one launch for the whole batch
    (csrc/kernels/segment.hip).

    score = alpha * <Q[q], xs[q][r]> * scales[q][r] + biases[q][r] + qbias[q].
    ``xs``: list of 2-D tensors with a common dtype (bf16 or fp32) and row
    stride; ``biases``/``scales``: None or lists of fp32 vectors. Returns
    (scores [nq, k] fp32, rows [nq, k] int64 local to each segment, -1 empty).
    """
    nq = Q.shape[0]
    assert len(xs) == nq
    dev = Q.device
    D = Q.shape[1]
    if not Q.is_cuda:
        out_s = torch.full((nq, k), float("-inf"))
        out_i = torch.full((nq, k), -1, dtype=torch.long)
        for q in range(nq):
            X = xs[q]
            if X.shape[0] == 0:
                continue
            s = alpha * (X[:, :D].float() @ Q[q].float())
            if scales is not None and scales[q] is not None:
                s = s * scales[q].float()
            if biases is not None and biases[q] is not None:
                s = s + biases[q].float()
            if qbias is not None:
                s = s + float(qbias[q])
            o = torch.argsort(-s, stable=True)[:k]
            keep = ~torch.isinf(s[o]) | (s[o] > 0)
            o = o[keep]
            out_s[q, : o.numel()] = s[o]
            out_i[q, : o.numel()] = o
        return out_s, out_i
    dt = Q.dtype
    ld = xs[0].stride(0) if nq else D
    for X in xs:
        assert X.dtype == dt and (X.shape[0] <= 1 or X.stride(0) == ld) and X.stride(-1) == 1

    def ptrs(ts):
        return torch.tensor([t.data_ptr() for t in ts], dtype=torch.int64).pin_memory().to(dev, non_blocking=True)
    nr = torch.tensor([X.shape[0] for X in xs], dtype=torch.int32).pin_memory().to(dev, non_blocking=True)
    return segment_topk_ptrs(ptrs(xs), nr, ld, Q, k, bptr=ptrs(biases) if biases is not None else None,
                             sptr=ptrs(scales) if scales is not None else None, alpha=alpha, qbias=qbias)


def segment_topk_ptrs(xptr: torch.Tensor, nrows: torch.Tensor, ld: int, Q: torch.Tensor, k: int, *,
                      bptr=None, sptr=None, alpha: float = 1.0, qbias=None):
    """Device-side form of :func:`segment_topk`: ``xptr``/``bptr``/``sptr`` are
    int64 device tensors of row / bias / scale base addresses per query and
    ``nrows`` int32 row counts (e.g. gathered from a tenant table with one
    indexing op), so a serving loop builds no Python lists per batch."""
    L = _lib.lib()
    kslot = L.lzk_flat_topk_kslot(int(k))
    if kslot < 0:
        raise ValueError("segment_topk supports k <= 16")
    nq, D = Q.shape
    dev = Q.device
    # the kernel dereferences these tables: a host tensor's address would fault the GPU
    for name, t in (("xptr", xptr), ("nrows", nrows), ("bptr", bptr), ("sptr", sptr), ("qbias", qbias)):
        if t is not None and (t.device != dev or not t.is_contiguous() or t.shape[0] != nq):
            raise ValueError(f"segment_topk_ptrs: {name} must be a contiguous [{nq}] tensor on {dev}, "
                             f"got {tuple(t.shape)} on {t.device}")
    if xptr.dtype != torch.int64 or nrows.dtype != torch.int32:
        raise ValueError("segment_topk_ptrs: xptr int64, nrows int32")
    dt = {torch.bfloat16: 0, torch.float32: 1}[Q.dtype]
    qb = qbias.float().contiguous() if qbias is not None else None
    os_ = torch.empty((nq, k), dtype=torch.float32, device=dev)
    oi = torch.empty((nq, k), dtype=torch.long, device=dev)
    rc = L.lzk_segment_topk(xptr.data_ptr(), nrows.data_ptr(), int(ld), _lib.ptr(bptr), _lib.ptr(sptr), Q.data_ptr(),
                            Q.stride(0), nq, D, dt, float(alpha), _lib.ptr(qb), kslot, int(k), os_.data_ptr(),
                            oi.data_ptr(), _lib.stream_ptr(dev))
    _lib.check(rc, "lzk_segment_topk")
    return os_, oi


def topk_large(X, Q, k, *, bias=None, alpha=1.0, idx_offset=0, chunk=1 << 20):
    """k > 16: per-chunk candidate generation with the fused kernel at k=16
    cannot be exact, so this path scores chunks with the GEMM library and
    keeps a running torch top-k (used only for rerank candidate lists)."""
    nq = Q.shape[0]
    best_s = None
    best_i = None
    for c0 in range(0, X.shape[0], chunk):
        c1 = min(X.shape[0], c0 + chunk)
        s = alpha * (Q.float() @ X[c0:c1].float().T)
        if bias is not None:
            s = s + bias[c0:c1][None, :]
        ts, ti = torch.topk(s, min(k, c1 - c0), dim=1)
        ti = ti + c0
        if best_s is None:
            best_s, best_i = ts, ti
        else:
            cs = torch.cat([best_s, ts], 1)
            ci = torch.cat([best_i, ti], 1)
            best_s, o = torch.topk(cs, min(k, cs.shape[1]), dim=1)
            best_i = torch.gather(ci, 1, o)
    return best_s, best_i + idx_offset


# ---------------------------------------------------------------------------
# Multi-tenant global search (csrc/kernels/mtscan.hip): every query against
# the rows of MANY small tenants in one MFMA pass over a tile table.
_lib.register("lzk_mt_cand", _lib.I, [_lib.P, _lib.P, _lib.P, _lib.I, _lib.L, _lib.P, _lib.L, _lib.I, _lib.I, _lib.F,
                                      _lib.P, _lib.I, _lib.P, _lib.P, _lib.P, _lib.P])
_lib.register("lzk_mt_sample", _lib.I, [_lib.P, _lib.P, _lib.P, _lib.P, _lib.I, _lib.L, _lib.I, _lib.P, _lib.P,
                                        _lib.P])
_lib.register("lzk_mt_rerank", _lib.I, [_lib.P, _lib.L, _lib.I, _lib.P, _lib.I, _lib.I, _lib.I, _lib.P, _lib.P,
                                        _lib.P, _lib.P, _lib.P, _lib.I, _lib.P, _lib.P, _lib.P])
MT_TILE = 256
MT_STRIDE = 64  # the threshold sample: rows 0, 64, 128, 192 of every tile


class MtTiles:
    """Tile table of a set of tenants (host-built, uploaded once per change):
    tile t = rows [row0[t], row0[t] + n[t]) (n <= 256) of tenant slot
    ``slot[t]``; ``x`` / ``b`` the addresses of its first bf16 row / store
    bias entry. ``s_tile`` / ``s_row``: the strided threshold sample."""

    def __init__(self, slots: np.ndarray, nrows: np.ndarray, e16: np.ndarray, bias: np.ndarray, ld16: int,
                 device):
        nrows = np.asarray(nrows, np.int64)
        keep = nrows > 0
        slots, nrows, e16, bias = slots[keep], nrows[keep], e16[keep], bias[keep]
        nt = (nrows + MT_TILE - 1) // MT_TILE
        T = int(nt.sum())
        first = np.repeat(np.cumsum(nt) - nt, nt)
        which = np.repeat(np.arange(slots.size), nt)
        row0 = (np.arange(T) - first) * MT_TILE
        tn = np.minimum(MT_TILE, nrows[which] - row0)
        self.n_tiles = T
        self.ld16 = int(ld16)
        self.rows = int(nrows.sum())
        h_x = e16[which] + row0 * self.ld16 * 2
        h_b = bias[which] + row0 * 4
        # sample rows: every MT_STRIDE-th row of every tile
        per = (tn + MT_STRIDE - 1) // MT_STRIDE
        s_first = np.repeat(np.cumsum(per) - per, per)
        s_tile = np.repeat(np.arange(T), per)
        s_row = (np.arange(int(per.sum())) - s_first) * MT_STRIDE
        self.n_sample = int(s_tile.size)

        def up(a, dt):
            t = torch.from_numpy(np.ascontiguousarray(a, dt))
            return t.pin_memory().to(device, non_blocking=True) if torch.device(device).type == "cuda" else t
        self.x, self.b, self.n = up(h_x, np.int64), up(h_b, np.int64), up(tn, np.int32)
        self.slot, self.row0 = up(slots[which], np.int32), up(row0, np.int32)
        self.s_tile, self.s_row = up(s_tile, np.int32), up(s_row, np.int32)


def _mt_threshold(Xs, bs, Q16, kc, kslot, alpha):
    """Lower bound of each query's kc-th best score: the sample's exact
    kc-th best, lowered by the accumulation-order margin (_sample_threshold)."""
    if Xs.shape[0] < kc:
        return torch.full((Q16.shape[0],), float("-inf"), dtype=torch.float32, device=Q16.device)
    ts, _ = _flat_topk_lane(Xs, Q16, kslot, kslot, bs, None, None, alpha, 0, None)
    thr = ts[:, kc - 1].contiguous()
    return torch.nan_to_num(thr - 2e-4 * (1.0 + thr.abs()), nan=float("-inf"))


def mt_topk(tiles: MtTiles, Q: torch.Tensor, k: int, p_e32: torch.Tensor, p_bias: torch.Tensor,
            p_kind: torch.Tensor, metric: str = "l2"):
    """Every query's top-k over all the table's tenants: store scores (L2:
    -|q-x|^2, ip: <q,x>, + the store bias), bf16 MFMA candidates above a
    sampled lower bound of the 2k-th best, the best 2k (<= 16) of them
    re-scored in fp32 from the tenants' rows. Returns (scores fp32 [nq, k],
    keys int64 [nq, k] = slot << 32 | row, overflow int32 [nq]): a query
    whose candidate list overflowed (ovf = 1) must be recomputed by the
    caller; rows that are not live nodes come back as (-inf, -1)."""
    L = _lib.lib()
    dev = Q.device
    nq, D = Q.shape
    Dp = tiles.ld16
    # 16 bf16 candidates for every k <= 16 (the per-tenant store search's
    # CAND_SLOTS): a bf16 near-tie just past the k-th cannot push the fp32
    # top-k out of the re-ranked set
    if k > 16:
        raise ValueError("mt_topk supports k <= 16")
    kc = 16
    kslot = L.lzk_flat_topk_kslot(int(kc))
    if kslot < 0:
        raise ValueError("mt_topk: no candidate slot count for k = 16")
    st = _lib.stream_ptr(dev)
    Qf = Q.to(dev, torch.float32).contiguous()
    Q16 = torch.zeros((nq, Dp), dtype=torch.bfloat16, device=dev)
    Q16[:, :D] = Qf
    alpha = 2.0 if metric == "l2" else 1.0
    ns = tiles.n_sample
    # 1. threshold: exact top-kc of the sample (a subset: its kc-th best is <=
    #    the whole table's), lowered by the accumulation-order margin
    Xs = torch.empty((ns, Dp), dtype=torch.bfloat16, device=dev)
    bs = torch.empty((ns,), dtype=torch.float32, device=dev)
    _lib.check(L.lzk_mt_sample(tiles.x.data_ptr(), tiles.b.data_ptr(), tiles.s_tile.data_ptr(),
                               tiles.s_row.data_ptr(), ns, Dp, Dp, Xs.data_ptr(), bs.data_ptr(), st), "lzk_mt_sample")
    thr = _mt_threshold(Xs, bs, Q16, kc, kslot, alpha)
    # 2. candidates over every tile
    cap = max(1024, 8 * kslot * MT_STRIDE)
    cnt, cs, ci = _cand_lists(dev, nq, cap, 0)
    _lib.check(L.lzk_mt_cand(tiles.x.data_ptr(), tiles.b.data_ptr(), tiles.n.data_ptr(), tiles.n_tiles, Dp,
                             Q16.data_ptr(), Dp, nq, Dp, float(alpha), thr.data_ptr(), cap, cnt.data_ptr(),
                             cs.data_ptr(), ci.data_ptr(), st), "lzk_mt_cand")
    # 3. best kc by bf16 score, 4. fp32 re-rank to k
    os_ = torch.empty((nq, kc), dtype=torch.float32, device=dev)
    oi = torch.empty((nq, kc), dtype=torch.long, device=dev)
    ovf = torch.empty((nq,), dtype=torch.int32, device=dev)
    _lib.check(L.lzk_cand_select(cnt.data_ptr(), cs.data_ptr(), ci.data_ptr(), cap, nq, kslot, kc, 0,
                                 os_.data_ptr(), oi.data_ptr(), ovf.data_ptr(), None, st), "lzk_cand_select")
    s = torch.empty((nq, k), dtype=torch.float32, device=dev)
    key = torch.empty((nq, k), dtype=torch.long, device=dev)
    _lib.check(L.lzk_mt_rerank(Qf.data_ptr(), D, D, oi.data_ptr(), kc, nq, int(k), tiles.slot.data_ptr(),
                               tiles.row0.data_ptr(), p_e32.data_ptr(), p_bias.data_ptr(), p_kind.data_ptr(),
                               0 if metric == "l2" else 1, s.data_ptr(), key.data_ptr(), st), "lzk_mt_rerank")
    return s, key, ovf
