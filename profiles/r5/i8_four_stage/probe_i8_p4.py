"""Probe: the int8 candidate scan's four-stage 64-B pipeline (lzk_g256.h
body4, OPT bit 6) against the default two-phase body2, on the headline shape
(10M x 768 rows, 1024 queries): time with the store search's thresholds,
+inf thresholds and without the epilogue, and the candidate lists of both
schedules compared record for record. Prints one JSON line."""
import ctypes
import json
import sys

import torch

from lazzaro_amd.ops import _lib
from lazzaro_amd.ops import search as S


def timeit(fn, reps=5):
    fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(reps):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / reps


def main():
    dev = torch.device("cuda")
    N, D, nq, k = int(sys.argv[1]) if len(sys.argv) > 1 else 10_000_000, 768, 1024, 10
    gen = torch.Generator(device=dev).manual_seed(3)
    X16 = torch.empty((N, D), dtype=torch.bfloat16, device=dev)
    X8 = torch.empty((N, D), dtype=torch.int8, device=dev)
    rs = torch.empty(N, dtype=torch.float32, device=dev)
    ch = 1 << 20
    for a in range(0, N, ch):
        x = torch.randn((min(ch, N - a), D), device=dev, generator=gen)
        x /= x.norm(dim=1, keepdim=True)
        X16[a:a + x.shape[0]] = x.to(torch.bfloat16)
        q8, s8 = S.quantize_i8_rows(X16[a:a + x.shape[0]])
        X8[a:a + x.shape[0]] = q8
        rs[a:a + x.shape[0]] = s8
    Q = torch.randn((nq, D), device=dev, generator=gen)
    Q16 = (Q / Q.norm(dim=1, keepdim=True)).to(torch.bfloat16)
    Q8, qs = S.quantize_i8_rows(Q16)
    bias = torch.zeros(N, dtype=torch.float32, device=dev)
    L = _lib.lib()
    L.lzk_set_i8_opt.argtypes = [ctypes.c_int]
    kslot = L.lzk_flat_topk_kslot(k)
    Ss = max(1, min(S.CAND_STRIDE, N // max(16 * kslot, 1)))
    thr = (S._sample_threshold(X16, Q16, k, kslot, bias, None, None, 2.0, Ss) - 0.01).contiguous()
    inf = torch.full_like(thr, float("inf"))
    cap = max(2048, 16 * kslot * Ss)
    grid = L.lzk_cand_grid_f8(N, nq)
    out = {"shape": [N, D, nq], "grid": grid}
    st = _lib.stream_ptr(dev)
    lists = {}
    for name, th in (("thr", thr), ("noncand", inf)):
        for opt in (24, 88, 28, 92):
            if name == "noncand" and opt in (28, 92):
                continue
            L.lzk_set_i8_opt(opt)
            cnt, cs, ci = S._cand_lists(dev, nq, cap, 0)
            bbuf, bcap, bcnt = S._blk_records(dev, grid, nq, kslot, 2 * Ss, 1)

            def run():
                cnt.zero_()
                _lib.check(L.lzk_flat_cand_i8(X8.data_ptr(), X8.stride(0), N, Q8.data_ptr(), Q8.stride(0), nq, D,
                                              bias.data_ptr(), rs.data_ptr(), qs.data_ptr(), 2.0, th.data_ptr(), cap,
                                              cnt.data_ptr(), cs.data_ptr(), ci.data_ptr(), bbuf.data_ptr(), bcap,
                                              bcnt.data_ptr(), st), "flat_cand_i8")
            ms = timeit(run)
            out[f"{name}_opt{opt}_ms"] = round(ms, 3)
            out[f"{name}_opt{opt}_pops"] = round(2.0 * N * D * nq / ms / 1e12, 3)
            if name == "thr" and opt in (24, 88):
                run()
                torch.cuda.synchronize()
                c = (cnt & 0x3FFFFFFF).clamp_max(cap)
                n = int(c.max())
                rows = ci.view(nq, cap)[:, :n].clone()
                sc = cs.view(nq, cap)[:, :n].clone()
                mask = torch.arange(n, device=dev)[None, :] < c[:, None]
                rows = torch.where(mask, rows, -1)
                o = torch.argsort(rows, dim=1)
                lists[opt] = (c, torch.gather(rows, 1, o), torch.where(mask, sc, 0.0).gather(1, o))
            print(name, opt, ms, file=sys.stderr, flush=True)
    L.lzk_set_i8_opt(-1)
    c0, r0, s0 = lists[24]
    c1, r1, s1 = lists[88]
    out["counts_equal"] = bool(torch.equal(c0, c1))
    out["rows_equal"] = bool(torch.equal(r0, r1))
    out["scores_equal"] = bool(torch.equal(s0, s1))
    out["mean_candidates"] = round(float(c0.float().mean()), 1)
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
