"""Probe: cost of the dual candidate scan vs list B's threshold. Times the
scan (lzk_flat_cand_dual + gather) on consolidation-shaped data with list B
thresholds: the safe sampled shard bound (default), a speculative bound from
the global sample's k'-th best, and list A's own threshold (timing only).
Prints one JSON object with ms and mean list-B candidate counts."""
import json
import os
import statistics
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from lazzaro_amd.ops import _lib  # noqa: E402
from lazzaro_amd.ops import search as S  # noqa: E402


def main():
    n, d, nq, k = 10_000_000, 768, 1024, 3
    dev = "cuda"
    g = torch.Generator(device=dev).manual_seed(0)
    X = torch.empty(n, d, device=dev, dtype=torch.bfloat16)
    for r0 in range(0, n, 1 << 20):
        x = torch.randn(min(1 << 20, n - r0), d, device=dev, generator=g)
        X[r0:r0 + x.shape[0]] = torch.nn.functional.normalize(x, dim=1).to(torch.bfloat16)
    lab = torch.randint(0, 64, (n,), device=dev, dtype=torch.int32, generator=g)
    bias = torch.where(torch.rand(n, device=dev, generator=g) < 0.01, float("-inf"), 0.0)
    base = X[torch.randint(0, n, (nq,), device=dev, generator=g)].float()
    noise = torch.randn(nq, d, device=dev, generator=g) / d ** 0.5
    dup = torch.rand(nq, device=dev, generator=g) < 0.1
    Q = torch.nn.functional.normalize(torch.where(dup[:, None], base + 0.1 * noise, base + 1.2 * noise), dim=1)
    Q = Q.to(torch.bfloat16)
    ql = torch.randint(0, 64, (nq,), device=dev, dtype=torch.int32, generator=g)
    L = _lib.lib()
    kslot = L.lzk_flat_topk_kslot(k)
    Sx = max(1, min(S.CAND_STRIDE, n // max(16 * kslot, 1)))
    thr_a = S._sample_threshold(X, Q, k, kslot, bias, None, None, 1.0, Sx)
    thr_b = S._sample_threshold(X, Q, k, kslot, bias, lab, ql, 1.0, Sx)
    out = {"kslot": kslot, "stride": Sx}
    # global sample's k'-th best (k' = 16): ~16 expected rows of a 1/64 shard above it
    t0 = time.perf_counter()
    ts16, _ = S._flat_topk_lane(X[::Sx], Q, 16, 16, bias[::Sx].contiguous(), None, None, 1.0, 0, None)
    torch.cuda.synchronize()
    out["sample16_ms"] = round((time.perf_counter() - t0) * 1e3, 3)
    spec16 = torch.maximum(thr_b, ts16[:, 15] - 2e-4 * (1 + ts16[:, 15].abs()))
    spec8 = torch.maximum(thr_b, ts16[:, 7] - 2e-4 * (1 + ts16[:, 7].abs()))
    arms = {"safe": thr_b, "spec16": spec16, "spec8": spec8, "a": thr_a}
    cap = max(1024, 8 * kslot * Sx)
    grid = L.lzk_cand_grid(n, nq, 1)
    bbuf, bcap, bcnt = S._blk_records(torch.device(dev), grid, nq, kslot, Sx, 2)
    st = _lib.stream_ptr(torch.device(dev))

    def scan(tb):
        ca = S._cand_lists(torch.device(dev), nq, cap, 0)
        cb = S._cand_lists(torch.device(dev), nq, cap, 1)
        rc = L.lzk_flat_cand_dual(X.data_ptr(), X.stride(0), n, Q.data_ptr(), Q.stride(0), nq, d,
                                  bias.data_ptr(), lab.data_ptr(), ql.data_ptr(), 1.0, thr_a.data_ptr(),
                                  tb.data_ptr(), cap, ca[0].data_ptr(), ca[1].data_ptr(), ca[2].data_ptr(),
                                  cb[0].data_ptr(), cb[1].data_ptr(), cb[2].data_ptr(), bbuf.data_ptr(), bcap,
                                  bcnt.data_ptr(), st)
        _lib.check(rc, "dual")
        _lib.check(L.lzk_cand_gather(bbuf.data_ptr(), bcap, bcnt.data_ptr(), grid, cap, nq, ca[0].data_ptr(),
                                     ca[1].data_ptr(), ca[2].data_ptr(), cb[0].data_ptr(), cb[1].data_ptr(),
                                     cb[2].data_ptr(), st), "gather")
        return cb[0]

    for a, tb in arms.items():
        c = scan(tb).float()
        out[a] = {"b_cnt_mean": round(float(c.mean()), 1), "b_cnt_min": float(c.min()),
                  "b_under_k": int((c < k).sum())}
    ts = {a: [] for a in arms}
    for _ in range(5):
        for a, tb in arms.items():
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(3):
                scan(tb)
            torch.cuda.synchronize()
            ts[a].append((time.perf_counter() - t0) / 3)
    for a, v in ts.items():
        out[a]["scan_ms"] = round(statistics.median(v) * 1e3, 3)
    print(json.dumps(out, indent=1), flush=True)


if __name__ == "__main__":
    main()
