"""A/B of one k-means pass at buffer scale (12.5M x 768, 4096 centroids):
assign = flat_topk(k=1) on the 128x128 lane kernel vs the 256x256 flat_top1
argmax kernel; centroid update (K8) = per-element fp32 atomics vs sort + one
workgroup per cluster (lzk_seg_sum_sorted). Prints one JSON line."""
from __future__ import annotations

import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from lazzaro_amd.index.kmeans import assign  # noqa: E402
from lazzaro_amd.ops import graph_ops as G  # noqa: E402


def timed(fn, reps=5):
    fn()
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(reps):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t) / reps * 1e3


def main(n=12_500_000, D=768, C=4096):
    dev = torch.device("cuda", 0)
    g = torch.Generator(device=dev).manual_seed(0)
    X = torch.empty((n, D), dtype=torch.bfloat16, device=dev)
    for r0 in range(0, n, 1 << 21):
        x = torch.randn((min(1 << 21, n - r0), D), device=dev, generator=g)
        X[r0:r0 + x.shape[0]] = torch.nn.functional.normalize(x, dim=1).to(torch.bfloat16)
    C16 = X[torch.randperm(n, device=dev, generator=g)[:C]].contiguous()
    lab, _ = assign(X, C16)
    import lazzaro_amd.index.kmeans as K
    out = {"n": n, "D": D, "C": C}
    for mode in ("lane", "top1"):
        K.ASSIGN = mode
        out[f"assign_{mode}_ms"] = round(timed(lambda: assign(X, C16), 3), 2)
        out[f"assign_{mode}_pflops"] = round(2.0 * n * C * D / (out[f"assign_{mode}_ms"] * 1e-3) / 1e15, 3)
    K.ASSIGN = "lane"
    la, _ = assign(X, C16)
    K.ASSIGN = "top1"
    lb, _ = assign(X, C16)
    out["assign_label_agreement"] = float((la == lb).float().mean())
    res = {}
    for atomic in (True, False):
        G.SEG_SUM_ATOMIC = atomic
        res[atomic] = G.centroids(X, lab, C, normalize=False)
        out["update_atomic_ms" if atomic else "update_sorted_ms"] = round(
            timed(lambda: G.centroids(X, lab, C, normalize=False)), 2)
    G.SEG_SUM_ATOMIC = False
    a, b = res[True], res[False]
    out["counts_equal"] = bool(torch.equal(a[2], b[2]))
    out["max_abs_diff_mean"] = float((a[0] - b[0]).abs().max())
    out["sorted_GBps"] = round(n * D * 2 / (out["update_sorted_ms"] * 1e-3) / 1e9, 1)
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
