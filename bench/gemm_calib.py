"""Calibration: the vendor library's (hipBLASLt via torch.matmul) bf16 rate on
the search scan's GEMM shape (rows x 768 @ 768 x 1024) and on a large square
GEMM, next to our fused scan kernel at 10M rows (JSON line)."""
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def rate(fn, flop, n=10):
    fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(n):
        fn()
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / n
    return {"ms": round(dt * 1e3, 3), "tflops": round(flop / dt / 1e12, 1)}


def main():
    dev = torch.device("cuda", 0)
    out = {}
    for rows in (1 << 20, 1 << 22):
        X = torch.randn(rows, 768, device=dev, dtype=torch.bfloat16)
        Q = torch.randn(1024, 768, device=dev, dtype=torch.bfloat16)
        out[f"hipblaslt_{rows}x768x1024"] = rate(lambda: X @ Q.T, 2.0 * rows * 768 * 1024)
        del X
    A = torch.randn(8192, 8192, device=dev, dtype=torch.bfloat16)
    out["hipblaslt_8192^3"] = rate(lambda: A @ A, 2.0 * 8192 ** 3)
    del A
    from lazzaro_amd.ops.search import flat_topk
    N = 10_000_000
    X = torch.randn(N, 768, device=dev, dtype=torch.bfloat16)
    Q = torch.randn(1024, 768, device=dev, dtype=torch.bfloat16)
    bias = torch.zeros(N, device=dev)
    out["flat_topk_10M_k16"] = rate(lambda: flat_topk(X, Q, 16, bias=bias, alpha=2.0), 2.0 * N * 768 * 1024, n=5)
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
