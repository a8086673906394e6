"""Ceiling probe for the flat-search GEMM: the vendor GEMM (torch.matmul ->
hipBLASLt) on the same 10M x 768 x 1024 bf16 shape, chunked so the fp32 /
bf16 score matrix fits, against the fused candidate kernel. Random data (the
chip's clock under load depends on operand values). Prints one JSON line."""
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from lazzaro_amd.ops.search import flat_topk  # noqa: E402


def timeit(fn, reps=5):
    fn()
    torch.cuda.synchronize()
    ts = []
    for _ in range(reps):
        t0 = time.perf_counter()
        fn()
        torch.cuda.synchronize()
        ts.append(time.perf_counter() - t0)
    ts.sort()
    return ts[len(ts) // 2]


def main():
    n = int(os.environ.get("P_ROWS", "10000000"))
    d = int(os.environ.get("P_DIM", "768"))
    nq = int(os.environ.get("P_Q", "1024"))
    dev = "cuda"
    g = torch.Generator(device=dev).manual_seed(0)
    X = (torch.randn(n, d, device=dev, generator=g, dtype=torch.bfloat16) * 0.036)
    Q = torch.nn.functional.normalize(torch.randn(nq, d, device=dev, generator=g), dim=1).to(torch.bfloat16)
    flop = 2.0 * n * d * nq
    out = {"rows": n, "dim": d, "nq": nq}
    chunk = 1 << 20
    C = torch.empty(chunk, nq, device=dev, dtype=torch.bfloat16)

    def lib_gemm():
        for r0 in range(0, n, chunk):
            r1 = min(n, r0 + chunk)
            torch.matmul(X[r0:r1], Q.T, out=C[: r1 - r0])
    t = timeit(lib_gemm)
    out["hipblaslt_bf16_out_ms"] = round(t * 1e3, 3)
    out["hipblaslt_tflops"] = round(flop / t / 1e12, 1)
    t = timeit(lambda: flat_topk(X, Q, 10))
    out["flat_topk_ms"] = round(t * 1e3, 3)
    out["flat_topk_tflops"] = round(flop / t / 1e12, 1)
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
