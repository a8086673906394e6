"""Minimal driver for PMC counter runs of the int8 store-search scan: 10M x
768 random unit rows (int8 + row scales, bf16 for the re-score), 1024 random
unit queries, 5 x flat_topk_i8(k=16) with a fixed 0.01 margin (the bench's
error model gives ~0.008 for alpha = 2). Run under rocprofv3 --pmc."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from lazzaro_amd.ops.search import flat_topk_i8, quantize_i8_rows  # noqa: E402


def main():
    n, d, nq = 10_000_000, 768, 1024
    g = torch.Generator(device="cuda").manual_seed(0)
    X16 = torch.empty(n, d, device="cuda", dtype=torch.bfloat16)
    X8 = torch.empty(n, d, device="cuda", dtype=torch.int8)
    rs = torch.empty(n, device="cuda", dtype=torch.float32)
    for r0 in range(0, n, 1 << 20):
        x = torch.randn(min(1 << 20, n - r0), d, device="cuda", generator=g)
        x16 = torch.nn.functional.normalize(x, dim=1).to(torch.bfloat16)
        X16[r0:r0 + x.shape[0]] = x16
        quantize_i8_rows(x16, out=X8[r0:r0 + x.shape[0]], scale_out=rs[r0:r0 + x.shape[0]])
    Q16 = torch.nn.functional.normalize(torch.randn(nq, d, device="cuda", generator=g), dim=1).to(torch.bfloat16)
    Q8, qs = quantize_i8_rows(Q16)
    bias = torch.full((n,), -1.0, device="cuda")  # unit rows: -|x|^2
    margin = torch.full((nq,), 0.01, device="cuda")
    for _ in range(5):
        flat_topk_i8(X8, rs, Q8, qs, X16, Q16, 16, bias=bias, alpha=2.0, margin=margin)
    torch.cuda.synchronize()
    print("done", flush=True)


if __name__ == "__main__":
    main()
