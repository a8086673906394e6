"""Minimal driver for PMC counter runs of the headline search kernel:
10M x 768 bf16 random index, 1024 random unit queries, 5 x flat_topk(k=10).
Run under rocprofv3 --pmc (one counter group per run)."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from lazzaro_amd.ops.search import flat_topk  # noqa: E402


def main():
    n, d, nq = 10_000_000, 768, 1024
    g = torch.Generator(device="cuda").manual_seed(0)
    X = torch.empty(n, d, device="cuda", dtype=torch.bfloat16)
    for r0 in range(0, n, 1 << 20):
        x = torch.randn(min(1 << 20, n - r0), d, device="cuda", generator=g)
        X[r0:r0 + x.shape[0]] = torch.nn.functional.normalize(x, dim=1).to(torch.bfloat16)
    Q = torch.nn.functional.normalize(torch.randn(nq, d, device="cuda", generator=g), dim=1).to(torch.bfloat16)
    for _ in range(5):
        flat_topk(X, Q, 10)
    torch.cuda.synchronize()
    print("done", flush=True)


if __name__ == "__main__":
    main()
