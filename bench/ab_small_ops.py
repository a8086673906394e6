"""Isolated timings of the encoder's memory-bound kernels at the headline
bench's half-batch shape (512 packed sequences of 12-26 tokens, bge-base):
attention (packed varlen) and residual LayerNorm, with their HBM-traffic
floors at 5 TB/s. Prints one JSON object."""
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from lazzaro_amd.ops import encoder_ops as E  # noqa: E402


def timeit(fn, it=200):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(it):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / it


def main():
    g = torch.Generator().manual_seed(0)
    B, H, nh = 512, 768, 12
    lens = torch.randint(12, 27, (B,), generator=g, dtype=torch.int32)
    T = int(lens.sum())
    cu = torch.zeros(B + 1, dtype=torch.int32)
    cu[1:] = torch.cumsum(lens, 0)
    S = int(lens.max())
    qkv = torch.randn(T, 3 * H, device="cuda").to(torch.bfloat16)
    lens_d, cu_d = lens.cuda(), cu.cuda()
    ta = timeit(lambda: E.attention(qkv, lens_d, B, S, nh, cu=cu_d))
    x = torch.randn(T, H, device="cuda").to(torch.bfloat16)
    r = torch.randn_like(x)
    gam = torch.rand(H, device="cuda") + 0.5
    bet = torch.randn(H, device="cuda")
    tl = timeit(lambda: E.layernorm(x, gam, bet, 1e-12, residual=r))
    bw = 5e12
    out = {"tokens": T, "attention_us": round(ta * 1e6, 2),
           "attention_floor_us": round((T * 3 * H * 2 + T * H * 2) / bw * 1e6, 2),
           "layernorm_us": round(tl * 1e6, 2), "layernorm_floor_us": round(3 * T * H * 2 / bw * 1e6, 2)}
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
