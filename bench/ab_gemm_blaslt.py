"""A/B: the encoder's hand-written 256x256 projection GEMM (lzk_gemm_bias_act)
vs hipBLASLt (torch.nn.functional.linear, bias fused) on the bge-base layer
shapes at the bench's packed token counts (1024 queries x ~22 real tokens =
~22.6k tokens, and the 2-stream half batch). Interleaved rounds, median ms
and TF/s per (shape, backend). JSON on stdout."""
import json
import os
import statistics
import sys
import time

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from lazzaro_amd.ops import encoder_ops as E  # noqa: E402


def timeit(fn, it=20):
    fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(it):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / it * 1e3


def main():
    dev = torch.device("cuda", 0)
    g = torch.Generator(device=dev).manual_seed(0)
    shapes = {"qkv": (768, 2304), "o": (768, 768), "ffn1": (768, 3072), "ffn2": (3072, 768)}
    out = {}
    for T in (22592, 11296):
        for name, (K, N) in shapes.items():
            x = (torch.randn(T, K, device=dev, generator=g) * 0.5).to(torch.bfloat16)
            w = (torch.randn(N, K, device=dev, generator=g) * 0.02).to(torch.bfloat16)
            b = torch.randn(N, device=dev, generator=g) * 0.1
            b16 = b.to(torch.bfloat16)
            act = "gelu" if name == "ffn1" else "none"
            ours = lambda: E.linear(x, w, b, act=act)  # noqa: E731
            blt = (lambda: F.gelu(F.linear(x, w, b16))) if act == "gelu" else (lambda: F.linear(x, w, b16))
            ta, tb = [], []
            for _ in range(5):
                ta.append(timeit(ours))
                tb.append(timeit(blt))
            fl = 2.0 * T * K * N
            ma, mb = statistics.median(ta), statistics.median(tb)
            ya, yb = ours().float(), blt().float()
            out[f"{name}_T{T}"] = {"ours_ms": round(ma, 4), "hipblaslt_ms": round(mb, 4),
                                   "ours_tflops": round(fl / ma / 1e9, 1), "hipblaslt_tflops": round(fl / mb / 1e9, 1),
                                   "max_abs_diff": float((ya - yb).abs().max())}
            print(name, T, out[f"{name}_T{T}"], flush=True)
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
