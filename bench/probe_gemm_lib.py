"""Probe: the encoder's hand-written GEMM (lzk_gemm_bias_act) against the
library GEMM (torch -> hipBLASLt) on the bge-base projection shapes, with and
without the fused bias / GELU / residual epilogue. Prints one JSON line."""
import json
import sys

import torch

from lazzaro_amd.ops import encoder_ops as E


def timeit(fn, reps=30):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(reps):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / reps * 1e3  # us


def main():
    dev = torch.device("cuda")
    out = {}
    for T in (22585, 11292):
        for name, K, N, act, res in (("qkv", 768, 2304, "none", False), ("o", 768, 768, "none", True),
                                     ("ffn1", 768, 3072, "gelu", False), ("ffn2", 3072, 768, "none", True)):
            x = torch.randn(T, K, device=dev).to(torch.bfloat16)
            w = (torch.randn(N, K, device=dev) / K ** 0.5).to(torch.bfloat16)
            b = torch.randn(N, device=dev) * 0.1
            r = torch.randn(T, N, device=dev).to(torch.bfloat16) if res else None
            y = torch.empty(T, N, device=dev, dtype=torch.bfloat16)
            b16 = b.to(torch.bfloat16)
            fl = 2.0 * T * K * N
            ours = timeit(lambda: E.linear(x, w, b, act, residual=r, out=y))
            mm = timeit(lambda: torch.matmul(x, w.T, out=y))
            if act == "gelu":
                lib = timeit(lambda: torch._addmm_activation(b16, x, w.T, use_gelu=True))
            elif res:
                lib = timeit(lambda: torch.addmm(b16, x, w.T).add_(r))
            else:
                lib = timeit(lambda: torch.addmm(b16, x, w.T))
            out[f"{name}_T{T}"] = {"ours_us": round(ours, 1), "lib_matmul_us": round(mm, 1),
                                   "lib_fused_us": round(lib, 1),
                                   "ours_tflops": round(fl / ours / 1e6, 1), "lib_matmul_tflops": round(fl / mm / 1e6, 1)}
            print(name, T, out[f"{name}_T{T}"], file=sys.stderr, flush=True)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
