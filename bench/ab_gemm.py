"""A/B of the encoder GEMM tiles in ONE process, interleaved rounds: 128x128
(4 waves, 2 blocks/CU) vs 256x256 (8 waves, counted-vmcnt pipeline) on the
bge-base / e5-large projection shapes at 32k tokens."""
import ctypes
import json
import os
import statistics
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from lazzaro_amd.ops import _lib  # noqa: E402
from lazzaro_amd.ops import encoder_ops as E  # noqa: E402

L = _lib.lib()
L.lzk_set_gemm_tile.argtypes = [ctypes.c_int]


def timeit(fn, it=10):
    fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(it):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / it


def main():
    T = int(os.environ.get("AB_TOKENS", "32768"))
    dev = "cuda"
    shapes = {"qkv": (2304, 768, "none", False), "o": (768, 768, "none", True), "ffn1": (3072, 768, "gelu", False),
              "ffn2": (768, 3072, "none", True), "e5_qkv": (3072, 1024, "none", False),
              "e5_ffn1": (4096, 1024, "gelu", False), "e5_ffn2": (1024, 4096, "none", True)}
    out = {"tokens": T}
    for name, (N, K, act, res) in shapes.items():
        x = torch.randn(T, K, device=dev).to(torch.bfloat16)
        w = (torch.randn(N, K, device=dev) * 0.05).to(torch.bfloat16)
        b = torch.randn(N, device=dev)
        r = torch.randn(T, N, device=dev).to(torch.bfloat16) if res else None
        ys = {}
        for tile in (128, 256):
            L.lzk_set_gemm_tile(tile)
            ys[tile] = E.linear(x, w, b, act=act, residual=r).float()
        diff = float((ys[128] - ys[256]).norm() / ys[128].norm())
        ts = {128: [], 256: []}
        for _ in range(5):
            for tile in (128, 256):
                L.lzk_set_gemm_tile(tile)
                ts[tile].append(timeit(lambda: E.linear(x, w, b, act=act, residual=r)))
        flop = 2.0 * T * N * K
        out[name] = {"rel_diff": diff}
        for tile, v in ts.items():
            m = statistics.median(v)
            out[name][str(tile)] = {"us": round(m * 1e6, 1), "tflops": round(flop / m / 1e12, 1)}
        # main loop only (epilogue skipped; measurement probe, act=9)
        if N >= 1024:
            L.lzk_set_gemm_tile(256)
            y9 = torch.empty((T, N), dtype=torch.bfloat16, device=dev)

            def probe():
                L.lzk_gemm_bias_act(x.data_ptr(), x.stride(0), T, w.data_ptr(), w.stride(0), N, b.data_ptr(), None,
                                    0, y9.data_ptr(), y9.stride(0), K, 9, _lib.stream_ptr(x.device))
            tp = statistics.median(timeit(probe) for _ in range(5))
            out[name]["256_mainloop_only_us"] = round(tp * 1e6, 1)

            def probe_nostore():
                L.lzk_gemm_bias_act(x.data_ptr(), x.stride(0), T, w.data_ptr(), w.stride(0), N, b.data_ptr(), None,
                                    0, y9.data_ptr(), y9.stride(0), K, 10, _lib.stream_ptr(x.device))
            tn = statistics.median(timeit(probe_nostore) for _ in range(5))
            out[name]["256_no_global_store_us"] = round(tn * 1e6, 1)
        # fp8 e4m3 (K % 128 == 0): GEMM alone and with the activation quantisation pass
        xq, sx = E.quantize_fp8_rows(x)
        wq, sw = E.quantize_fp8_rows(w)
        y8 = E.linear_fp8(xq, sx, wq, sw, b, act=act, residual=r).float()
        t8 = statistics.median(timeit(lambda: E.linear_fp8(xq, sx, wq, sw, b, act=act, residual=r)) for _ in range(5))
        tq = statistics.median(timeit(lambda: E.quantize_fp8_rows(x)) for _ in range(5))
        out[name]["fp8"] = {"us": round(t8 * 1e6, 1), "tflops": round(flop / t8 / 1e12, 1),
                            "quant_us": round(tq * 1e6, 1),
                            "rel_err_vs_bf16": round(float((y8 - ys[256]).norm() / ys[256].norm()), 4)}
    print(json.dumps(out, indent=1), flush=True)


if __name__ == "__main__":
    main()
