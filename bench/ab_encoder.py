"""Encoder GEMM anatomy on the headline's token counts (1024 synthetic queries
-> 22,585 packed tokens; 11,292 per sub-batch with two streams): per
projection shape the full kernel, the main loop alone (act=9 probe) and
everything but the global store (act=10 probe), plus the whole bge-base
forward on 1 and 2 streams. One process, interleaved repetitions, medians.
Usage: python bench/ab_encoder.py [out.json]"""
import json
import os
import random
import statistics
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from lazzaro_amd.ops import _lib  # noqa: E402
from lazzaro_amd.ops import encoder_ops as E  # noqa: E402


def timeit(fn, it=20):
    fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(it):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / it


def med(fn, reps=5, it=20):
    return statistics.median(timeit(fn, it) for _ in range(reps))


def main():
    dev = torch.device("cuda", 0)
    L = _lib.lib()
    st = _lib.stream_ptr(dev)
    shapes = {"qkv": (2304, 768, "none", False), "o": (768, 768, "none", True), "ffn1": (3072, 768, "gelu", False),
              "ffn2": (768, 3072, "none", True)}
    out = {}
    for T in [int(t) for t in os.environ.get("AB_TOKENS", "22585,11292").split(",")]:
        for name, (N, K, act, res) in shapes.items():
            x = torch.randn(T, K, device=dev).to(torch.bfloat16)
            w = (torch.randn(N, K, device=dev) * 0.05).to(torch.bfloat16)
            b = torch.randn(N, device=dev)
            r = torch.randn(T, N, device=dev).to(torch.bfloat16) if res else None
            y = torch.empty((T, N), dtype=torch.bfloat16, device=dev)
            ref = (x.float() @ w.float().T + b)
            if act == "gelu":
                ref = torch.nn.functional.gelu(ref)
            if r is not None:
                ref = ref + r.float()
            got = E.linear(x, w, b, act=act, residual=r, out=y).float()
            rel = float((got - ref).norm() / ref.norm())

            def probe(a):
                def f():
                    L.lzk_gemm_bias_act(x.data_ptr(), x.stride(0), T, w.data_ptr(), w.stride(0), N, b.data_ptr(),
                                        None, 0, y.data_ptr(), y.stride(0), K, a, st)
                return f
            full = med(lambda: E.linear(x, w, b, act=act, residual=r, out=y))
            flop = 2.0 * T * N * K
            rec = {"rel_err": round(rel, 5), "us": round(full * 1e6, 1), "tflops": round(flop / full / 1e12, 1),
                   "mainloop_only_us": round(med(probe(9)) * 1e6, 1),
                   "no_global_store_us": round(med(probe(10)) * 1e6, 1)}
            out[f"{name}_T{T}"] = rec
            print(name, T, rec, flush=True)
    from lazzaro_amd.core.embedders import OnDeviceEmbedder
    import bench
    emb = OnDeviceEmbedder("bge-base", device=dev, max_len=64)
    texts = bench.synth_texts(1024, random.Random(1234))
    ids, lens = emb.tok.encode_batch(texts, emb.max_len)
    out["tokens"] = int(lens.sum())
    fw = {}
    for parts in (1, 2):
        fw[str(parts)] = round(med(lambda: emb.encoder.forward_streams(ids, lens, pad_to=768, parts=parts),
                                   reps=5, it=10) * 1e3, 3)
    out["forward_ms"] = fw
    print(json.dumps(out, indent=1), flush=True)
    if len(sys.argv) > 1:
        with open(sys.argv[1], "w") as f:
            json.dump(out, f, indent=1)


if __name__ == "__main__":
    main()
