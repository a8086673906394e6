"""A/B of the persistent 256x256 encoder GEMM (gemm256p_kernel) against the
one-tile-per-block kernel
at the headline bench's token count, per projection and for the whole
bge-base forward (1 vs 2 sub-batch streams). Interleaved rounds, one process.
Prints one JSON object."""
import ctypes
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

L = _lib.lib()
L.lzk_set_g256_persist.argtypes = [ctypes.c_int]
TAILS = [int(v) for v in os.environ.get("AB_PERSIST", "0,1").split(",")]


def timeit(fn, it=10):
    fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(it):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / it


def main():
    dev = "cuda"
    out = {"persist": TAILS}
    for T in (22585, 11292):
        for name, (N, K, act, res) in {"qkv": (2304, 768, "none", False), "ffn1": (3072, 768, "gelu", False),
                                       "o": (768, 768, "none", True), "ffn2": (768, 3072, "none", True)}.items():
            x = torch.randn(T, K, device=dev).to(torch.bfloat16)
            w = (torch.randn(N, K, device=dev) * 0.05).to(torch.bfloat16)
            b = torch.randn(N, device=dev)
            r = torch.randn(T, N, device=dev).to(torch.bfloat16) if res else None
            ref = (x.float() @ w.float().T + b)
            if act == "gelu":
                ref = torch.nn.functional.gelu(ref)
            if res:
                ref = ref + r.float()
            rec = {}
            ts = {t: [] for t in TAILS}
            for t in TAILS:
                L.lzk_set_g256_persist(t)
                y = E.linear(x, w, b, act=act, residual=r).float()
                rec[f"rel_err_{t}"] = float((y - ref).norm() / ref.norm())
            for _ in range(5):
                for t in TAILS:
                    L.lzk_set_g256_persist(t)
                    ts[t].append(timeit(lambda: E.linear(x, w, b, act=act, residual=r)))
            flop = 2.0 * T * N * K
            for t, v in ts.items():
                m = statistics.median(v)
                rec[f"persist{t}"] = {"us": round(m * 1e6, 1), "tflops": round(flop / m / 1e12, 1)}
            out[f"{name}_T{T}"] = rec
            print(json.dumps({f"{name}_T{T}": rec}), flush=True)
    import bench as B
    from lazzaro_amd.core.embedders import OnDeviceEmbedder
    emb = OnDeviceEmbedder("bge-base", device=torch.device(dev), max_len=64, seed=0)
    texts = B.synth_texts(1024, random.Random(1234))
    ids, lens = emb.tok.encode_batch(texts, emb.max_len)
    arms = {f"persist{t}_{p}s": (t, p) for t in TAILS for p in (1, 2)}
    ts = {a: [] for a in arms}
    for _ in range(5):
        for a, (t, parts) in arms.items():
            L.lzk_set_g256_persist(t)
            ts[a].append(timeit(lambda: emb.encoder.forward_streams(ids, lens, pad_to=768, parts=parts), it=5))
    out["embed_forward_ms"] = {a: round(statistics.median(v) * 1e3, 3) for a, v in ts.items()}
    L.lzk_set_g256_persist(-1)
    print(json.dumps(out, indent=1), flush=True)


if __name__ == "__main__":
    main()
