"""A/B of the two 256x256 main loops of lzk_g256.h (four-phase `body` vs
two-phase `body2`) in ONE process, interleaved rounds: the encoder projection
GEMMs that take the 256 path (N >= 1024) at the headline bench's token counts,
and the whole bge-base forward of the bench batch. Prints one JSON object."""
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
L.lzk_set_g256_body.argtypes = [ctypes.c_int]
L.lzk_set_g256_min_n.argtypes = [ctypes.c_int]
L.lzk_set_g256_min_tiles.argtypes = [ctypes.c_int]


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
    out = {}
    for T in (11264, 22528):
        for name, (N, K, act) in {"qkv": (2304, 768, "none"), "ffn1": (3072, 768, "gelu"),
                                  "o": (768, 768, "none"), "ffn2": (768, 3072, "none")}.items():
            x = torch.randn(T, K, device=dev).to(torch.bfloat16)
            w = (torch.randn(N, K, device=dev) * 0.05).to(torch.bfloat16)
            b = torch.randn(N, device=dev)
            ys, ts = {}, {0: [], 1: []}
            L.lzk_set_g256_min_tiles(1)
            L.lzk_set_g256_min_n(N)  # arm 1 = two-phase 256x256; arm 0 = four-phase (N >= 1024) / 128x128 (N = 768)
            for bd in (0, 1):
                L.lzk_set_g256_body(bd)
                L.lzk_set_g256_min_n(N if bd else 1024)
                ys[bd] = E.linear(x, w, b, act=act).float()
            for _ in range(5):
                for bd in (0, 1):
                    L.lzk_set_g256_body(bd)
                    L.lzk_set_g256_min_n(N if bd else 1024)
                    ts[bd].append(timeit(lambda: E.linear(x, w, b, act=act)))
            flop = 2.0 * T * N * K
            r = {"rel_diff": float((ys[0] - ys[1]).norm() / ys[0].norm())}
            for bd, v in ts.items():
                m = statistics.median(v)
                r[f"body{bd}"] = {"us": round(m * 1e6, 1), "tflops": round(flop / m / 1e12, 1)}
            out[f"{name}_T{T}"] = r
    # whole forward of the bench batch (bge-base, 1024 synthetic queries, two streams)
    sys.path.insert(0, ROOT)
    import bench as B
    from lazzaro_amd.core.embedders import OnDeviceEmbedder
    emb = OnDeviceEmbedder("bge-base", device=torch.device(dev), max_len=64, seed=0)
    texts = B.synth_texts(1024, random.Random(1234))
    ids, lens = emb.tok.encode_batch(texts, emb.max_len)
    # arms: (main loop, smallest N on the 256 path, sub-batch streams)
    # arms: (main loop, smallest N on the 256 path, smallest grid on it, sub-batch streams)
    arms = {"body0": (0, 1024, 256, 2), "body1": (1, 1024, 256, 2), "body1_n768_t128": (1, 768, 128, 2),
            "body1_t128": (1, 1024, 128, 2), "body1_n768_t128_3s": (1, 768, 128, 3),
            "body1_n768_t64_4s": (1, 768, 64, 4), "body1_n768_1s": (1, 768, 256, 1)}
    ts = {a: [] for a in arms}
    for _ in range(5):
        for a, (bd, mn, mt, parts) in arms.items():
            L.lzk_set_g256_body(bd)
            L.lzk_set_g256_min_n(mn)
            L.lzk_set_g256_min_tiles(mt)
            ts[a].append(timeit(lambda: emb.encoder.forward_streams(ids, lens, pad_to=768, parts=parts), it=5))
    out["embed_forward_ms"] = {a: round(statistics.median(v) * 1e3, 3) for a, v in ts.items()}
    L.lzk_set_g256_body(-1)
    L.lzk_set_g256_min_n(-1)
    L.lzk_set_g256_min_tiles(-1)
    print(json.dumps(out, indent=1), flush=True)


if __name__ == "__main__":
    main()
