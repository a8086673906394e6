"""A/B of the tile staging variants (register vs LDS-DMA) in ONE process,
interleaved rounds (cdna guide §5.4 rule 24): flat top-k on N x 768 at Q=1024
and the bge-base encoder GEMM shapes."""
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
from lazzaro_amd.ops.search import _ref_topk, flat_topk  # noqa: E402

L = _lib.lib()
L.lzk_set_staging.argtypes = [ctypes.c_int]
L.lzk_set_search_staging.argtypes = [ctypes.c_int]


def setv(g):
    L.lzk_set_staging(g)
    L.lzk_set_search_staging(g)


def timeit(fn, it=5):
    fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(it):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / it


def main():
    n = int(os.environ.get("AB_ROWS", "10000000"))
    dev = "cuda"
    # correctness of both variants
    Xs = torch.randn(20000, 768, device=dev).to(torch.bfloat16)
    Qs = torch.randn(300, 768, device=dev).to(torch.bfloat16)
    b = torch.randn(20000, device=dev)
    rs, ri = _ref_topk(Xs.cpu(), Qs.cpu(), 10, b.cpu(), None, None, 2.0)
    ok = {}
    for g in (0, 1):
        setv(g)
        s, i = flat_topk(Xs, Qs, 10, bias=b, alpha=2.0)
        ok[g] = bool(torch.allclose(s.cpu(), rs, atol=2e-3) and (i.cpu() == ri).float().mean() > 0.995)
        w = (torch.randn(2304, 768, device=dev) * 0.05).to(torch.bfloat16)
        x = torch.randn(1000, 768, device=dev).to(torch.bfloat16)
        bb = torch.randn(2304, device=dev)
        y = E.linear(x, w, bb)
        yr = E.linear(x.cpu(), w.cpu(), bb.cpu())
        ok[g] = ok[g] and float(((y.cpu().float() - yr.float()).norm() / yr.float().norm())) < 1e-2
    X = torch.randn(n, 768, device=dev).to(torch.bfloat16)
    Q = torch.randn(1024, 768, device=dev).to(torch.bfloat16)
    T = 32768
    x768 = torch.randn(T, 768, device=dev).to(torch.bfloat16)
    x3072 = torch.randn(T, 3072, device=dev).to(torch.bfloat16)
    shapes = {"qkv": (x768, (torch.randn(2304, 768, device=dev) * 0.02).to(torch.bfloat16), "none"),
              "ffn1": (x768, (torch.randn(3072, 768, device=dev) * 0.02).to(torch.bfloat16), "gelu"),
              "ffn2": (x3072, (torch.randn(768, 3072, device=dev) * 0.02).to(torch.bfloat16), "none")}
    res = {g: {"search": [], **{k: [] for k in shapes}} for g in (0, 1)}
    for rnd in range(4):
        for g in (0, 1):
            setv(g)
            res[g]["search"].append(timeit(lambda: flat_topk(X, Q, 10), 3))
            for k, (x, w, act) in shapes.items():
                bias = torch.zeros(w.shape[0], device=dev)
                res[g][k].append(timeit(lambda: E.linear(x, w, bias, act=act), 10))
    out = {"correct": ok, "rows": n}
    for g in (0, 1):
        name = "glds" if g else "register"
        d = {}
        for k, v in res[g].items():
            med = statistics.median(v)
            if k == "search":
                fl = 2.0 * n * 768 * 1024
            else:
                x, w, _ = shapes[k]
                fl = 2.0 * x.shape[0] * x.shape[1] * w.shape[0]
            d[k] = {"ms_median": round(med * 1e3, 3), "ms_min": round(min(v) * 1e3, 3),
                    "tflops": round(fl / med / 1e12, 1)}
        out[name] = d
    print(json.dumps(out, indent=1), flush=True)


if __name__ == "__main__":
    main()
