"""A/B of the two exact flat top-k paths in ONE process, interleaved rounds:
the per-lane running top-K kernel (search.hip, 128x128 tile) vs the sampled
threshold + 256x256 candidate pipeline (search256.hip). Same inputs, results
compared for equality. Prints one JSON object."""
import json
import os
import statistics
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from lazzaro_amd.ops import search as S  # noqa: E402


import ctypes  # noqa: E402

from lazzaro_amd.ops import _lib  # noqa: E402

_L = _lib.lib()
_L.lzk_set_cand_persist.argtypes = [ctypes.c_int]
_L.lzk_set_g256_opt.argtypes = [ctypes.c_int]
VARIANTS = os.environ.get("AB_VARIANTS", "lane,cand,cand_p").split(",")


def run(path, X, Q, k, bias):
    if path.startswith("cand"):
        _L.lzk_set_cand_persist(0 if path == "cand" else 1)
        _L.lzk_set_g256_opt(int(path[len("cand_p"):]) if path.startswith("cand_p") and len(path) > 6 else 0)
        path = "cand"
    os.environ["LZK_SEARCH"] = path
    return S.flat_topk(X, Q, k, bias=bias, alpha=2.0 if bias is not None else 1.0)


def main():
    n = int(os.environ.get("AB_ROWS", "10000000"))
    d = int(os.environ.get("AB_DIM", "768"))
    nq = int(os.environ.get("AB_Q", "1024"))
    k = 10
    dev = "cuda"
    g = torch.Generator(device=dev).manual_seed(0)
    X = torch.empty(n, d, device=dev, dtype=torch.bfloat16)
    for r0 in range(0, n, 1 << 20):
        x = torch.randn(min(1 << 20, n - r0), d, device=dev, generator=g)
        X[r0:r0 + x.shape[0]] = torch.nn.functional.normalize(x, dim=1).to(torch.bfloat16)
    Q = torch.nn.functional.normalize(torch.randn(nq, d, device=dev, generator=g), dim=1).to(torch.bfloat16)
    out = {"rows": n, "dim": d, "nq": nq, "k": k}
    for name, bias in (("ip", None), ("l2", -(X.float() ** 2).sum(1) if n <= 2_000_000 else None)):
        if bias is None and name == "l2":
            # |x|^2 in chunks to bound memory
            bias = torch.empty(n, device=dev)
            for r0 in range(0, n, 1 << 20):
                bias[r0:r0 + (1 << 20)] = -(X[r0:r0 + (1 << 20)].float() ** 2).sum(1)
        base_s, base_i = run(VARIANTS[0], X, Q, k, bias)
        same, maxdiff = {}, {}
        for v in VARIANTS[1:]:
            sv, iv = run(v, X, Q, k, bias)
            same[v] = float((iv == base_i).float().mean())
            maxdiff[v] = float((sv - base_s).abs().max())
        torch.cuda.synchronize()
        times = {v: [] for v in VARIANTS}
        for _ in range(5):
            for p in VARIANTS:
                torch.cuda.synchronize()
                t0 = time.perf_counter()
                for _ in range(3):
                    run(p, X, Q, k, bias)
                torch.cuda.synchronize()
                times[p].append((time.perf_counter() - t0) / 3)
        flop = 2.0 * n * d * nq
        res = {"ids_equal_frac": same, "score_maxdiff": maxdiff}
        for p, ts in times.items():
            m = statistics.median(ts)
            res[p] = {"ms_median": round(m * 1e3, 3), "ms_min": round(min(ts) * 1e3, 3),
                      "tflops": round(flop / m / 1e12, 1), "qps": round(nq / m, 1)}
        out[name] = res
    os.environ.pop("LZK_SEARCH", None)
    print(json.dumps(out, indent=1), flush=True)


if __name__ == "__main__":
    main()
