"""A/B of the dual candidate kernel's schedules (flat_topk_dual: one scan,
unfiltered + shard-filtered lists) on consolidation-shaped data: a 10M x 768
buffer in 64 topic shards with tombstones, 1024 new facts that are
perturbations of existing memories (10 % near-duplicates), k = 3. Interleaved
rounds in one process; prints one JSON object."""
import ctypes
import json
import os
import statistics
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from lazzaro_amd.ops import _lib  # noqa: E402
from lazzaro_amd.ops.search import flat_topk_dual  # noqa: E402

L = _lib.lib()
L.lzk_set_dual_opt.argtypes = [ctypes.c_int]


def main():
    n = int(os.environ.get("AB_ROWS", "10000000"))
    d, nq, k = 768, 1024, 3
    dev = "cuda"
    g = torch.Generator(device=dev).manual_seed(0)
    X = torch.empty(n, d, device=dev, dtype=torch.bfloat16)
    for r0 in range(0, n, 1 << 20):
        x = torch.randn(min(1 << 20, n - r0), d, device=dev, generator=g)
        X[r0:r0 + x.shape[0]] = torch.nn.functional.normalize(x, dim=1).to(torch.bfloat16)
    lab = torch.randint(0, 64, (n,), device=dev, dtype=torch.int32, generator=g)
    bias = torch.where(torch.rand(n, device=dev, generator=g) < 0.01, float("-inf"), 0.0)
    base = X[torch.randint(0, n, (nq,), device=dev, generator=g)].float()
    noise = torch.randn(nq, d, device=dev, generator=g) / d ** 0.5
    dup = torch.rand(nq, device=dev, generator=g) < 0.1
    Q = torch.nn.functional.normalize(torch.where(dup[:, None], base + 0.1 * noise, base + 1.2 * noise), dim=1)
    Q = Q.to(torch.bfloat16)
    ql = torch.randint(0, 64, (nq,), device=dev, dtype=torch.int32, generator=g)
    opts = [int(v) for v in os.environ.get("AB_OPTS", "0,8,16,24").split(",")]
    res = {}
    for o in opts:
        L.lzk_set_dual_opt(o)
        res[o] = flat_topk_dual(X, Q, k, bias=bias, row_label=lab, q_label=ql)
    same = {o: float(((res[o][0][1] == res[opts[0]][0][1]).float().mean() +
                      (res[o][1][1] == res[opts[0]][1][1]).float().mean()) / 2) for o in opts[1:]}
    ts = {o: [] for o in opts}
    for _ in range(5):
        for o in opts:
            L.lzk_set_dual_opt(o)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(3):
                flat_topk_dual(X, Q, k, bias=bias, row_label=lab, q_label=ql)
            torch.cuda.synchronize()
            ts[o].append((time.perf_counter() - t0) / 3)
    L.lzk_set_dual_opt(-1)
    print(json.dumps({"rows": n, "nq": nq, "k": k, "ids_equal_frac": same,
                      "ms_median": {o: round(statistics.median(v) * 1e3, 3) for o, v in ts.items()}}, indent=1))


if __name__ == "__main__":
    main()
