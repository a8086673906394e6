"""A/B of flat_topk_dual's list-B threshold (safe sampled shard bound vs the
speculative bound of search._spec_threshold_b with exact underflow fallback),
whole call incl. sample passes, selects and fallbacks, on consolidation-shaped
data: a 10M x 768 buffer in 64 topic shards with tombstones, 1024 new facts
that are perturbations of existing memories (10 % near-duplicates), k = 3.
Interleaved rounds in one process; prints one JSON object."""
import json
import os
import statistics
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from lazzaro_amd.ops import _lib  # noqa: E402
from lazzaro_amd.ops import search  # noqa: E402
from lazzaro_amd.ops.search import flat_topk_dual  # noqa: E402


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
    arms = {"safe": (False, 16.0), "spec16": (True, 16.0), "spec24": (True, 24.0), "spec10": (True, 10.0)}
    opts = list(arms)

    def run(o):
        search.DUAL_SPEC, search.DUAL_SPEC_E = arms[o]
        return flat_topk_dual(X, Q, k, bias=bias, row_label=lab, q_label=ql, n_labels=64)
    res = {}
    for o in opts:
        res[o] = run(o)
    same = {o: [float((res[o][0][1] == res[opts[0]][0][1]).float().mean()),
                float((res[o][1][1] == res[opts[0]][1][1]).float().mean()),
                float((res[o][1][0] - res[opts[0]][1][0]).abs().max())] for o in opts[1:]}
    ts = {o: [] for o in opts}
    for _ in range(5):
        for o in opts:
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(3):
                run(o)
            torch.cuda.synchronize()
            ts[o].append((time.perf_counter() - t0) / 3)
    print(json.dumps({"rows": n, "nq": nq, "k": k, "ids_equal_frac": same,
                      "ms_median": {o: round(statistics.median(v) * 1e3, 3) for o, v in ts.items()}}, indent=1))


if __name__ == "__main__":
    main()
