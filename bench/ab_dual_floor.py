"""A/B of the consolidation scan with and without the score floor
(TenantGraph.cos_topk(min_score=0.5), the dual scan's thresholds raised to
LINK_THRESHOLD - COS_FLOOR_SLACK) on the bench's 10M x 768 tenant and 1024
consolidation-shaped facts (10 % near-duplicates, the rest related memories),
k = 3. Checks that every entry above the floor is identical in both arms and
times the whole call (sample passes, dual scan, selects, fp64 re-rank).
Prints one JSON object."""
import json
import os
import statistics
import sys
import tempfile
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "bench"))


def main():
    from bench_consolidate import build_tenant, synth_vectors
    from lazzaro_amd.engine.tenant_graph import NODE

    n = int(os.environ.get("AB_ROWS", "10000000"))
    dev = torch.device("cuda", 0)
    ms = build_tenant(dev, n, 768, None, 7, tempfile.mkdtemp(), 640, 4096, 64, 2, None)
    g = ms.graph
    gen = torch.Generator(device=dev).manual_seed(5)
    Q = synth_vectors(ms, 1024, 768, 0.1, gen)
    codes = g.shard[torch.randint(0, g.n, (1024,), device=dev, generator=gen)]
    mask = (g.kind[: g.n] == NODE) & (g.sup[: g.n] == 0)

    def run(ms_):
        return g.cos_topk(Q, 3, mask, dual_label=codes, min_score=ms_)
    arms = {"no_floor": None, "floor_0.5": 0.5}
    res = {a: run(v) for a, v in arms.items()}
    (ga, gra), (wa, wra) = res["no_floor"]
    (gb, grb), (wb, wrb) = res["floor_0.5"]
    eq = {}
    for name, (sa, ra, sb, rb) in {"global": (ga, gra, gb, grb), "shard": (wa, wra, wb, wrb)}.items():
        keep = sa > 0.5
        eq[name] = {"above_floor_entries": int(keep.sum()),
                    "rows_equal": bool(torch.equal(torch.where(keep, ra, -1), torch.where(sb > 0.5, rb, -1))),
                    "scores_equal": bool(torch.equal(torch.where(keep, sa, 0.0), torch.where(sb > 0.5, sb, 0.0)))}
    ts = {a: [] for a in arms}
    for _ in range(5):
        for a, v in arms.items():
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(3):
                run(v)
            torch.cuda.synchronize()
            ts[a].append((time.perf_counter() - t0) / 3)
    print(json.dumps({"rows": g.n, "facts": 1024, "k": 3, "equal_above_floor": eq,
                      "ms_median": {a: round(statistics.median(v) * 1e3, 3) for a, v in ts.items()}}, indent=1))


if __name__ == "__main__":
    main()
