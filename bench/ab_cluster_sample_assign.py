"""A/B of the warm k-means hierarchy pass on the bench's 10M x 768 tenant
(TenantGraph.cluster_pass, 4096 fine / 64 topic clusters, 2 iterations): the
mini-batch step's assign over all 4096 fine centroids (flat argmax) vs the
two-level assign (nearest topic, then its fine clusters) that the full-data
step already uses. Every timed pass starts from the same seed-pass state.
Quality: mean cosine of 1M sampled rows to their assigned fine centroid.
Prints one JSON object."""
import copy
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
    from bench_consolidate import build_tenant
    from lazzaro_amd.engine.tenant_graph import TenantGraph

    n = int(os.environ.get("AB_ROWS", "10000000"))
    dev = torch.device("cuda", 0)
    ms = build_tenant(dev, n, 768, None, 7, tempfile.mkdtemp(), 640, 4096, 64, 2, None)
    g = ms.graph
    t0 = time.perf_counter()
    g.cluster_pass(4096, 64, iters=2)
    torch.cuda.synchronize()
    seed_ms = (time.perf_counter() - t0) * 1e3
    seed_state = copy.copy(g.hier)
    gen = torch.Generator(device=dev).manual_seed(3)
    probe = torch.randint(0, g.n, (1 << 20,), device=dev, generator=gen)

    def quality():
        lab = g.hier["fine"][probe].long()
        ok = lab >= 0
        c = g.hier["fine_c"][lab.clamp_min(0)]
        x = g.emb32[probe].float()
        cos = (x * c[:, : x.shape[1]]).sum(1) / x.norm(dim=1).clamp_min(1e-30) / c.norm(dim=1).clamp_min(1e-30)
        return float(cos[ok].mean())

    arms = {"flat_sample_assign": False, "two_level_sample_assign": True}
    ts = {a: [] for a in arms}
    qual = {}
    for rnd in range(4):
        for a, two in arms.items():
            TenantGraph.SAMPLE_TWO_LEVEL = two
            g.hier = copy.copy(seed_state)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            g.cluster_pass(4096, 64, iters=2, seed=rnd)
            torch.cuda.synchronize()
            if rnd > 0:
                ts[a].append((time.perf_counter() - t0) * 1e3)
            qual[a] = round(quality(), 5)
    print(json.dumps({"rows": g.n, "fine": 4096, "top": 64, "seed_pass_ms": round(seed_ms, 1),
                      "warm_pass_ms_median": {a: round(statistics.median(v), 2) for a, v in ts.items()},
                      "mean_cos_to_fine_centroid": qual}, indent=1))


if __name__ == "__main__":
    main()
