"""Where a warm k-means hierarchy pass spends its time on the bench's 10M x
768 tenant: each component of TenantGraph.cluster_pass timed on its own
(HIP-synchronised wall time, median of 5). Prints one JSON object."""
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
    from lazzaro_amd.engine.tenant_graph import NODE
    from lazzaro_amd.index.kmeans import assign, assign_two_level, kmeans
    from lazzaro_amd.ops import graph_ops as G

    dev = torch.device("cuda", 0)
    ms = build_tenant(dev, 10_000_000, 768, None, 7, tempfile.mkdtemp(), 640, 4096, 64, 2, None)
    g = ms.graph
    g.cluster_pass(4096, 64, iters=2)
    h = g.hier
    n = g.n
    X = g.emb16[:n]
    C16 = h["fine_c"].to(torch.bfloat16)
    T16, tof = h["top_c16"], h["top_of_fine"]
    Dp = X.shape[1]

    def t(fn, reps=5):
        fn()
        torch.cuda.synchronize()
        v = []
        for _ in range(reps):
            t0 = time.perf_counter()
            fn()
            torch.cuda.synchronize()
            v.append((time.perf_counter() - t0) * 1e3)
        return round(statistics.median(v), 3)

    live = (g.kind[:n] == NODE) & (g.sup[:n] == 0) & (g.has_emb[:n] == 1)
    rows_all = torch.nonzero(live).flatten()
    pick = torch.randint(0, rows_all.numel(), (1 << 20,), device=dev)
    Xs = X[rows_all[pick]]
    lab, _ = assign_two_level(X, C16, T16, tof)
    lab = lab.long()
    out = {
        "live_mask_nonzero": t(lambda: torch.nonzero((g.kind[:n] == NODE) & (g.sup[:n] == 0) & (g.has_emb[:n] == 1))),
        "sample_gather_1M": t(lambda: X[rows_all[pick]]),
        "sample_assign_two_level_1M": t(lambda: assign_two_level(Xs, C16, T16, tof)),
        "sample_assign_flat_1M": t(lambda: assign(Xs, C16)),
        "sample_centroids_1M": t(lambda: G.centroids(Xs, assign(Xs, C16)[0], 4096, normalize=True, pad_to=Dp)),
        "top_assign_10M": t(lambda: assign(X, T16)),
        "full_assign_two_level_10M": t(lambda: assign_two_level(X, C16, T16, tof)),
        "full_centroids_10M": t(lambda: G.centroids(X, lab.to(torch.int32), 4096, normalize=True, pad_to=Dp)),
        "top_kmeans_4096": t(lambda: kmeans(C16, 64, iters=4, seed=1, init=h["top_c"])),
        "hier_order_argsort_10M": t(lambda: torch.argsort(lab * n + torch.arange(n, device=dev))),
        "whole_warm_pass": t(lambda: g.cluster_pass(4096, 64, iters=2)),
    }
    print(json.dumps({"rows": n, "ms_median": out}, indent=1))


if __name__ == "__main__":
    main()
