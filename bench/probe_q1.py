"""Kernel timeline of single-query store searches over a 10M x 768 tenant
(the interactive search_memories path): builds the tenant
with TenantGraph directly, warms up, then runs --iters Q=1 store searches
with a host timer. Run under `rocprofv3 --kernel-trace` and read the last
dispatches with bench/rocpd_summary.py --timeline. Synthetic unit rows."""
import argparse
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=int, default=10_000_000)
    ap.add_argument("--iters", type=int, default=30)
    ap.add_argument("--q", type=int, default=1)
    a = ap.parse_args()
    from lazzaro_amd.engine.tenant_graph import TenantGraph
    dev = torch.device("cuda", 0)
    N, D = a.rows, 768
    g = TenantGraph(device=dev, dim=D, capacity=N)
    code = g.shard_id("default")
    gen = torch.Generator(device=dev).manual_seed(5)
    chunk = 1 << 21
    for c0 in range(0, N, chunk):
        c1 = min(N, c0 + chunk)
        X = torch.randn(c1 - c0, D, device=dev, generator=gen)
        X /= X.norm(dim=1, keepdim=True)
        g.add_nodes([f"n{i}" for i in range(c0, c1)], [""] * (c1 - c0), X, shard=code, stored=True)
    Qs = torch.randn(a.iters + 5, a.q, D, device=dev, generator=gen)
    Qs /= Qs.norm(dim=2, keepdim=True)
    for i in range(5):
        g.store_search(Qs[i], 10)
    torch.cuda.synchronize()
    ts = []
    for i in range(a.iters):
        t0 = time.perf_counter()
        g.store_search(Qs[5 + i], 10)
        torch.cuda.synchronize()
        ts.append(time.perf_counter() - t0)
    ts.sort()
    print(json.dumps({"rows": N, "q": a.q, "p50_ms": round(ts[len(ts) // 2] * 1e3, 3),
                      "min_ms": round(ts[0] * 1e3, 3)}), flush=True)


if __name__ == "__main__":
    main()
