"""Kernel-time profile target for the headline's store search: a 10M x 768
tenant (random unit rows, int8 + bf16 + fp32 columns as bench.py builds it)
and P_REPS store searches of 1024 random unit queries (k = 10, L2).
Run under: rocprofv3 --kernel-trace --stats -- python bench/prof_store_search.py"""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    from lazzaro_amd.engine.tenant_graph import TenantGraph
    dev = torch.device("cuda", 0)
    N, D, nq = int(os.environ.get("P_ROWS", 10_000_000)), 768, int(os.environ.get("P_Q", 1024))
    g = TenantGraph(device=dev)
    g._set_dim(D)
    g.reserve(N)
    gen = torch.Generator(device=dev).manual_seed(1)
    code = g.shard_id("work")
    for r0 in range(0, N, 1 << 20):
        r1 = min(N, r0 + (1 << 20))
        v = torch.randn(r1 - r0, D, device=dev, generator=gen)
        g.add_nodes([f"n{i}" for i in range(r0, r1)], [""] * (r1 - r0), v / v.norm(dim=1, keepdim=True),
                    shard=code, stored=True)
    Q = torch.randn(nq, D, device=dev, generator=gen)
    Q = Q / Q.norm(dim=1, keepdim=True)
    for _ in range(3):
        g.store_search(Q, 10, "l2")
    torch.cuda.synchronize()
    reps = int(os.environ.get("P_REPS", "10"))
    t0 = time.perf_counter()
    for _ in range(reps):
        g.store_search(Q, 10, "l2")
    torch.cuda.synchronize()
    print("store_search_ms", round((time.perf_counter() - t0) / reps * 1e3, 3), flush=True)


if __name__ == "__main__":
    main()
