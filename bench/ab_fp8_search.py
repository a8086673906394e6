"""A/B of the store search's candidate scan: fp8 (e4m3 rows, 16x16x128 MFMA,
bf16 re-score) vs bf16, on a 10M x 768 tenant with 1024 random unit queries.
Prints per-variant ms and candidate-list statistics (JSON)."""
import json
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    from lazzaro_amd.engine import tenant_graph as TG
    from lazzaro_amd.ops import search as S

    dev = torch.device("cuda", 0)
    N, D, nq = int(os.environ.get("AB_ROWS", 10_000_000)), 768, 1024
    g = TG.TenantGraph(device=dev)
    g._set_dim(D)
    g.reserve(N)
    gen = torch.Generator(device=dev).manual_seed(1)
    for r0 in range(0, N, 1 << 20):
        r1 = min(N, r0 + (1 << 20))
        v = torch.randn(r1 - r0, D, device=dev, generator=gen)
        g.add_nodes([f"n{i}" for i in range(r0, r1)], [""] * (r1 - r0), v / v.norm(dim=1, keepdim=True),
                    shard=g.shard_id("work"), stored=True)
    Q = torch.randn(nq, D, device=dev, generator=gen)
    Q = Q / Q.norm(dim=1, keepdim=True)
    out = {}

    def timeit(fn, n=5):
        fn()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(n):
            r = fn()
        torch.cuda.synchronize()
        return (time.perf_counter() - t0) / n * 1e3, r

    bias = g.store_bias("l2")
    q16 = g._q16(Q)
    out["bf16_store_search_ms"], (_, r16) = timeit(lambda: g._rerank_store(
        Q, S.flat_topk(g.emb16[:N], q16, 16, bias=bias, alpha=2.0)[1], 10, "l2", bias))
    out["fp8_store_search_ms"], (_, r8) = timeit(lambda: g._rerank_store(
        Q, g._fp8_candidates(Q, q16, 16, bias, 2.0)[1], 10, "l2", bias))
    out["same_rows"] = bool(torch.equal(r16, r8))
    # candidate-list sizes of the fp8 pass
    g._fp8_candidates(Q, q16, 16, bias, 2.0)
    torch.cuda.synchronize()
    ws = S._ws_cand.get(dev, 0)
    c = ws[: nq * 4].view(torch.int32) & 0x3FFFFFFF
    out["fp8_candidates_per_query"] = {"mean": float(c.float().mean()), "max": int(c.max())}
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
