"""run_consolidation's component digest on a large graph (10M rows, 20M
edges): total time of TenantGraph.component_digest and of each of its device
stages, to find what dominates (bench_consolidate --prune-threshold 0 showed
~170 ms per digest)."""
import json
import os
import sys
import tempfile
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "bench"))


def main():
    nodes = int(os.environ.get("NODES", 10_000_000))
    edges = int(os.environ.get("EDGES", 20_000_000))
    from bench_consolidate import build_tenant
    from lazzaro_amd.engine import tenant_graph as TGm
    from lazzaro_amd.ops import tenant_ops as T

    dev = torch.device("cuda", 0)
    ms = build_tenant(dev, nodes, 768, None, 1, tempfile.mkdtemp(), 640, 64, 8, 1, edges)
    g = ms.graph
    out = {"nodes": nodes, "edges": g.num_edges}

    def t(fn, n=3):
        fn()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(n):
            r = fn()
        torch.cuda.synchronize()
        return round((time.perf_counter() - t0) / n * 1e3, 3), r

    out["digest_ms"], comps = t(lambda: g.component_digest())
    out["n_qualifying"] = len(comps)
    g._digest_sorted = True
    out["digest_sorted_ms"], comps2 = t(lambda: g.component_digest())
    g._digest_sorted = False
    out["digest_equal"] = [c.tolist() for c in comps] == [c.tolist() for c in comps2]
    src, dst = g.e["src"].long(), g.e["dst"].long()
    E = src.numel()
    out["unique_ms"], (verts, inv) = t(lambda: torch.unique(torch.cat([src, dst]), return_inverse=True))
    nv = verts.numel()
    s32, d32 = inv[:E].to(torch.int32), inv[E:].to(torch.int32)
    out["cc_ms"], cl = t(lambda: T.components(s32, d32, nv))
    from lazzaro_amd.ops import graph_ops as G
    out["cc_full_n_ms"], _ = t(lambda: T.components(g.e["src"], g.e["dst"], g.n))
    cl = cl.long()
    kind_v = g.kind[verts]
    member = kind_v != TGm.FREE
    out["segsum_size_ms"], _ = t(lambda: TGm._seg_sum_count(cl[member], torch.zeros(int(member.sum()), dtype=torch.float32, device=dev), nv))
    out["segsum_w_ms"], _ = t(lambda: TGm._seg_sum_count(cl[inv[:E]], g.e["w"], nv))
    okey = verts.clone()
    first = torch.full((nv,), 1 << 62, dtype=torch.long, device=dev)
    key = torch.randint(0, 1 << 20, (nv,), device=dev)
    out["argsort_nv_ms"], _ = t(lambda: torch.argsort(key * g.n + verts))
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
