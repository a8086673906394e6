"""Component digest on the bench's persistent graph (10M rows, 20M seeded
edges): edge-order descents before / after the first digest, then the
digest and the bare union-find timed warm."""
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
    from bench_consolidate import build_tenant
    from lazzaro_amd.ops import tenant_ops as T
    dev = torch.device("cuda", 0)
    ms = build_tenant(dev, 10_000_000, 768, None, 1, tempfile.mkdtemp(), 640, 64, 8, 1, 20_000_000, 0.0)
    g = ms.graph
    out = {}

    def desc():
        s = g.e["src"]
        return int((s[1:] < s[:-1]).sum())

    def t(fn, n=5):
        fn()
        torch.cuda.synchronize()
        ts = []
        for _ in range(n):
            t0 = time.perf_counter()
            fn()
            torch.cuda.synchronize()
            ts.append((time.perf_counter() - t0) * 1e3)
        return round(sorted(ts)[n // 2], 3)

    out["descents_before"] = desc()
    g.component_digest()
    out["descents_after"] = desc()
    out["digest_ms"] = t(lambda: g.component_digest())
    out["cc_ms"] = t(lambda: T.components(g.e["src"], g.e["dst"], g.n))
    s, d = g.e["src"].contiguous(), g.e["dst"].contiguous()
    out["cc_contig_ms"] = t(lambda: T.components(s, d, g.n))
    out["maybe_sort_ms"] = t(lambda: g._maybe_sort_edges())
    # the same union-find on a fresh uniform graph of the same size, sorted the same way
    n, ne = g.n, g.num_edges
    gen = torch.Generator(device=dev).manual_seed(8)
    rs = torch.randint(0, n, (ne,), device=dev, generator=gen).int()
    rd = torch.randint(0, n, (ne,), device=dev, generator=gen).int()
    o = torch.sort(rs, stable=True).indices
    rs, rd = rs[o].contiguous(), rd[o].contiguous()
    out["cc_fresh_sorted_ms"] = t(lambda: T.components(rs, rd, n))
    # the bench graph's own edges: degree / self-loop / duplicate structure
    src, dst = g.e["src"].long(), g.e["dst"].long()
    out["bench_self_loops"] = int((src == dst).sum())
    out["bench_src_range"] = [int(src.min()), int(src.max())]
    out["bench_dst_range"] = [int(dst.min()), int(dst.max())]
    # swap roles: dst-sorted copy
    o = torch.sort(g.e["dst"], stable=True).indices
    ds, dd = g.e["dst"][o].contiguous(), g.e["src"][o].contiguous()
    out["cc_bench_by_dst_ms"] = t(lambda: T.components(ds, dd, n))
    # fresh graph by dst, then the bench's src order again (order / clock effects)
    o = torch.sort(rd, stable=True).indices
    fs, fd = rd[o].contiguous(), rs[o].contiguous()
    out["cc_fresh_by_dst_ms"] = t(lambda: T.components(fs, fd, n))
    out["cc_ms_again"] = t(lambda: T.components(g.e["src"], g.e["dst"], g.n))
    # the bench pairs shuffled, then stable-sorted by src afresh
    perm = torch.randperm(ne, device=dev, generator=gen)
    ps, pd = g.e["src"][perm], g.e["dst"][perm]
    o = torch.sort(ps, stable=True).indices
    ps, pd = ps[o].contiguous(), pd[o].contiguous()
    out["cc_bench_resorted_ms"] = t(lambda: T.components(ps, pd, n))
    # sort keys: max(src, dst) / min(src, dst) (kernel src = the key endpoint)
    for name, (a_, b_) in {"bench": (g.e["src"], g.e["dst"]), "fresh": (rs, rd)}.items():
        hi, lo = torch.maximum(a_, b_), torch.minimum(a_, b_)
        o = torch.sort(hi, stable=True).indices
        h1, l1 = hi[o].contiguous(), lo[o].contiguous()
        out[f"cc_{name}_by_max_ms"] = t(lambda: T.components(h1, l1, n))
        out[f"cc_{name}_by_max_swapped_ms"] = t(lambda: T.components(l1, h1, n))
        o = torch.sort(lo, stable=True).indices
        h2, l2 = hi[o].contiguous(), lo[o].contiguous()
        out[f"cc_{name}_by_min_ms"] = t(lambda: T.components(l2, h2, n))
    # degree skew: max in/out degree and the share of edges with src > dst
    out["bench_src_gt_dst"] = round(float((g.e["src"] > g.e["dst"]).float().mean()), 4)
    out["fresh_src_gt_dst"] = round(float((rs > rd).float().mean()), 4)
    out["bench_max_outdeg"] = int(torch.bincount(g.e["src"].long()).max())
    out["bench_max_indeg"] = int(torch.bincount(g.e["dst"].long()).max())
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
