"""Union-find time vs the seed of a uniform random graph (10M rows, 20M
edges, generated like bench_consolidate.build_tenant), sorted by src / by dst
/ unsorted, one union pass vs staged passes (union + compress per chunk), plus
a check for generator correlation between the two draws. T.components is the
staged production path."""
import json
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    from lazzaro_amd.ops import tenant_ops as T
    from lazzaro_amd.ops import _lib
    def t(fn, k=9):
        fn()
        torch.cuda.synchronize()
        ts = []
        for _ in range(k):
            t0 = time.perf_counter()
            fn()
            torch.cuda.synchronize()
            ts.append((time.perf_counter() - t0) * 1e3)
        return round(sorted(ts)[k // 2], 3)

    for seed in (2, 3, 8, 11):
        gen = torch.Generator(device=dev).manual_seed(seed)
        src = torch.randint(0, n, (ne,), device=dev, generator=gen).int()
        dst = torch.randint(0, n, (ne,), device=dev, generator=gen).int()
        row = {"seed": seed}
        row["unsorted_ms"] = t(lambda: T.components(src, dst, n))
        o = torch.sort(src, stable=True).indices
        s1, d1 = src[o].contiguous(), dst[o].contiguous()
        row["by_src_ms"] = t(lambda: T.components(s1, d1, n))
        o = torch.sort(dst, stable=True).indices
        s2, d2 = dst[o].contiguous(), src[o].contiguous()
        row["by_dst_ms"] = t(lambda: T.components(s2, d2, n))
        # correlation: dst[i] == src[i + k]
        row["shift_match"] = {k: int((dst[max(0, -k): ne - max(0, k)] == src[max(0, k): ne - max(0, -k)]).sum())
                              for k in (-2, -1, 0, 1, 2)}
        lab = T.components(s1, d1, n)
        big = torch.bincount(lab.long()).max()
        row["giant"] = int(big)
        ref = T.components(s1, d1, n)
        from lazzaro_amd.ops.graph_ops import connected_components as CC
        assert torch.equal(CC(s1, d1, n, method="hook"), ref)
        def staged(s_, d_, k):
            parent = torch.arange(n, dtype=torch.int32, device=s_.device)
            L_, st = _lib.lib(), _lib.stream_ptr(s_.device)
            step = (ne + k - 1) // k
            for c0 in range(0, ne, step):
                c1 = min(ne, c0 + step)
                _lib.check(L_.lzk_uf_union(s_[c0:].data_ptr(), d_[c0:].data_ptr(), c1 - c0, None, 0.0,
                                           parent.data_ptr(), st), "uf")
                _lib.check(L_.lzk_cc_compress(parent.data_ptr(), n, st), "cc_compress")
            return parent
        for k in (2, 4, 8, 16):
            assert torch.equal(staged(s1, d1, k), ref), k
            row[f"staged{k}_src"] = t(lambda: staged(s1, d1, k))
            row[f"staged{k}_dst"] = t(lambda: staged(s2, d2, k))
            row[f"staged{k}_uns"] = t(lambda: staged(src, dst, k))
        # independent draws: dst from a second generator
        g2 = torch.Generator(device=dev).manual_seed(seed + 1000)
        dst2 = torch.randint(0, n, (ne,), device=dev, generator=g2).int()
        o = torch.sort(src, stable=True).indices
        s3, d3 = src[o].contiguous(), dst2[o].contiguous()
        row["indep_by_src_ms"] = t(lambda: T.components(s3, d3, n))
        print(json.dumps(row), flush=True)


if __name__ == "__main__":
    main()
