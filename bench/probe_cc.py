"""Why is union-find CC ~7.6 ms inside bench_consolidate and ~3.3 ms in a
warm loop (10M rows, 20M random edges)? Times T.components warm, after a
2 GiB buffer write (cold caches), and with the edge list re-ordered (sorted
by src; by min(src, dst)), plus the whole digest cold."""
import json
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    from lazzaro_amd.ops import tenant_ops as T
    n = int(os.environ.get("NODES", 10_000_000))
    ne = int(os.environ.get("EDGES", 20_000_000))
    dev = torch.device("cuda", 0)
    gen = torch.Generator(device=dev).manual_seed(8)
    src = torch.randint(0, n, (ne,), device=dev, generator=gen).int()
    dst = torch.randint(0, n, (ne,), device=dev, generator=gen).int()
    junk = torch.empty(1 << 29, dtype=torch.float32, device=dev)
    out = {}

    def t(fn, cold, reps=5):
        fn()
        ts = []
        for _ in range(reps):
            if cold:
                junk.fill_(1.0)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            fn()
            torch.cuda.synchronize()
            ts.append((time.perf_counter() - t0) * 1e3)
        return round(sorted(ts)[len(ts) // 2], 3)

    ref = T.components(src, dst, n)
    out["warm_ms"] = t(lambda: T.components(src, dst, n), False)
    out["cold_ms"] = t(lambda: T.components(src, dst, n), True)
    o = torch.argsort(src)
    s1, d1 = src[o].contiguous(), dst[o].contiguous()
    out["sorted_src_cold_ms"] = t(lambda: T.components(s1, d1, n), True)
    out["sorted_src_equal"] = bool(torch.equal(T.components(s1, d1, n), ref))
    lo, hi = torch.minimum(src, dst), torch.maximum(src, dst)
    o = torch.argsort(hi.long() * n + lo.long())
    s2, d2 = hi[o].contiguous(), lo[o].contiguous()
    out["sorted_hi_cold_ms"] = t(lambda: T.components(s2, d2, n), True)
    out["sorted_hi_equal"] = bool(torch.equal(T.components(s2, d2, n), ref))
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
