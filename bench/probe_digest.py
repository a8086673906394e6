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
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
