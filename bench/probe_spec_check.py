"""Speculative-threshold check A/B on one 10M x 768 tenant: the number of
queries each formulation (kernel-side count vs torch over the lists) sends
to the exact fallback, with the int8 query kernel on and off, and the store
search time. Random unit rows; random and clustered unit queries."""
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    from lazzaro_amd.engine import tenant_graph as TG
    from lazzaro_amd.ops import search as S
    dev = torch.device("cuda", 0)
    N, D = 10_000_000, 768
    g = TG.TenantGraph(device=dev, dim=D, capacity=N)
    code = g.shard_id("default")
    gen = torch.Generator(device=dev).manual_seed(5)
    for c0 in range(0, N, 1 << 21):
        c1 = min(N, c0 + (1 << 21))
        X = torch.randn(c1 - c0, D, device=dev, generator=gen)
        X /= X.norm(dim=1, keepdim=True)
        g.add_nodes([f"n{i}" for i in range(c0, c1)], [""] * (c1 - c0), X, shard=code, stored=True)
    Qr = torch.randn(1024, D, device=dev, generator=gen)
    Qr /= Qr.norm(dim=1, keepdim=True)
    base = torch.randn(1, D, device=dev, generator=gen)
    Qc = base + 0.3 * torch.randn(1024, D, device=dev, generator=gen)  # anisotropic, like untrained encoders
    Qc /= Qc.norm(dim=1, keepdim=True)
    seen = {}
    orig = S._select_with_fallback

    def spy(*a, **k):
        nd = k.get("need")
        if nd is not None:
            seen["flagged"] = int((nd != 0).sum())
        return orig(*a, **k)
    S._select_with_fallback = spy
    out = {}
    for qname, Q in (("random", Qr), ("clustered", Qc)):
        for qk in (True, False):
            for ck in (True, False):
                TG.I8_QUERY_KERNEL = qk
                S.SPEC_CHECK_KERNEL = ck
                g.store_search(Q, 10)
                torch.cuda.synchronize()
                t0 = time.perf_counter()
                for _ in range(5):
                    s, r = g.store_search(Q, 10)
                torch.cuda.synchronize()
                out[f"{qname}_qk{int(qk)}_ck{int(ck)}"] = {"flagged": seen.get("flagged"),
                                                          "ms": round((time.perf_counter() - t0) / 5 * 1e3, 3),
                                                          "rows_sum": int(r.sum())}
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
