"""PMC probe of the wide int8 scan (scan8.hip) on 10M x 768 x 1024: the
kernel with the store search's sampled thresholds (candidates flow) or with
thr = +inf (no candidates; PROBE_INF=1). Run under rocprofv3 --pmc."""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    from lazzaro_amd.engine import tenant_graph as TG
    from lazzaro_amd.ops import search as S
    dev = torch.device("cuda", 0)
    N, D, nq = int(os.environ.get("AB_ROWS", 10_000_000)), 768, 1024
    TG.TenantGraph.LOWP = "i8"
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
    bias = g.store_bias("l2")
    q16 = g._q16(Q)
    q8, qs, margin = g._i8_query(q16, 2.0)
    kslot = 16
    Sd = 64
    thr = S._sample_threshold(g.emb16[:N], q16, 16, kslot, bias, None, None, 2.0, Sd)
    thr = (thr - margin).contiguous()
    if os.environ.get("PROBE_INF") == "1":
        thr = torch.full_like(thr, float("inf"))
    S.SCAN8 = os.environ.get("PROBE_TEMPLATE") != "1"
    cap = max(2048, 16 * kslot * Sd)
    for _ in range(5):
        ca = S._cand_lists(dev, nq, cap, 0)
        if S.SCAN8:
            S._scan8(g.emb8[:N], g.rs8[:N], q8, qs, bias, 2.0, thr, None, None, None, kslot, 2 * Sd, 1, cap, ca, None)
        else:
            from lazzaro_amd.ops import _lib
            L = _lib.lib()
            grid = L.lzk_cand_grid_f8(N, nq)
            bbuf, bcap, bcnt = S._blk_records(dev, grid, nq, kslot, 2 * Sd, 1)
            _lib.check(L.lzk_flat_cand_i8(g.emb8.data_ptr(), g.emb8.stride(0), N, q8.data_ptr(), q8.stride(0), nq, D,
                                          bias.data_ptr(), g.rs8.data_ptr(), qs.data_ptr(), 2.0, thr.data_ptr(), cap,
                                          ca[0].data_ptr(), ca[1].data_ptr(), ca[2].data_ptr(), bbuf.data_ptr(), bcap,
                                          bcnt.data_ptr(), _lib.stream_ptr(dev)), "i8")
    torch.cuda.synchronize()
    c = ca[0] & 0x3FFFFFFF
    print("candidates per query", float(c.float().mean()), flush=True)


if __name__ == "__main__":
    main()
