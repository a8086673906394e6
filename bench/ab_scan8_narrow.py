"""Narrow batches on a 10M x 768 tenant: the store search's candidate pass
with the HBM-bound int8 narrow kernel (scan8.hip scan8_narrow_kernel) vs the
bf16 per-lane kernel, Q = 1 / 16 / 64 / 127, interleaved rounds in one
process; plus the raw narrow scan (thr = +inf) as an effective-bandwidth
figure. Prints JSON."""
import json
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    from lazzaro_amd.engine import tenant_graph as TG
    from lazzaro_amd.ops import _lib
    from lazzaro_amd.ops import search as S

    dev = torch.device("cuda", 0)
    N, D = int(os.environ.get("AB_ROWS", 10_000_000)), 768
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
    bias = g.store_bias("l2")
    L = _lib.lib()
    st = _lib.stream_ptr(dev)

    def timeit(fn, n=20):
        fn()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(n):
            r = fn()
        torch.cuda.synchronize()
        return (time.perf_counter() - t0) / n * 1e3, r

    out = {"rows": N, "dim": D}
    for nq in (1, 16, 64, 127):
        Q = torch.randn(nq, D, device=dev, generator=gen)
        Q = Q / Q.norm(dim=1, keepdim=True)
        q16 = g._q16(Q)
        q8, qs = S.quantize_i8_rows(q16)
        inf = torch.full((nq,), float("inf"), device=dev)

        def raw():
            grid = L.lzk_scan8_narrow_grid(N)
            bbuf, bcap, bcnt, _ = S._wave_records(dev, grid, nq, 16, 128, 1)
            _lib.check(L.lzk_scan8_narrow(g.emb8.data_ptr(), g.emb8.stride(0), N, q8.data_ptr(), q8.stride(0), nq,
                                          D, bias.data_ptr(), g.rs8.data_ptr(), qs.data_ptr(), 2.0, inf.data_ptr(),
                                          bbuf.data_ptr(), bcap, bcnt.data_ptr(), st), "narrow")

        def i8():
            return g._i8_candidates(Q, q16, 16, bias, 2.0)

        def bf16():
            return S.flat_topk(g.emb16[:N], q16, 16, bias=bias, alpha=2.0)

        def api():
            return g.store_search(Q, 10, "l2")
        res = {"raw_narrow_ms": [], "i8_cand_ms": [], "bf16_cand_ms": [], "store_search_ms": []}
        outs = {}
        for _ in range(3):
            for k, fn in (("raw_narrow_ms", raw), ("i8_cand_ms", i8), ("bf16_cand_ms", bf16),
                          ("store_search_ms", api)):
                t, r = timeit(fn)
                res[k].append(round(t, 4))
                outs[k] = r
        ent = {k: sorted(v)[1] for k, v in res.items()}
        ent["raw_narrow_tb_s"] = round(N * D / (ent["raw_narrow_ms"] * 1e-3) / 1e12, 2)
        ent["same_rows"] = bool(torch.equal(outs["i8_cand_ms"][1][:, :10], outs["bf16_cand_ms"][1][:, :10]))
        out[f"q{nq}"] = ent
        print(json.dumps({f"q{nq}": ent}), flush=True)
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
