"""A/B of the int8 store-search scan kernels on a 10M x 768 tenant, 1024
random unit queries: the dedicated scan8.hip kernel vs the shared 256^2
template (search256.hip MmaI8), interleaved rounds in one process. Raw scans
use thr = +inf (no candidates); full store searches go through
TenantGraph._i8_candidates + the fp32 re-rank. Prints JSON."""
import json
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    os.environ.setdefault("LZK_SEARCH_LOWP", "i8")
    from lazzaro_amd.engine import tenant_graph as TG
    from lazzaro_amd.ops import _lib
    from lazzaro_amd.ops import search as S

    dev = torch.device("cuda", 0)
    N, D, nq = int(os.environ.get("AB_ROWS", 10_000_000)), 768, int(os.environ.get("AB_Q", 1024))
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
    q8, qs = S.quantize_i8_rows(q16)
    L = _lib.lib()
    st = _lib.stream_ptr(dev)
    inf = torch.full((nq,), float("inf"), device=dev)
    cnt, cs, ci = S._cand_lists(dev, nq, 2048, 0)

    def raw_template():
        grid = L.lzk_cand_grid_f8(N, nq)
        bbuf, bcap, bcnt = S._blk_records(dev, grid, nq, 16, 128, 1)
        _lib.check(L.lzk_flat_cand_i8(g.emb8.data_ptr(), g.emb8.stride(0), N, q8.data_ptr(), q8.stride(0), nq, D,
                                      bias.data_ptr(), g.rs8.data_ptr(), qs.data_ptr(), 2.0, inf.data_ptr(), 2048,
                                      cnt.data_ptr(), cs.data_ptr(), ci.data_ptr(), bbuf.data_ptr(), bcap,
                                      bcnt.data_ptr(), st), "raw8")

    def raw_scan8():
        grid = L.lzk_scan8_grid(N, nq)
        bbuf, bcap, bcnt, _ = S._wave_records(dev, grid, nq, 16, 128, 1)
        ws = S._ws_scan8.get(dev, int(L.lzk_scan8_ws_bytes(N)))
        _lib.check(L.lzk_scan8(g.emb8.data_ptr(), g.emb8.stride(0), N, q8.data_ptr(), q8.stride(0), nq, D,
                               bias.data_ptr(), g.rs8.data_ptr(), qs.data_ptr(), None, None, 2.0, inf.data_ptr(),
                               None, ws.data_ptr(), bbuf.data_ptr(), bcap, bcnt.data_ptr(), st), "scan8")

    def store(mode):
        S.SCAN8 = mode
        return g._rerank_store(Q, g._i8_candidates(Q, q16, 16, bias, 2.0)[1], 10, "l2", bias)

    def timeit(fn, n=10):
        fn()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(n):
            r = fn()
        torch.cuda.synchronize()
        return (time.perf_counter() - t0) / n * 1e3, r

    arms = {"raw_template_ms": raw_template, "raw_scan8_ms": raw_scan8,
            "store_template_ms": lambda: store(False), "store_scan8_ms": lambda: store(True)}
    res = {k: [] for k in arms}
    outs = {}
    for _ in range(int(os.environ.get("AB_ROUNDS", 5))):
        for k, fn in arms.items():
            t, r = timeit(fn)
            res[k].append(round(t, 4))
            outs[k] = r
    out = {"rows": N, "queries": nq, "dim": D}
    for k, v in res.items():
        out[k] = {"median": sorted(v)[len(v) // 2], "min": min(v), "all": v}
    flop = 2.0 * N * nq * D
    out["raw_scan8_tops"] = round(flop / out["raw_scan8_ms"]["median"] / 1e9, 1)
    out["raw_template_tops"] = round(flop / out["raw_template_ms"]["median"] / 1e9, 1)
    (sa, ra), (sb, rb) = outs["store_scan8_ms"], outs["store_template_ms"]
    out["same_rows"] = bool(torch.equal(ra, rb))
    out["same_scores"] = bool(torch.equal(sa, sb))
    S.SCAN8 = True
    g._i8_candidates(Q, q16, 16, bias, 2.0)
    torch.cuda.synchronize()
    c = S._ws_cand.get(dev, 0)[: nq * 4].view(torch.int32) & 0x3FFFFFFF
    out["candidates_per_query"] = {"mean": float(c.float().mean()), "max": int(c.max())}
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
