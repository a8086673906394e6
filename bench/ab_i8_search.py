"""A/B of the store search's candidate scan: int8 (per-row int8 rows,
v_mfma_i32_16x16x64_i8, error cut + bf16 re-score) vs bf16, on a 10M x 768
tenant with 1024 random unit queries -- plus the raw scan kernels with no
candidate passing (thr = +inf), which isolates the GEMM pipeline rate.
Prints per-variant ms and candidate-list statistics (JSON)."""
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
    out = {"rows": N, "queries": nq}

    def timeit(fn, n=10):
        fn()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(n):
            r = fn()
        torch.cuda.synchronize()
        return (time.perf_counter() - t0) / n * 1e3, r

    bias = g.store_bias("l2")
    q16 = g._q16(Q)
    L = _lib.lib()
    st = _lib.stream_ptr(dev)

    # raw kernels, nothing passes the threshold
    inf = torch.full((nq,), float("inf"), device=dev)
    cnt, cs, ci = S._cand_lists(dev, nq, 2048, 0)
    grid = L.lzk_cand_grid(N, nq, 0)
    bbuf, bcap, bcnt = S._blk_records(dev, grid, nq, 16, 64, 1)

    def raw16():
        _lib.check(L.lzk_flat_cand(g.emb16.data_ptr(), g.emb16.stride(0), N, q16.data_ptr(), q16.stride(0), nq, D,
                                   bias.data_ptr(), None, None, 2.0, inf.data_ptr(), 2048, cnt.data_ptr(),
                                   cs.data_ptr(), ci.data_ptr(), bbuf.data_ptr(), bcap, bcnt.data_ptr(), st), "raw16")

    q8, qs = S.quantize_i8_rows(q16)

    def raw8():
        _lib.check(L.lzk_flat_cand_i8(g.emb8.data_ptr(), g.emb8.stride(0), N, q8.data_ptr(), q8.stride(0), nq, D,
                                      bias.data_ptr(), g.rs8.data_ptr(), qs.data_ptr(), 2.0, inf.data_ptr(), 2048,
                                      cnt.data_ptr(), cs.data_ptr(), ci.data_ptr(), bbuf.data_ptr(), bcap,
                                      bcnt.data_ptr(), st), "raw8")

    out["raw_bf16_scan_ms"], _ = timeit(raw16)
    out["raw_i8_scan_ms"], _ = timeit(raw8)
    flop = 2.0 * N * nq * D
    out["raw_bf16_tflops"] = round(flop / out["raw_bf16_scan_ms"] / 1e9, 1)
    out["raw_i8_tops"] = round(flop / out["raw_i8_scan_ms"] / 1e9, 1)

    out["bf16_store_search_ms"], (s16, r16) = timeit(lambda: g._rerank_store(
        Q, S.flat_topk(g.emb16[:N], q16, 16, bias=bias, alpha=2.0)[1], 10, "l2", bias))
    out["i8_store_search_ms"], (s8, r8) = timeit(lambda: g._rerank_store(
        Q, g._i8_candidates(Q, q16, 16, bias, 2.0)[1], 10, "l2", bias))
    for stride in (32, 128, 64):
        S.CAND_STRIDE = stride
        out[f"i8_store_search_ms_stride{stride}"], _ = timeit(lambda: g._rerank_store(
            Q, g._i8_candidates(Q, q16, 16, bias, 2.0)[1], 10, "l2", bias))
    S.CAND_STRIDE = 64
    for m in (128, 200):  # small batches: bf16 lane kernel vs the int8 scan with a mostly empty query tile
        Qm, qm16 = Q[:m].contiguous(), q16[:m].contiguous()
        out[f"bf16_store_search_ms_q{m}"], (_, ra) = timeit(lambda: g._rerank_store(
            Qm, S.flat_topk(g.emb16[:N], qm16, 16, bias=bias, alpha=2.0)[1], 10, "l2", bias))
        out[f"i8_store_search_ms_q{m}"], (_, rb) = timeit(lambda: g._rerank_store(
            Qm, g._i8_candidates(Qm, qm16, 16, bias, 2.0)[1], 10, "l2", bias))
        out[f"same_rows_q{m}"] = bool(torch.equal(ra, rb))
    out["same_rows"] = bool(torch.equal(r16, r8))
    out["same_scores"] = bool(torch.equal(s16, s8))
    # candidate-list sizes of the int8 pass and the entries re-scored
    g._i8_candidates(Q, q16, 16, bias, 2.0)
    torch.cuda.synchronize()
    ws = S._ws_cand.get(dev, 0)
    c = ws[: nq * 4].view(torch.int32) & 0x3FFFFFFF
    out["i8_candidates_per_query"] = {"mean": float(c.float().mean()), "max": int(c.max())}
    cap = max(2048, 16 * 16 * 64)
    csv = ws[nq * 4: nq * 4 + nq * cap * 4].view(torch.float32).view(nq, cap)
    live = torch.arange(cap, device=dev)[None, :] < c[:, None]
    resc = (live & torch.isfinite(csv)).sum(1)
    out["i8_rescored_per_query"] = {"mean": float(resc.float().mean()), "max": int(resc.max())}
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
