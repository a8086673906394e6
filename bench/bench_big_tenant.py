"""One very large tenant on one GPU ("sized for 288 GB"):
``--rows`` x 768 unit vectors in ONE TenantGraph with the lean HBM layout
(fp32 + int8 + row scale, no bf16 copy: ``TenantGraph.LEAN_HBM``), searched
with 1024-query batches through the store search (int8 MFMA candidate scan
-> fp32 re-score above the error cut -> fp32 L2 re-rank).

Reports the vector bytes per row, the HBM the tenant holds, store-search
QPS and recall@10 of ``--recall-queries`` queries against a float64 exact
scan of the stored fp32 rows. Synthetic data (clustered unit vectors).
Prints one JSON line."""
import argparse
import json
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def log(*a):
    print(f"[{time.strftime('%H:%M:%S')}]", *a, flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=int, default=40_000_000)
    ap.add_argument("--dim", type=int, default=768)
    ap.add_argument("--batch", type=int, default=1024)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--k", type=int, default=10)
    ap.add_argument("--recall-queries", type=int, default=256)
    ap.add_argument("--no-lean", dest="lean", action="store_false")
    ap.add_argument("--out", default="")
    a = ap.parse_args()
    from lazzaro_amd.engine import tenant_graph as TG
    TG.TenantGraph.LEAN_HBM = a.lean
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    N, D = a.rows, a.dim
    g = TG.TenantGraph(device=dev, dim=D, capacity=N)
    code = g.shard_id("default")
    gen = torch.Generator(device=dev).manual_seed(3)
    C = torch.randn(4096, D, device=dev, generator=gen)
    C /= C.norm(dim=1, keepdim=True)
    t0 = time.time()
    chunk = 1 << 21
    for c0 in range(0, N, chunk):
        c1 = min(N, c0 + chunk)
        X = C[torch.randint(0, 4096, (c1 - c0,), device=dev, generator=gen)] + 0.05 * torch.randn(
            c1 - c0, D, device=dev, generator=gen)
        X /= X.norm(dim=1, keepdim=True)
        g.add_nodes([f"n{i}" for i in range(c0, c1)], [""] * (c1 - c0), X, shard=code, stored=True)
        if (c0 // chunk) % 4 == 0:
            log(f"{c1:,} rows ({time.time() - t0:.0f}s), HBM {torch.cuda.memory_allocated(dev) / 2**30:.1f} GiB")
    torch.cuda.synchronize()
    t_load = time.time() - t0
    cols = [g.emb32, g.emb16, g.emb8, g.rs8, g.sqn]
    vec_bytes = sum(t[0].numel() * t.element_size() for t in cols if t is not None)
    node_bytes = sum(getattr(g, c)[0].numel() * getattr(g, c).element_size() for c, _, _ in TG.TenantGraph.NODE_COLS)
    Qs = [C[torch.randint(0, 4096, (a.batch,), device=dev, generator=gen)]
          + 0.06 * torch.randn(a.batch, D, device=dev, generator=gen) for _ in range(a.steps + 2)]
    Qs = [q / q.norm(dim=1, keepdim=True) for q in Qs]
    g.store_search(Qs[0], a.k)  # warm
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(a.steps):
        s, r = g.store_search(Qs[1 + i], a.k)
    torch.cuda.synchronize()
    el = time.perf_counter() - t0
    # recall against float64 exact L2 over the stored fp32 rows
    Qr = Qs[-1][: a.recall_queries]
    _, rows = g.store_search(Qr, a.k)
    Qd = Qr.double()
    best_v = best_i = None
    for c0 in range(0, N, 1 << 20):
        Xd = g.emb32[c0:c0 + (1 << 20)].double()
        sc = 2 * Qd @ Xd.T - (Xd * Xd).sum(1)[None, :]
        v, i = torch.topk(sc, a.k, dim=1)
        i = i + c0
        if best_v is None:
            best_v, best_i = v, i
        else:
            v, i = torch.cat([best_v, v], 1), torch.cat([best_i, i], 1)
            o = torch.topk(v, a.k, dim=1).indices
            best_v, best_i = torch.gather(v, 1, o), torch.gather(i, 1, o)
    hit = sum(len(set(x) & set(y)) for x, y in zip(rows.cpu().tolist(), best_i.cpu().tolist()))
    res = {"metric": "store_search QPS, one large tenant", "rows": N, "dim": D, "lean_hbm": bool(g.lean),
           "value": round(a.batch * a.steps / el, 1), "unit": "queries/s", "ms_per_batch": round(el / a.steps * 1e3, 3),
           "batch": a.batch, "k": a.k, "recall_at_10": round(hit / (len(Qr) * a.k), 4),
           "recall_queries": len(Qr), "recall_truth": "float64 exact L2 over the stored fp32 rows",
           "vector_bytes_per_row": vec_bytes, "node_column_bytes_per_row": node_bytes,
           "tenant_hbm_gib": round((vec_bytes + node_bytes) * g.cap / 2**30, 1),
           "hbm_allocated_gib": round(torch.cuda.memory_allocated(dev) / 2**30, 1), "load_s": round(t_load, 1),
           "path": "TenantGraph.store_search: int8 MFMA candidate scan -> fp32 re-score above the error "
                   "cut (lzk_cand_rescore32) -> fp32 L2 re-rank" if g.lean else
                   "TenantGraph.store_search: int8 scan -> bf16 re-score -> fp32 re-rank",
           "data": "synthetic clustered unit vectors (4096 centres)"}
    print(json.dumps(res), flush=True)
    if a.out:
        with open(a.out, "w") as f:
            f.write(json.dumps(res) + "\n")


if __name__ == "__main__":
    main()
