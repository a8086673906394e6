"""IVF-PQ benchmark (BASELINE config 5 direction): e5-large (d=1024) query
embedding on device + IVF-PQ search, QPS and recall@10 vs the exact flat scan.

Synthetic clustered corpus (random-init encoder weights give no semantic
structure), generated on device; ground truth from the fused flat top-k over
the same rows kept in bf16 (so N is bounded by the bf16 copy, 2 KB/row).
Reports the projected capacity of the code layout on 288 GB.
"""
import argparse
import json
import os
import random
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from lazzaro_amd.index.ivfpq import IVFPQIndex, recall_at_k  # noqa: E402
from lazzaro_amd.ops.search import flat_topk  # noqa: E402


def corpus(n, d, n_centers, dev, seed, batch=1 << 20):
    g = torch.Generator(device=dev).manual_seed(seed)
    centers = torch.nn.functional.normalize(torch.randn(n_centers, d, device=dev, generator=g), dim=1)
    for r0 in range(0, n, batch):
        m = min(batch, n - r0)
        lab = torch.randint(0, n_centers, (m,), device=dev, generator=g)
        x = centers[lab] + 0.6 * torch.randn(m, d, device=dev, generator=g) / d ** 0.5
        yield torch.nn.functional.normalize(x, dim=1)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=20_000_000)
    ap.add_argument("--dim", type=int, default=1024)
    ap.add_argument("--nlist", type=int, default=8192)
    ap.add_argument("--m", type=int, default=64)
    ap.add_argument("--nq", type=int, default=1024)
    ap.add_argument("--train", type=int, default=262144)
    ap.add_argument("--model", default="e5-large")
    ap.add_argument("--nprobes", default="16,32,64")
    ap.add_argument("--rerank", type=int, default=256, help="re-rank depth over the kept copy (0 = PQ only)")
    ap.add_argument("--rerank-dtype", default="fp8", choices=["fp8", "bf16"],
                    help="re-rank copy: fp8 e4m3 + row scale (D+4 B/vector) or bf16 (2D B/vector)")
    ap.add_argument("--precision", default="fp8", choices=["fp8", "bf16"], help="query encoder projections")
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    idx = IVFPQIndex(a.dim, nlist=a.nlist, m=a.m, device=dev, keep_vectors=a.rerank_dtype if a.rerank > 0 else False)
    flat = torch.empty((a.n, a.dim), dtype=torch.bfloat16, device=dev)
    t0 = time.time()
    r0 = 0
    for x in corpus(a.n, a.dim, 100_000, dev, 1):
        flat[r0:r0 + x.shape[0]] = x.to(torch.bfloat16)
        r0 += x.shape[0]
    tr = flat[torch.randperm(a.n, device=dev)[: a.train]].float()
    idx.train(tr, iters=8, pq_iters=8)
    t_train = time.time() - t0
    t0 = time.time()
    for r0 in range(0, a.n, 1 << 21):
        idx.add(flat[r0:r0 + (1 << 21)].float())
    idx._finalize()
    torch.cuda.synchronize()
    t_add = time.time() - t0
    # queries: embed synthetic texts with e5-large (cost measured), search with
    # perturbed corpus rows so recall is meaningful
    from lazzaro_amd.core.embedders import OnDeviceEmbedder
    emb = OnDeviceEmbedder(a.model, device=dev, max_len=64, precision=a.precision)
    rng = random.Random(0)
    texts = [" ".join(rng.choice("memory user likes python graph kernel music travel".split()) for _ in range(16))
             for _ in range(a.nq)]
    ids_, lens = emb.tok.encode_batch(texts, 64)
    emb.encoder.forward_streams(ids_, lens, parts=2)
    torch.cuda.synchronize()
    t1 = time.time()
    for _ in range(3):
        emb.encoder.forward_streams(ids_, lens, parts=2)
    torch.cuda.synchronize()
    t_embed = (time.time() - t1) / 3
    g = torch.Generator(device=dev).manual_seed(9)
    qsel = torch.randint(0, a.n, (a.nq,), device=dev, generator=g)
    q = torch.nn.functional.normalize(flat[qsel].float() + 0.3 * torch.randn(a.nq, a.dim, device=dev, generator=g)
                                      / a.dim ** 0.5, dim=1)
    _, truth = flat_topk(flat, q.to(torch.bfloat16), 10)
    res = []
    for nprobe in map(int, a.nprobes.split(",")):
        for rr in sorted({0, a.rerank}):
            idx.search(q, 10, nprobe=nprobe, rerank=rr)
            torch.cuda.synchronize()
            t1 = time.time()
            for _ in range(5):
                s, ids = idx.search(q, 10, nprobe=nprobe, rerank=rr)
            torch.cuda.synchronize()
            dt = (time.time() - t1) / 5
            res.append({"nprobe": nprobe, "rerank": rr, "ms": round(dt * 1e3, 3), "qps_search": round(a.nq / dt, 1),
                        "qps_end_to_end": round(a.nq / (dt + t_embed), 1),
                        "recall_at_10": round(recall_at_k(ids, truth), 4)})
    per_vec = idx.memory_bytes() / a.n
    out = {"metric": "IVF-PQ search QPS @ recall@10", "n": a.n, "dim": a.dim, "nlist": a.nlist, "m": a.m,
           "encoder": f"{a.model} {a.precision}", "rerank_copy": a.rerank_dtype if a.rerank else None,
           "bytes_per_vector": round(per_vec, 1), "projected_vectors_in_288GB": int(270e9 / per_vec),
           "codes_only_bytes_per_vector": a.m + 8, "projected_codes_only_in_288GB": int(270e9 / (a.m + 8)),
           "train_s": round(t_train, 1), "add_s": round(t_add, 1), "add_vectors_per_s": round(a.n / t_add),
           "embed_ms_%s_%s_batch%d" % (a.model, a.precision, a.nq): round(t_embed * 1e3, 2), "results": res}
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
