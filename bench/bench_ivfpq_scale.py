"""IVF-PQ at BASELINE config-5 scale: an index that fills most of one MI355X's
288 GB -- N x 1024 clustered vectors (default 200M) with PQ codes (m=64) and an
int8 re-rank copy (1024 + 4 B/vector) -- swept over nprobe and re-rank depth:
QPS vs recall@10 against the exact fp32 inner product.

Data: a Gaussian mixture (``--clusters`` unit centres, points = centre +
N(0, noise^2/d) per dimension, unit-normalised), generated on the GPU chunk by
chunk from per-chunk seeds, so the exact ground truth is computed by
regenerating every chunk (never held whole): per chunk a bf16 top-16 by the
fused flat scan, re-scored in fp32, merged into a running top-10. Queries are
fresh draws from the same mixture. Synthetic data (no dataset access).

Prints progress lines and one JSON result line; ``--out`` also writes it.
"""
import argparse
import json
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from lazzaro_amd.index.ivfpq import IVFPQIndex, recall_at_k  # noqa: E402
from lazzaro_amd.ops.search import flat_topk  # noqa: E402


def log(*a):
    print(f"[{time.strftime('%H:%M:%S')}]", *a, flush=True)


class Mixture:
    """Gaussian mixture. ``intrinsic`` = 0: isotropic in all d dimensions
    (every direction carries cluster noise -- product quantisation's worst
    case); ``intrinsic`` = k > 0: the mixture lives in a random k-dimensional
    subspace (orthonormal basis P) plus a small isotropic ambient term
    (``ambient`` of the energy) -- the low intrinsic dimensionality that
    learned embeddings have."""

    def __init__(self, d, clusters, noise, seed, dev, intrinsic=0, ambient=0.1):
        self.d, self.noise, self.seed, self.dev = d, noise, seed, dev
        self.k, self.ambient = intrinsic or d, ambient if intrinsic else 0.0
        g = torch.Generator(device=dev).manual_seed(seed)
        self.centers = torch.nn.functional.normalize(torch.randn(clusters, self.k, device=dev, generator=g), dim=1)
        self.P = None
        if intrinsic:
            q, _ = torch.linalg.qr(torch.randn(d, self.k, device=dev, generator=g))
            self.P = q.T.contiguous()  # [k, d]

    def chunk(self, c, m):
        """Chunk ``c`` of ``m`` points (deterministic in (seed, c))."""
        g = torch.Generator(device=self.dev).manual_seed(self.seed * 1_000_003 + 7919 * (c + 1))
        lab = torch.randint(0, self.centers.shape[0], (m,), device=self.dev, generator=g)
        z = self.centers[lab]
        z += torch.randn(m, self.k, device=self.dev, generator=g).mul_(self.noise / self.k ** 0.5)
        if self.P is None:
            return torch.nn.functional.normalize(z, dim=1)
        x = torch.nn.functional.normalize(z, dim=1) @ self.P
        x += torch.randn(m, self.d, device=self.dev, generator=g).mul_(self.ambient / self.d ** 0.5)
        return torch.nn.functional.normalize(x, dim=1)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=200_000_000)
    ap.add_argument("--dim", type=int, default=1024)
    ap.add_argument("--clusters", type=int, default=100_000)
    ap.add_argument("--noise", type=float, default=1.0)
    ap.add_argument("--intrinsic", type=int, default=0, help="mixture subspace dimension (0 = isotropic)")
    ap.add_argument("--ambient", type=float, default=0.1)
    ap.add_argument("--nlist", type=int, default=16384)
    ap.add_argument("--m", type=int, default=64)
    ap.add_argument("--keep", default="int8", choices=["int8", "fp8", "bf16"])
    ap.add_argument("--train", type=int, default=4_194_304,
                    help="coarse k-means training rows (~256 per list: 524k left the lists too coarse, coarse recall 0.66)")
    ap.add_argument("--nq", type=int, default=1024)
    ap.add_argument("--chunk", type=int, default=1 << 20)
    ap.add_argument("--nprobes", default="16,32,64,128")
    ap.add_argument("--reranks", default="0,256,1024")
    ap.add_argument("--embed-model", default="e5-large", help="query encoder timed per batch ('' = none)")
    ap.add_argument("--embed-precision", default="fp8", choices=["fp8", "bf16"])
    ap.add_argument("--pipeline", default="8,4096",
                    help="nprobe,rerank of the pipelined embed + search run ('' = skip): batch i+1's embed on one "
                         "stream under batch i's search on another (each search waits for its batch's embed)")
    ap.add_argument("--pipeline-reps", type=int, default=10)
    ap.add_argument("--out", default="")
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    mix = Mixture(a.dim, a.clusters, a.noise, 1, dev, a.intrinsic, a.ambient)
    n_chunks = (a.n + a.chunk - 1) // a.chunk
    sizes = [min(a.chunk, a.n - c * a.chunk) for c in range(n_chunks)]

    idx = IVFPQIndex(a.dim, nlist=a.nlist, m=a.m, device=dev, keep_vectors=a.keep)
    t0 = time.time()
    tr = torch.cat([mix.chunk(c, sizes[c]) for c in range(max(1, -(-a.train // a.chunk)))])[: a.train]
    idx.train(tr, iters=8, pq_iters=8)
    del tr
    torch.cuda.synchronize()
    t_train = time.time() - t0
    log(f"trained nlist={a.nlist} m={a.m} in {t_train:.1f}s")
    idx.reserve(a.n)
    t0 = time.time()
    for c in range(n_chunks):
        idx.add(mix.chunk(c, sizes[c]), batch=1 << 19)
        if c % 10 == 0:
            torch.cuda.synchronize()
            log(f"added {sum(sizes[:c + 1]):,} / {a.n:,}  ({time.time() - t0:.0f}s, "
                f"{torch.cuda.memory_allocated() / 2**30:.0f} GiB)")
    idx._finalize()
    torch.cuda.synchronize()
    t_add = time.time() - t0
    log(f"built {a.n:,} vectors in {t_add:.0f}s; index {idx.memory_bytes() / 1e9:.1f} GB")

    q = Mixture(a.dim, a.clusters, a.noise, 1, dev, a.intrinsic, a.ambient)
    q.seed = 99  # same centres and subspace, fresh points
    Q = q.chunk(0, a.nq)
    Q16 = Q.to(torch.bfloat16)
    best_s = torch.full((a.nq, 10), float("-inf"), device=dev)
    best_i = torch.full((a.nq, 10), -1, dtype=torch.long, device=dev)
    t0 = time.time()
    off = 0
    for c in range(n_chunks):
        x = mix.chunk(c, sizes[c])
        _, cand = flat_topk(x.to(torch.bfloat16), Q16, 16)
        s = torch.einsum("qd,qkd->qk", Q, x[cand])
        cs, ci = torch.cat([best_s, s], 1), torch.cat([best_i, cand + off], 1)
        o = torch.topk(cs, 10, dim=1).indices
        best_s, best_i = torch.gather(cs, 1, o), torch.gather(ci, 1, o)
        off += sizes[c]
        del x
        if c % 20 == 0:
            log(f"truth {off:,} / {a.n:,}")
    torch.cuda.synchronize()
    log(f"exact truth in {time.time() - t0:.0f}s")

    # the query side of config 5: e5-large (d=1024) on-device embed of nq
    # synthetic texts, timed; the search itself uses mixture queries (a
    # random-init encoder maps every text to nearly one vector, so recall
    # needs controlled query vectors)
    t_embed = 0.0
    if a.embed_model:
        import random as _r

        from lazzaro_amd.core.embedders import OnDeviceEmbedder
        enc = OnDeviceEmbedder(a.embed_model, device=dev, max_len=64, precision=a.embed_precision)
        rr = _r.Random(0)
        words = "memory user likes python graph kernel music travel project deadline family".split()
        texts = [" ".join(rr.choice(words) for _ in range(16)) for _ in range(a.nq)]
        enc.batch_embed_tensor(texts)
        torch.cuda.synchronize()
        t1 = time.time()
        for _ in range(3):
            enc.batch_embed_tensor(texts)
        torch.cuda.synchronize()
        t_embed = (time.time() - t1) / 3
        log(f"{a.embed_model} {a.embed_precision} embed of {a.nq} queries: {t_embed * 1e3:.2f} ms")
    res = []
    # the coarse quantiser's share of the recall: how many true top-10 rows sit
    # in one of the query's probed lists (row -> list through the sorted layout)
    inv = torch.empty_like(idx._pos[: idx.n])
    inv[idx._pos[: idx.n]] = torch.arange(idx.n, device=dev)
    truth_list = idx._list[: idx.n][inv[best_i.clamp_min(0)]]
    cs_q = torch.nn.functional.normalize(Q.float(), dim=1) @ idx.centroids.T
    for nprobe in map(int, a.nprobes.split(",")):
        pr = torch.topk(cs_q, nprobe, dim=1).indices
        hit = (truth_list[:, :, None] == pr[:, None, :].to(truth_list.dtype)).any(-1)
        log(f"nprobe {nprobe}: coarse recall@10 {float(hit.float().mean()):.4f}")
        for rr in map(int, a.reranks.split(",")):
            idx.search(Q, 10, nprobe=nprobe, rerank=rr)
            torch.cuda.synchronize()
            t1 = time.time()
            for _ in range(3):
                _, ids = idx.search(Q, 10, nprobe=nprobe, rerank=rr)
            torch.cuda.synchronize()
            dt = (time.time() - t1) / 3
            r = {"nprobe": nprobe, "rerank": rr, "ms_per_batch": round(dt * 1e3, 2), "qps": round(a.nq / dt, 1),
                 "recall_at_10": round(recall_at_k(ids, best_i), 4)}
            if t_embed:
                r["qps_with_embed"] = round(a.nq / (dt + t_embed), 1)
            lc = getattr(idx, "last_candidates", None)
            if rr > 16 and lc is not None:
                cap = max(idx.CAND_CAP * rr, idx.CAND_MIN)
                r["threshold_rows_mean"] = round(float(lc.float().mean()), 1)
                r["overflow_queries"] = int((lc > cap).sum())
            res.append(r)
            log(json.dumps(r))
    pipe = None
    if a.embed_model and a.pipeline:
        # end to end, pipelined: the embed of batch i+1 (stream A) runs under
        # the search of batch i (stream B); search i waits for embed i's event
        # (the mixture queries stand in for its vectors, see above)
        nprobe, rr = (int(x) for x in a.pipeline.split(","))
        sA, sB = torch.cuda.Stream(), torch.cuda.Stream()

        def run(R):
            evs = []
            for i in range(R + 1):
                if i < R:
                    with torch.cuda.stream(sA):
                        enc.batch_embed_tensor(texts)
                        ev = torch.cuda.Event()
                        ev.record(sA)
                        evs.append(ev)
                if i > 0:
                    with torch.cuda.stream(sB):
                        sB.wait_event(evs[i - 1])
                        _, ids_p = idx.search(Q, 10, nprobe=nprobe, rerank=rr)
            torch.cuda.synchronize()
            return ids_p
        run(2)
        t1 = time.time()
        ids_p = run(a.pipeline_reps)
        dt = time.time() - t1
        pipe = {"nprobe": nprobe, "rerank": rr, "batches": a.pipeline_reps,
                "ms_per_batch": round(dt / a.pipeline_reps * 1e3, 2),
                "qps_e2e_pipelined": round(a.pipeline_reps * a.nq / dt, 1),
                "recall_at_10": round(recall_at_k(ids_p, best_i), 4),
                "path": "embed (e5-large) on stream A, IVF-PQ search on stream B, batch i+1's embed under batch i's search"}
        log(json.dumps(pipe))
    out = {"metric": "IVF-PQ QPS vs recall@10 (exact fp32 truth)", "n": a.n, "dim": a.dim,
           "data": (f"synthetic Gaussian mixture, {a.clusters} clusters, noise {a.noise}, "
                    + (f"in a random {a.intrinsic}-d subspace + {a.ambient} ambient noise, " if a.intrinsic
                       else "isotropic, ") + "unit-normalised"),
           "nlist": a.nlist, "m": a.m, "rerank_copy": a.keep, "nq": a.nq,
           "index_bytes": idx.memory_bytes(), "bytes_per_vector": round(idx.memory_bytes() / a.n, 1),
           "hbm_allocated_gib": round(torch.cuda.max_memory_allocated() / 2**30, 1),
           "train_s": round(t_train, 1), "build_s": round(t_add, 1),
           "query_embed": {"model": a.embed_model, "precision": a.embed_precision,
                           "ms_per_batch": round(t_embed * 1e3, 2)} if a.embed_model else None,
           "results": res, "pipelined_e2e": pipe}
    line = json.dumps(out)
    print(line, flush=True)
    if a.out:
        with open(a.out, "w") as f:
            f.write(line + "\n")


if __name__ == "__main__":
    main()
