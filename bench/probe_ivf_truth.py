"""Probe (diagnostic): the IVF-PQ bench's ground truth and recall on a small
mixture. Truth two ways -- the bench's per-chunk flat_topk(k=16) + fp32
re-score, and a plain fp32 matmul top-10 -- then the IVF-PQ recall against
each. Prints one JSON line."""
import json
import sys

import torch

sys.path.insert(0, "bench")
sys.path.insert(1, ".")
from bench_ivfpq_scale import Mixture  # noqa: E402
from lazzaro_amd.index.ivfpq import IVFPQIndex, recall_at_k  # noqa: E402
from lazzaro_amd.ops.search import flat_topk  # noqa: E402


def main():
    dev = torch.device("cuda", 0)
    n, chunk, d, nq = 4 << 20, 1 << 20, 1024, 1024
    mix = Mixture(d, 4000, 1.0, 1, dev)
    q = Mixture(d, 4000, 1.0, 1, dev)
    q.seed = 99
    Q = q.chunk(0, nq)
    Q16 = Q.to(torch.bfloat16)
    bs = torch.full((nq, 10), float("-inf"), device=dev)
    bi = torch.full((nq, 10), -1, dtype=torch.long, device=dev)
    es = bs.clone()
    ei = bi.clone()
    for c in range(n // chunk):
        x = mix.chunk(c, chunk)
        _, cand = flat_topk(x.to(torch.bfloat16), Q16, 16)
        s = torch.einsum("qd,qkd->qk", Q, x[cand])
        cs, ci = torch.cat([bs, s], 1), torch.cat([bi, cand + c * chunk], 1)
        o = torch.topk(cs, 10, dim=1).indices
        bs, bi = torch.gather(cs, 1, o), torch.gather(ci, 1, o)
        s2, i2 = torch.topk(Q @ x.T, 10, dim=1)
        cs, ci = torch.cat([es, s2], 1), torch.cat([ei, i2 + c * chunk], 1)
        o = torch.topk(cs, 10, dim=1).indices
        es, ei = torch.gather(cs, 1, o), torch.gather(ci, 1, o)
    agree = recall_at_k(bi, ei)
    idx = IVFPQIndex(d, nlist=1024, m=64, device=dev, keep_vectors="int8")
    tr = torch.cat([mix.chunk(c, chunk) for c in range(1)])[: 262144]
    idx.train(tr, iters=8, pq_iters=8)
    idx.reserve(n)
    for c in range(n // chunk):
        idx.add(mix.chunk(c, chunk), batch=1 << 19)
    idx._finalize()
    out = {"truth_flat_vs_fp32_recall": round(agree, 4)}
    for nprobe, rr in ((8, 1024), (8, 4096), (32, 4096)):
        _, ids = idx.search(Q, 10, nprobe=nprobe, rerank=rr)
        out[f"np{nprobe}_rr{rr}"] = {"vs_flat_truth": round(recall_at_k(ids, bi), 4),
                                     "vs_fp32_truth": round(recall_at_k(ids, ei), 4)}
    # the coarse quantiser: how often a query's true nearest row is in its probed lists
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
