"""BASELINE config 3: multi-tenant serving -- 100k users partitioned across the
GPUs of a node (tenant-DP by rendezvous hashing), each query searching only
its own user's memories, results gathered across ranks (RCCL all-gather, C1).

Per rank: the tenants it owns live contiguously in one HBM arena (bf16,
SURVEY.md §2.4 K3 "tenant segments"); a step embeds a batch of synthetic
queries from random local users with the on-device bge-base encoder and runs
ONE segment-kernel launch for the whole batch (every query scans its user's
rows only), then all-gathers (score, global row) to rank 0. Exact: recall vs
a torch fp32 scan of each queried user's rows is reported.

    python bench/bench_multitenant.py                       # 1 GPU: 100k/8 users
    torchrun --nproc-per-node 8 ... bench/bench_multitenant.py --gpus 8
Synthetic data and random-init encoder weights.
"""
import argparse
import json
import os
import random
import sys
import time

import torch
import torch.distributed as dist

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

WORDS = ("memory user likes python graph kernel music travel coffee tea rust async team project deadline "
         "sister brother city moved learning guitar piano book novel running marathon cooking garden").split()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--users", type=int, default=100_000, help="users in the whole job")
    ap.add_argument("--rows-per-user", type=int, default=800, help="mean memories per user (uniform 1/2x..3/2x)")
    ap.add_argument("--batch", type=int, default=1024, help="queries per GPU per step")
    ap.add_argument("--dim", type=int, default=768)
    ap.add_argument("--k", type=int, default=10)
    ap.add_argument("--model", default="bge-base")
    ap.add_argument("--max-len", type=int, default=64)
    a = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    dev = torch.device("cuda", local)
    torch.cuda.set_device(dev)

    from lazzaro_amd.core.embedders import OnDeviceEmbedder
    from lazzaro_amd.ops.search import segment_topk_ptrs
    from lazzaro_amd.parallel.placement import tenant_rank

    # ---- placement: the users this rank owns (rendezvous hashing) ----
    users = [f"user{i}" for i in range(a.users)]
    mine = [u for u in users if tenant_rank(u, world) == rank] if world > 1 else users[: a.users // 8]
    rng = random.Random(7 + rank)
    counts = [rng.randint(a.rows_per_user // 2, a.rows_per_user * 3 // 2) for _ in mine]
    off = [0]
    for c in counts:
        off.append(off[-1] + c)
    N = off[-1]
    g = torch.Generator(device=dev).manual_seed(100 + rank)
    X = torch.empty((N, a.dim), dtype=torch.bfloat16, device=dev)
    for r0 in range(0, N, 1 << 20):
        x = torch.randn(min(1 << 20, N - r0), a.dim, device=dev, generator=g)
        X[r0:r0 + x.shape[0]] = torch.nn.functional.normalize(x, dim=1).to(torch.bfloat16)
    base = X.data_ptr()
    row_bytes = X.stride(0) * X.element_size()
    t_ptr = torch.tensor([base + o * row_bytes for o in off[:-1]], dtype=torch.int64, device=dev)
    t_n = torch.tensor(counts, dtype=torch.int32, device=dev)
    t_off = torch.tensor(off[:-1], dtype=torch.int64, device=dev)

    emb = OnDeviceEmbedder(a.model, device=dev, max_len=a.max_len, seed=0)
    texts = [[" ".join(rng.choice(WORDS) for _ in range(12)) for _ in range(a.batch)] for _ in range(4)]
    tsel = [torch.randint(0, len(mine), (a.batch,), device=dev, generator=g) for _ in range(4)]
    pending = {}

    def tok(i):
        return emb.tok.encode_batch(texts[i % 4], emb.max_len)

    def step(i):
        ids, lens = pending.pop(i) if i in pending else tok(i)
        _, q16 = emb.encoder.forward(ids, lens, pad_to=a.dim)
        pending[i + 1] = tok(i + 1)
        t = tsel[i % 4]
        s, r = segment_topk_ptrs(t_ptr[t], t_n[t], X.stride(0), q16, a.k)
        grow = torch.where(r >= 0, r + t_off[t][:, None], r)  # global row ids
        if world > 1:
            out_s = torch.empty((world * a.batch, a.k), dtype=s.dtype, device=dev)
            out_r = torch.empty((world * a.batch, a.k), dtype=grow.dtype, device=dev)
            dist.all_gather_into_tensor(out_s, s)
            dist.all_gather_into_tensor(out_r, grow)
        return q16, s, r

    for i in range(a.warmup):
        step(i)
    pending.clear()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(a.steps):
        step(i)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    el = time.perf_counter() - t0
    if world > 1:
        tt = torch.tensor([el], device=dev, dtype=torch.float64)
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        el = float(tt.item())

    # ---- untimed: breakdown + exactness vs torch fp32 per user ----
    ids, lens = tok(0)
    torch.cuda.synchronize()
    t1 = time.perf_counter()
    for _ in range(3):
        _, q16 = emb.encoder.forward(ids, lens, pad_to=a.dim)
    torch.cuda.synchronize()
    t_embed = (time.perf_counter() - t1) / 3
    t = tsel[0]
    tp, tn = t_ptr[t], t_n[t]
    t1 = time.perf_counter()
    for _ in range(10):
        s, r = segment_topk_ptrs(tp, tn, X.stride(0), q16, a.k)
    torch.cuda.synchronize()
    t_search = (time.perf_counter() - t1) / 10
    hit = tot = 0
    tl = t.cpu().tolist()
    for j in range(0, a.batch, max(1, a.batch // 64)):
        u = tl[j]
        Xu = X[off[u]:off[u + 1]].float()
        ref = torch.topk(Xu @ q16[j].float(), min(a.k, Xu.shape[0])).indices.tolist()
        got = [x for x in r[j].tolist() if x >= 0]
        hit += len(set(ref) & set(got))
        tot += len(ref)
    scanned = float(tn.sum().item()) * X.stride(0) * 2
    res = {"metric": "multi-tenant search_memories QPS (per-user scan, 100k users)", "value": round(world * a.batch * a.steps / el, 1),
           "unit": "queries/s", "n_gpus": world, "steps": a.steps, "warmup": a.warmup,
           "ms_per_step": round(el / a.steps * 1e3, 3), "higher_is_better": True, "scaling": "weak",
           "dtype": "bf16", "data": "synthetic users/memories/queries, random-init bge-base",
           "config": {"users_total": a.users, "users_per_gpu": len(mine), "rows_per_gpu": N,
                      "rows_per_user_mean": a.rows_per_user, "global_batch": world * a.batch, "k": a.k,
                      "parallelism": "tenant-dp%d" % world},
           "recall_at_10": round(hit / max(1, tot), 4),
           "breakdown_ms": {"embed": round(t_embed * 1e3, 3), "segment_search": round(t_search * 1e3, 3)},
           "segment_scan_GBps": round(scanned / t_search / 1e9, 1)}
    if rank == 0:
        print(json.dumps(res), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
