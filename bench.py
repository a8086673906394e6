#!/usr/bin/env python
"""Headline benchmark (BASELINE.json config 2, tenant-sharded for N GPUs).

Metric: search_memories QPS (+ recall@10) on a 10M x d=768 index with the
bge-base-en (d=768) encoder running on-device; one step = one batch of
``--batch`` query texts per GPU going through the full search_memories path:

    native tokenizer -> bge-base forward (MFMA GEMM/attention/LN kernels)
    -> fused MFMA flat top-10 over the GPU's 10M-row HBM arena
    -> RCCL all-gather of (score, row) results to the router rank

Scaling is weak: every GPU owns its own 10M-row tenant shard (tenant-DP, the
framework's primary scale-out axis) and serves its own query stream, so the
whole-job value is the sum over GPUs. Data is synthetic: random unit vectors
for the index, synthetic query sentences, random-init encoder weights (no
checkpoints offline). recall@10 is measured outside the timed region against an
exact fp32 scan of the same rows.

Usage: python bench.py [--gpus N --steps K --warmup W]; for N>1 launch with
torch.distributed.run (one rank per GPU, RCCL backend).
"""
import argparse
import json
import os
import random
import sys
import time

import torch
import torch.distributed as dist

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "search_memories QPS + recall@10 on 10M x d=768 index; consolidate turns/sec"

WORDS = ("memory project meeting deadline client python rust family friend hobby home learn study course "
         "book tutorial health exercise diet sleep fitness travel music coffee garden kernel graph vector "
         "search index cluster agent profile language data science model train deploy server cache user "
         "prefers likes works lives started finished visited reading writing running cooking painting").split()


def synth_texts(n, rng, lo=12, hi=26):
    return [" ".join(rng.choice(WORDS) for _ in range(rng.randint(lo, hi))) + "." for _ in range(n)]


def make_index(rows, dim, dev, seed):
    g = torch.Generator(device=dev).manual_seed(seed)
    X = torch.empty((rows, dim), dtype=torch.bfloat16, device=dev)
    step = 1 << 20
    for r0 in range(0, rows, step):
        r1 = min(rows, r0 + step)
        v = torch.randn((r1 - r0, dim), device=dev, generator=g)
        X[r0:r1] = (v / v.norm(dim=1, keepdim=True)).to(torch.bfloat16)
    return X


def exact_topk(X, Q, k, chunk=1 << 21):
    best_s = best_i = None
    Qf = Q.float()
    for c0 in range(0, X.shape[0], chunk):
        s = Qf @ X[c0:c0 + chunk].float().T
        ts, ti = torch.topk(s, k, dim=1)
        ti += c0
        if best_s is None:
            best_s, best_i = ts, ti
        else:
            cs, ci = torch.cat([best_s, ts], 1), torch.cat([best_i, ti], 1)
            best_s, o = torch.topk(cs, k, dim=1)
            best_i = torch.gather(ci, 1, o)
    return best_s, best_i


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--rows", type=int, default=10_000_000, help="index rows per GPU")
    ap.add_argument("--dim", type=int, default=768)
    ap.add_argument("--batch", type=int, default=1024, help="queries per GPU per step")
    ap.add_argument("--k", type=int, default=10)
    ap.add_argument("--model", default="bge-base")
    ap.add_argument("--max-len", type=int, default=64)
    ap.add_argument("--recall-queries", type=int, default=256)
    ap.add_argument("--json-out", default="")
    ap.add_argument("--consolidate-steps", type=int, default=5,
                    help="second half of the metric: timed consolidation steps on a --rows-node buffer (0 = skip)")
    ap.add_argument("--consolidate-convs", type=int, default=128, help="conversations per GPU per step")
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
    from lazzaro_amd.ops.search import flat_topk

    # sub-batch streams of the embed (bge-base at 1024 queries: 2 fills the GEMM tail waves)
    parts = int(os.environ.get("LZK_EMBED_PARTS", "2"))
    frac = float(os.environ.get("LZK_EMBED_FRAC", "0"))  # share of sub-batch 0 (0 = equal parts)
    rng = random.Random(1234 + rank)
    emb = OnDeviceEmbedder(a.model, device=dev, max_len=a.max_len, seed=0)
    assert emb.dim == a.dim, f"model width {emb.dim} != --dim {a.dim}"
    X = make_index(a.rows, a.dim, dev, seed=100 + rank)
    pool = [synth_texts(a.batch, rng) for _ in range(4)]

    def tokenize(i):
        return emb.tok.encode_batch(pool[i % len(pool)], emb.max_len)

    # host tokenization of batch i+1 overlaps the device work of batch i
    # (serving-style pipelining; the tokenizer still runs inside the timed loop).
    # It runs after batch i's search is enqueued: in the embed's shadow (~5 ms)
    # it sometimes finished late and the search started up to 1.7 ms after the
    # embed (rocprofv3 trace, profiles/r1_bench_rocprof_v4); the search gives it ~12 ms.
    pending = {}

    def step(i):
        ids, lens = pending.pop(i) if i in pending else tokenize(i)
        _, q16 = emb.encoder.forward_streams(ids, lens, pad_to=a.dim, parts=parts, first_frac=frac)
        s, r = flat_topk(X, q16, a.k)
        if world > 1:
            out_r = torch.empty((world * r.shape[0], a.k), dtype=r.dtype, device=dev)
            out_s = torch.empty((world * s.shape[0], a.k), dtype=s.dtype, device=dev)
            dist.all_gather_into_tensor(out_r, r)
            dist.all_gather_into_tensor(out_s, s)
        pending[i + 1] = tokenize(i + 1)
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
        t = torch.tensor([el], device=dev, dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        el = float(t.item())

    # ---- untimed: component breakdown + recall@10 vs exact fp32 scan ----
    texts = pool[0]
    ids, lens = emb.tok.encode_batch(texts, emb.max_len)
    torch.cuda.synchronize()
    t1 = time.perf_counter()
    for _ in range(3):
        _, q16 = emb.encoder.forward_streams(ids, lens, pad_to=a.dim, parts=parts, first_frac=frac)
    torch.cuda.synchronize()
    t_embed = (time.perf_counter() - t1) / 3
    t1 = time.perf_counter()
    for _ in range(3):
        s, r = flat_topk(X, q16, a.k)
    torch.cuda.synchronize()
    t_search = (time.perf_counter() - t1) / 3
    nr = min(a.recall_queries, q16.shape[0])
    _, ei = exact_topk(X, q16[:nr], a.k)
    hit = sum(len(set(r[j].tolist()) & set(ei[j].tolist())) for j in range(nr))
    recall = hit / float(nr * a.k)
    S_tok = int(ids.shape[1])
    tflops_embed = emb.encoder.flops(int(lens.sum())) / t_embed / 1e12  # real (unpadded) tokens
    tflops_search = 2.0 * a.rows * a.dim * q16.shape[0] / t_search / 1e12

    qps = world * a.batch * a.steps / el

    # ---- second half of the metric: consolidate turns/sec (BASELINE config 4
    # shape: a --rows-node episodic buffer per GPU, batches of conversations
    # consolidated on device, all-to-all routing + cross-shard dedupe/links) ----
    consolidate = None
    if a.consolidate_steps > 0:
        del X
        torch.cuda.empty_cache()
        sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "bench"))
        from bench_consolidate import run as run_consolidate
        from lazzaro_amd.parallel import Communicator
        comm = Communicator() if world > 1 else Communicator.local(dev)
        consolidate = run_consolidate(comm, dev, a.rows, a.consolidate_convs, 8, a.consolidate_steps, 1, emb,
                                      dim=a.dim)
    res = {
        "metric": METRIC,
        "value": round(qps, 2),
        "unit": "queries/s",
        "n_gpus": world,
        "steps": a.steps,
        "warmup": a.warmup,
        "ms_per_step": round(el / a.steps * 1e3, 3),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "bf16",
        "data": "synthetic (random unit-vector index, synthetic query texts, random-init encoder weights)",
        "config": {"model": "bge-base-en (d=768) on-device embed + flat top-%d over %d x %d per GPU" % (a.k, a.rows, a.dim),
                   "global_batch": world * a.batch, "seq_len": S_tok, "parallelism": "tenant-dp%d" % world},
        "recall_at_10": round(recall, 4),
        "breakdown_ms": {"embed": round(t_embed * 1e3, 3), "search": round(t_search * 1e3, 3)},
        "tokens_per_query": {"padded": S_tok, "real_mean": round(float(lens.float().mean()), 2),
                             "encoder_layout": "packed varlen (padding never computed)"},
        "tflops": {"embed": round(tflops_embed, 1), "search": round(tflops_search, 1)},
    }
    if consolidate is not None:
        res["consolidate_turns_per_s"] = consolidate["turns_per_s"]
        res["consolidate"] = {k: consolidate[k] for k in ("ms_per_step", "nodes_per_rank", "convs_per_rank_step",
                                                          "facts_per_conv", "per_step_rank0")}
    if rank == 0:
        line = json.dumps(res)
        print(line, flush=True)
        if a.json_out:
            with open(a.json_out, "w") as f:
                f.write(line + "\n")
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
