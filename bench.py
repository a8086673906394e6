#!/usr/bin/env python
"""Headline benchmark (BASELINE.json config 2; tenant-DP over N GPUs).

Metric: ``search_memories`` QPS + recall@10 on a 10M x d=768 tenant, measured
through the public API. One step = one batch of ``--batch`` query texts per
GPU through ``MemorySystem.search_memories_stream`` (the pipelined form of
``search_memories_batch``; reference flow memory_system.py:1460-1472 ->
vector_store.py:132-140):

    native tokenizer -> bge-base forward on device (MFMA GEMM / attention / LN
    kernels) -> store search over the tenant's HBM rows: fused MFMA candidate
    scan (L2 = 2<q,x> - |x|^2, the store's default metric like LanceDB) +
    exact fp32 re-rank against the fp32 vectors (the reference stores fp32,
    vector_store.py:37) -> row -> Node mapping (rows the graph does not hold
    as nodes are skipped, as in the reference)

Nothing is skipped inside the timed region; host tokenisation and result
mapping of one batch overlap the device work of the next (serving pipeline).

Scaling is weak: the job is a ``DistributedMemoryService`` (one process per
GPU, RCCL); every GPU owns a 10M-row tenant (tenant-DP, the framework's
primary scale-out axis, placed by rendezvous hashing) and serves the query
stream of its tenants -- front ends route users to owners with the same hash,
so the timed path has no collective -- and the whole-job value is the sum over
GPUs. The routed path (queries for remote tenants: all-to-all there and back)
and the global cross-tenant search (all-gather + merge) are measured
separately under "serving". Data is synthetic: random unit
vectors for the stored memories, synthetic query sentences, random-init
encoder weights (no checkpoints offline).

recall@10 (outside the timed region) is measured against a float64 exact scan
of the ORIGINAL fp32 vectors, for (a) the benchmark's encoder queries and (b)
random unit queries (the random-init encoder's outputs are nearly identical,
so (a) alone would be a weak test).

The second half of the metric (consolidate turns/sec) follows in the same JSON
line (``--consolidate-steps``): ``MemorySystem.consolidate_batch`` on a
10M-memory tenant per GPU -- embed, dedupe, links, decay/prune, eviction,
run_consolidation, k-means hierarchy and the persistence commit, all timed
(bench/bench_consolidate.py).

Usage: python bench.py [--gpus N --steps K --warmup W]; for N>1 launch with
torch.distributed.run (one rank per GPU, RCCL backend).
"""
import argparse
import json
import os
import random
import sys
import tempfile
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
SHARDS = ("work", "personal", "learning", "health", "2026-10")


def synth_texts(n, rng, lo=12, hi=26):
    return [" ".join(rng.choice(WORDS) for _ in range(rng.randint(lo, hi))) + "." for _ in range(n)]


def populate(ms, rows, dim, dev, seed, chunk=1 << 20):
    """A ``rows``-memory tenant: random unit fp32 vectors written straight
    into the tenant graph's HBM columns as stored nodes (what a reload of a
    persisted tenant produces), spread over the reference's keyword shards."""
    g = ms.graph
    g._set_dim(dim)
    g.reserve(rows)
    codes = torch.tensor([g.shard_id(s) for s in SHARDS], dtype=torch.int32, device=dev)
    gen = torch.Generator(device=dev).manual_seed(seed)
    now = time.time()
    for r0 in range(0, rows, chunk):
        r1 = min(rows, r0 + chunk)
        v = torch.randn((r1 - r0, dim), device=dev, generator=gen)
        v /= v.norm(dim=1, keepdim=True)
        ids = [f"node_{i}" for i in range(r0 + 1, r1 + 1)]
        contents = [f"memory {i}" for i in range(r0 + 1, r1 + 1)]
        sh = codes[torch.arange(r0, r1, device=dev) % len(SHARDS)]
        g.add_nodes(ids, contents, v, shard=sh, stored=True, now=now, sal=0.5)
    ms.node_counter = rows
    g.clear_tracking()


def exact_l2_topk(g, Q, k, chunk=1 << 20):
    """Ground truth: float64 L2 top-k over the fp32 rows (ties -> lower row)."""
    n = g.n
    Qd = Q.double()
    best_s = best_i = None
    for c0 in range(0, n, chunk):
        c1 = min(n, c0 + chunk)
        X = g.emb32[c0:c1].double()
        s = -((Qd * Qd).sum(1, keepdim=True) - 2.0 * (Qd @ X.T) + (X * X).sum(1)[None, :])
        ts, ti = torch.topk(s, k, dim=1)
        ti += c0
        if best_s is None:
            best_s, best_i = ts, ti
        else:
            cs, ci = torch.cat([best_s, ts], 1), torch.cat([best_i, ti], 1)
            best_s, o = torch.topk(cs, k, dim=1)
            best_i = torch.gather(ci, 1, o)
    return best_s, best_i


def recall(found_rows, truth_rows):
    hit = tot = 0
    for f, t in zip(found_rows, truth_rows.tolist()):
        hit += len(set(f) & set(t))
        tot += len(t)
    return hit / max(tot, 1)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--rows", type=int, default=10_000_000, help="memories in each GPU's tenant")
    ap.add_argument("--dim", type=int, default=768)
    ap.add_argument("--batch", type=int, default=1024, help="queries per GPU per step")
    ap.add_argument("--k", type=int, default=10)
    ap.add_argument("--model", default="bge-base")
    ap.add_argument("--max-len", type=int, default=64)
    ap.add_argument("--recall-queries", type=int, default=256)
    ap.add_argument("--json-out", default="")
    ap.add_argument("--prewarm-s", type=float, default=3.0, help="untimed GPU clock ramp before the warmup steps")
    ap.add_argument("--consolidate-steps", type=int, default=10,
                    help="second half of the metric: timed consolidation steps on a --rows-node buffer (0 = skip)")
    ap.add_argument("--consolidate-convs", type=int, default=128, help="conversations per GPU per step")
    ap.add_argument("--no-persistent-graph", dest="persistent_graph", action="store_false",
                    help="skip the consolidation variant whose seeded edges are never pruned")
    ap.add_argument("--cpu", action="store_true", help="CPU / gloo dry run of the whole flow (tests only)")
    a = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    # launched by torchrun (even with one rank): the process group and every
    # collective code path are live -- a 1-rank torchrun run on one GPU
    # exercises the RCCL calls of the N-GPU job
    distributed = world > 1 or "TORCHELASTIC_RUN_ID" in os.environ
    if a.cpu:
        if distributed:
            dist.init_process_group("gloo")
        dev = torch.device("cpu")
    else:
        if distributed:
            torch.cuda.set_device(local)
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        dev = torch.device("cuda", local)
        torch.cuda.set_device(dev)

    def sync():
        if dev.type == "cuda":
            torch.cuda.synchronize()

    from lazzaro_amd.core.embedders import OnDeviceEmbedder
    from lazzaro_amd.core.memory_system import MemorySystem
    from lazzaro_amd.core.providers import LocalLLM
    from lazzaro_amd.ops.search import flat_topk
    from lazzaro_amd.parallel import Communicator
    from lazzaro_amd.parallel.service import DistributedMemoryService

    rng = random.Random(1234 + rank)
    emb = OnDeviceEmbedder(a.model, device=dev, max_len=a.max_len, seed=0)
    assert emb.dim == a.dim, f"model width {emb.dim} != --dim {a.dim}"
    # the serving layer: tenants placed on ranks by rendezvous hashing; each
    # rank's tenant is the first name the placement gives it (a real HRW
    # assignment), holding --rows memories in this GPU's HBM
    comm = Communicator() if distributed else Communicator.local(dev)
    tmp = os.environ.get("LZK_BENCH_DB") or tempfile.mkdtemp(prefix="lzbench_")

    def factory(user):
        return MemorySystem(llm_provider=LocalLLM(), embedding_provider=emb, device=dev, db_dir=tmp,
                            load_from_disk=False, enable_async=False, max_buffer_size=2 * a.rows, user_id=user)

    svc = DistributedMemoryService(comm, factory)
    tenants = {}
    for j in range(100000):
        o = svc.owner(f"tenant{j}")
        tenants.setdefault(o, f"tenant{j}")
        if len(tenants) == world:
            break
    me = tenants[rank]
    ms = svc.system(me)
    t_load = time.perf_counter()
    populate(ms, a.rows, a.dim, dev, seed=100 + rank)
    sync()
    t_load = time.perf_counter() - t_load
    g = ms.graph
    pool = [synth_texts(a.batch, rng) for _ in range(4)]

    def batches(n, start=0):
        return (pool[(start + i) % len(pool)] for i in range(n))

    # setup: bring the GPU out of its idle power state before the warmup steps
    # (on a freshly leased box the first ~seconds of work run at low clocks:
    # the same binary measured 46.6k then 56.4k QPS back to back). Untimed
    # passes of the serving loop for --prewarm-s seconds, then the W warmup steps.
    t_pre = time.perf_counter()
    while time.perf_counter() - t_pre < a.prewarm_s:
        for _ in ms.search_memories_stream(batches(4), limit=a.k):
            pass
        sync()
    t_pre = time.perf_counter() - t_pre
    for _ in ms.search_memories_stream(batches(a.warmup), limit=a.k):
        pass
    sync()
    if distributed:
        dist.barrier()
    sync()
    t0 = time.perf_counter()
    n_res = 0
    for res in ms.search_memories_stream(batches(a.steps), limit=a.k):
        n_res += len(res)
    sync()
    if distributed:
        dist.barrier()
    sync()
    el = time.perf_counter() - t0
    assert n_res == a.steps * a.batch
    if distributed:
        t = torch.tensor([el], device=dev, dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        el = float(t.item())
    qps = world * a.batch * a.steps / el

    # ---- untimed: the routed path (requests for every rank's tenant cross the
    # network: one all-to-all-v of the queries, one back with the results) and
    # a global cross-tenant search (all-gather of candidates + merge) ----
    routed = {}
    if distributed:
        reqs = [(tenants[r], "search_memories", q, a.k) for r in range(world) for q in pool[1][: a.batch // world]]
        svc.serve(reqs)
        sync()
        dist.barrier()
        t1 = time.perf_counter()
        out = svc.serve(reqs)
        sync()
        dist.barrier()
        routed["routed_search_ms"] = round((time.perf_counter() - t1) * 1e3, 3)
        routed["routed_queries_per_rank"] = len(reqs)
        assert all(len(r) == a.k for r in out)
        qv = emb.batch_embed_tensor(pool[2][:1])[0]
        svc.search_global(qv, limit=a.k)
        t1 = time.perf_counter()
        svc.search_global(qv, limit=a.k)
        routed["global_search_ms"] = round((time.perf_counter() - t1) * 1e3, 3)

    # ---- untimed: breakdown + recall vs float64 truth over the fp32 vectors ----
    def timeit(fn, n=3):
        fn()
        sync()
        t1 = time.perf_counter()
        for _ in range(n):
            out = fn()
        sync()
        return (time.perf_counter() - t1) / n * 1e3, out

    t_embed, Qe = timeit(lambda: emb.batch_embed_tensor(pool[0]))
    t_store, (_, rows_e) = timeit(lambda: g.store_search(Qe, a.k, "l2"))
    Xb = bias = q16 = None
    t_kernel = None
    if dev.type == "cuda":  # the bare candidate-scan kernel, for reference
        Xb, bias = g.emb16[: g.n], g.store_bias("l2")
        q16 = g._q16(Qe)
        t_kernel, _ = timeit(lambda: flat_topk(Xb, q16, 16, bias=bias, alpha=2.0))
    t_batch, res0 = timeit(lambda: ms.search_memories_batch(pool[0], limit=a.k))
    nr = min(a.recall_queries, a.batch)
    _, truth_e = exact_l2_topk(g, Qe[:nr], a.k)
    api_rows = [[n._r for n in r] for r in res0[:nr]]
    rec_api = recall(api_rows, truth_e)
    gen = torch.Generator(device=dev).manual_seed(999 + rank)
    Qr = torch.randn((nr, a.dim), device=dev, generator=gen)
    Qr /= Qr.norm(dim=1, keepdim=True)
    _, rows_r = g.store_search(Qr, a.k, "l2")
    _, truth_r = exact_l2_topk(g, Qr, a.k)
    rec_rand = recall(rows_r.cpu().tolist(), truth_r)
    S_tok = int(emb.tok.encode_batch(pool[0], emb.max_len)[0].shape[1])
    lens = emb.tok.encode_batch(pool[0], emb.max_len)[1]

    # ---- second half of the metric: consolidate turns/sec ----
    consolidate = persistent = None
    if a.consolidate_steps > 0:
        svc.close()
        del ms, g, Xb, bias, q16, Qe, res0, api_rows, svc
        if dev.type == "cuda":
            torch.cuda.empty_cache()
        sys.path.insert(0, os.path.join(ROOT, "bench"))
        from bench_consolidate import run as run_consolidate
        consolidate = run_consolidate(comm, dev, a.rows, a.consolidate_convs, 8, a.consolidate_steps, 1, emb,
                                      dim=a.dim)
        if a.persistent_graph:
            # same pipeline, MemorySystem(prune_threshold=0): the 2 x rows seeded
            # edges are never pruned (decay still scales every edge each
            # conversation), so decay / components / eviction's edge drops run
            # on a graph of tens of millions of edges
            if dev.type == "cuda":
                torch.cuda.empty_cache()
            persistent = run_consolidate(comm, dev, a.rows, a.consolidate_convs, 8, a.consolidate_steps, 1, emb,
                                         dim=a.dim, prune_threshold=0.0)
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
        "data": "synthetic (random unit fp32 memory vectors, synthetic query texts, random-init encoder weights)",
        "config": {"model": "%s (d=%d) on-device embed + MemorySystem.search_memories top-%d over a "
                            "%d x %d fp32 tenant per GPU (L2, fp32 re-rank)"
                            % ({"bge-base": "bge-base-en"}.get(a.model, a.model), a.dim, a.k, a.rows, a.dim),
                   "global_batch": world * a.batch, "seq_len": S_tok, "parallelism": "tenant-dp%d" % world},
        "path": "DistributedMemoryService -> owner's MemorySystem.search_memories_stream (pipelined "
                "search_memories_batch); tenants placed by rendezvous hashing, one per GPU",
        "serving": routed,
        "recall_at_10": round(rec_api, 4),
        "recall_at_10_random_queries": round(rec_rand, 4),
        "recall_truth": "float64 exact L2 over the stored fp32 vectors",
        "breakdown_ms": {"embed": round(t_embed, 3), "store_search": round(t_store, 3),
                         "raw_scan_kernel": None if t_kernel is None else round(t_kernel, 3), "search_memories_batch_unpipelined": round(t_batch, 3)},
        "tokens_per_query": {"padded": S_tok, "real_mean": round(float(lens.float().mean()), 2)},
        "load_s": round(t_load, 1),
        "prewarm_s": round(t_pre, 1),
    }
    if consolidate is not None:
        res["consolidate_turns_per_s"] = consolidate["turns_per_s"]
        res["consolidate"] = {k: consolidate[k] for k in ("ms_per_step", "nodes_per_rank", "convs_per_rank_step",
                                                          "facts_per_conv", "per_step_rank0", "nodes_rank0",
                                                          "edges_rank0", "edges_rank0_at_start", "prune_threshold",
                                                          "path", "hierarchical_clustering", "persistence")}
        res["consolidate"]["edge_lifetime_note"] = (
            "reference semantics (prune_threshold 0.5, decay 1%/conversation): a link (w <= 0.8) is pruned within "
            "47 conversations, so the seeded edges are gone after the first step and the steady state holds only "
            "the last conversations' links; see consolidate_persistent_graph for a graph that keeps its edges")
    if persistent is not None:
        res["consolidate_persistent_graph"] = {k: persistent[k] for k in (
            "turns_per_s", "ms_per_step", "per_step_rank0", "nodes_rank0", "edges_rank0_at_start", "edges_rank0",
            "prune_threshold")}
    if rank == 0:
        line = json.dumps(res)
        print(line, flush=True)
        if a.json_out:
            with open(a.json_out, "w") as f:
                f.write(line + "\n")
    if distributed:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
