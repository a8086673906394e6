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

Multi-GPU work inside the JSON line (all timed, every rank, RCCL over xGMI):

* ``serving.routed_*``: the same query stream, but each front end's queries go
  to tenants on ALL ranks ((N-1)/N remote): embed on the receiving rank, one
  all-to-all of packed [embedding | tenant key | limit] rows to the owners,
  the owners' store search, one all-to-all of [score | row] back
  (``DistributedMemoryService.search_routed``; reference per-user flow
  memory_system.py:1460-1472).
* ``serving.global_*``: every front end's queries against EVERY rank's tenant
  (all-gather of the queries, local scans, one all-to-all of the candidates
  back to their origin, merge -- SURVEY §2.5 C1 + K2).
* ``consolidate_sharded``: config 4 as ONE buffer row-sharded over the ranks
  (``ShardedMemorySystem.consolidate_batch`` at the reference's
  per-conversation cadence: facts all-gathered, top-8 candidate lists merged
  by global row, one replicated native plan of the B conversations, eviction
  and run_consolidation (distributed components) at every planned point,
  distributed k-means) on
  topic-clustered rows with cluster placement; ``scan_facts_x_rows_per_rank_step``
  is the measured per-rank scan work after the exact cone pruning (the
  unpruned figure alongside).

Usage: python bench.py [--gpus N --steps K --warmup W]. Without a torchrun
environment the script launches N ranks itself through torch.distributed.run
(127.0.0.1 rendezvous) before touching any GPU -- N = 1 included, so every
serving path runs its collectives on RCCL -- and exits with their status
(``--no-launch``: one plain process at N = 1); under torchrun, --gpus must
equal WORLD_SIZE.
"""
import argparse
import json
import os
import random
import socket
import subprocess
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


def recall_misses(g, Q, found_rows, truth_s, truth_rows, limit: int = 8):
    """The misses of a recall check: for each returned row outside the float64
    top-k, the float64 score gap between it and the k-th true row. A gap at
    the fp32 rounding level (~1e-7 of scores of magnitude ~1) is a near-tie
    that the store's fp32 ranking (the reference's LanceDB precision) may
    order either way; a larger gap would be a search error."""
    out = []
    ts = truth_s.cpu().tolist()
    for q, (f, t) in enumerate(zip(found_rows, truth_rows.tolist())):
        for r in set(f) - set(t):
            x = g.emb32[r].double()
            qd = Q[q].double()
            sc = float(-((qd - x) ** 2).sum())
            out.append({"query": q, "row": int(r), "gap_to_kth": ts[q][-1] - sc})
            if len(out) >= limit:
                return out
    return out


def _free_port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def launch_ranks(n: int) -> int:
    """Run this script as ``n`` ranks under torch.distributed.run (children;
    this process never initialises the GPU) and return their exit status."""
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
           "--master-addr", "127.0.0.1", f"--master-port={_free_port()}", os.path.abspath(__file__)] + sys.argv[1:]
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    env["PYTHONPATH"] = ROOT + (os.pathsep + env["PYTHONPATH"] if env.get("PYTHONPATH") else "")
    return subprocess.call(cmd, env=env)


HBM_PER_GPU = 288e9  # MI355X HBM3E per GPU (bytes)


def hbm_plan(rows: int, dim: int, batch: int, consolidate_convs: int, facts: int = 8, world: int = 1) -> dict:
    """Per-rank HBM plan of every section of this bench (they run one after
    another, each freeing its tenant: the job's peak is the largest section),
    from the tenant's column layout (TenantGraph.hbm_bytes_per_row) plus each
    section's large workspaces. Rows are PER RANK, so the plan does not change
    with --gpus (weak scaling) except for the row-sharded buffer's ghost rows
    (edge endpoints held elsewhere; bounded by its edges). Used by
    --hbm-check and tests/distributed/test_bench_cpu.py; the GPU run reports
    the measured peaks next to it (hbm_peak_gib)."""
    from lazzaro_amd.engine.tenant_graph import TenantGraph
    bpr = TenantGraph.hbm_bytes_per_row(dim)
    eb = TenantGraph.EDGE_BYTES
    cap = int(rows * 1.05)  # reserve slack of the loaders
    encoder = 0.5e9  # bge-base weights + activations of a 1024 x 64-token batch
    # store search: int8 queries + candidate lists (cap 2048 x 16 slots x 8 B per query) + block records
    search_ws = batch * (2048 * 16 * 8 + 4 * dim) + 256 * 8 * 2048 * 16
    # transients: the loader's 1M-row chunk (fp32 rows + the bf16 / int8
    # copies and the quantiser's fp32 temporary), and the headline's recall
    # truth (a 1M-row float64 chunk, its squared copy, and two 1,024-query
    # float64 score blocks against it: the product and its scaled copy)
    chunk = 1 << 20
    load_ws = chunk * dim * (4 + 2 + 1 + 4)
    recall_ws = chunk * dim * 8 * 2 + 2 * 1024 * chunk * 8
    head = cap * bpr + encoder + search_ws + max(load_ws, recall_ws)
    # consolidation: the tenant, 2 x rows seeded edges (+1/8 append slack), the
    # dual scan's two candidate lists, k-means (4096 centroids, per-row labels).
    # Consolidation appends every new fact as a fresh row (an evicted row is
    # not reused), so the first timed steps take the tenant past the loader's
    # capacity and TenantGraph.reserve grows every column by 1.5x: the
    # consolidation sections are planned at that grown capacity (measured:
    # 81.8 GiB for a 10M-row tenant, profiles/r6/full_bench/)
    F = consolidate_convs * facts
    dual_ws = 2 * F * (2048 * 16 * 8) + 256 * 8 * 2048 * 16 * 2
    kmeans = 4096 * dim * 6 + rows * 16
    ccap = int(cap * 1.5) + 1
    cons = ccap * bpr + 2 * rows * eb * 9 // 8 + encoder + dual_ws + kmeans + load_ws
    sharded = ccap * bpr + 2 * rows * eb * 9 // 8 + F * 2 * (bpr + 64) + encoder + dual_ws + kmeans + load_ws
    secs = {"headline": head, "consolidate": cons, "consolidate_persistent_graph": cons,
            "consolidate_sharded": sharded,
            # + the replicated stable base of the incremental digest (int32
            # endpoints + fp32 weight, and its all-gather staging at 24 B) --
            # world-sized: every rank holds every rank's stable edges
            "consolidate_sharded_persistent_graph": sharded + 2 * rows * world * (12 + 24)}
    peak = max(secs.values())
    return {"bytes_per_row": bpr, "sections_gib": {k: round(v / 2 ** 30, 2) for k, v in secs.items()},
            "peak_gib": round(peak / 2 ** 30, 2), "hbm_gib": round(HBM_PER_GPU / 2 ** 30, 2),
            "fits": peak <= 0.92 * HBM_PER_GPU}


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
    ap.add_argument("--recall-queries", type=int, default=1024)
    ap.add_argument("--json-out", default="")
    ap.add_argument("--prewarm-s", type=float, default=3.0, help="untimed GPU clock ramp before the warmup steps")
    ap.add_argument("--consolidate-steps", type=int, default=10,
                    help="second half of the metric: timed consolidation steps on a --rows-node buffer (0 = skip)")
    ap.add_argument("--consolidate-convs", type=int, default=128, help="conversations per GPU per step")
    ap.add_argument("--consolidate-calls", dest="consolidate_stream", action="store_false",
                    help="one consolidate_batch call per step instead of consolidate_stream (A/B)")
    ap.add_argument("--no-persistent-graph", dest="persistent_graph", action="store_false",
                    help="skip the consolidation variant whose seeded edges are never pruned")
    ap.add_argument("--routed-steps", type=int, default=-1, help="timed routed-search steps (-1: --steps, 0: skip)")
    ap.add_argument("--global-batch", type=int, default=128, help="queries per rank per global-search step (0: skip)")
    ap.add_argument("--sharded-steps", type=int, default=5,
                    help="timed steps of config 4 as one row-sharded buffer (--rows per rank; 0 = skip)")
    ap.add_argument("--sharded-persistent-steps", type=int, default=3,
                    help="timed steps of the row-sharded buffer with prune_threshold 0 (0 = skip)")
    ap.add_argument("--cpu", action="store_true", help="CPU / gloo dry run of the whole flow (tests only)")
    ap.add_argument("--gc-freeze", dest="gc_freeze", action="store_true",
                    help="freeze the startup heap before the timed loops (off by default: the library's results "
                         "are array-backed, so the loop allocates nothing per row; see gc_in_timed_loop)")
    ap.add_argument("--no-launch", action="store_true",
                    help="--gpus 1 without the torch.distributed.run child (no process group, no collectives)")
    ap.add_argument("--hbm-check", action="store_true",
                    help="print the per-rank HBM plan of every section for these flags (no GPU) and exit")
    a = ap.parse_args()
    if a.hbm_check:
        plan = hbm_plan(a.rows, a.dim, a.batch, a.consolidate_convs, world=a.gpus)
        print(json.dumps({"n_gpus": a.gpus, "rows_per_rank": a.rows, **plan}))
        sys.exit(0 if plan["fits"] else 1)

    # every GPU job runs as torch.distributed.run ranks -- N = 1 included, so
    # the driver's 1-GPU run times the RCCL all-to-all / all-gather calls of
    # the serving paths too; this parent never touches the GPU
    if "WORLD_SIZE" not in os.environ and (a.gpus > 1 or (a.gpus == 1 and not a.cpu and not a.no_launch)):
        sys.exit(launch_ranks(a.gpus))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if world != a.gpus:
        raise SystemExit(f"bench.py: --gpus {a.gpus} but WORLD_SIZE={world}: one rank per GPU is required")
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
            # no device_id: RCCL's communicator (its internal streams and proxy
            # thread) is created at the first GPU collective -- the serving
            # section's, after the headline loop. Created before it, it cost
            # the 1-rank headline ~6 % (the encoder and search streams then
            # overlap less; profiles/r5/README.md, ab_r4)
            dist.init_process_group("nccl")
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

    # under torch.distributed.run every exchange goes through the communicator,
    # even at world 1: the RCCL all-to-all / all-gather calls of the N-GPU job
    # run (and are timed) on one GPU
    svc = DistributedMemoryService(comm, factory, force_collectives=distributed)
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
    # the headline's own synchronisation runs on the host (gloo) group: each
    # rank serves its own tenant, and no RCCL communicator exists yet
    hg = comm._host_group if distributed else None
    if distributed:
        dist.barrier(group=hg)
    sync()
    hprof = None

    def _cg():
        out = {}
        for f in ("/sys/fs/cgroup/cpu.stat", "/sys/fs/cgroup/cpu.max"):
            try:
                out[f] = open(f).read().split()
            except OSError:
                pass
        try:
            out["threads"] = [ln for ln in open("/proc/self/status") if ln.startswith("Threads")]
        except OSError:
            pass
        out["affinity"] = len(os.sched_getaffinity(0))
        out["load"] = os.getloadavg()
        return out
    if os.environ.get("LZK_PROF_HEADLINE") == "1":  # host profile of the timed loop (stderr; diagnostic)
        import cProfile
        print("cgroup before:", _cg(), file=sys.stderr)
        hprof = cProfile.Profile()
        hprof.enable()
    # No gc.freeze() by default: a batch's results are a ResultBatch over the
    # row array (engine/views.py; NodeViews made when read), the tenant's host
    # index lives in native StrColumns, so a serving step allocates nothing
    # per row and the collector's full pass over torch's ~170k module objects
    # is not triggered inside the loop (round 5 needed the freeze: it built
    # 10k views per step, profiles/r5/headline_no_gc_freeze/). --gc-freeze
    # restores it for an A/B; gc_in_timed_loop reports the passes either way.
    import gc
    if a.gc_freeze:
        gc.collect()
        gc.freeze()
    gc_log = {0: [0, 0.0], 1: [0, 0.0], 2: [0, 0.0]}
    gc_t0 = [0.0]

    def _gc_cb(phase, info):
        if phase == "start":
            gc_t0[0] = time.perf_counter()
        else:
            e = gc_log[info["generation"]]
            e[0] += 1
            e[1] += time.perf_counter() - gc_t0[0]
    gc.callbacks.append(_gc_cb)
    t0 = time.perf_counter()
    n_res = 0
    res = None
    for res in ms.search_memories_stream(batches(a.steps), limit=a.k):
        n_res += len(res)
    sync()
    gc.callbacks.remove(_gc_cb)
    if hprof is not None:
        import pstats
        import threading
        hprof.disable()
        print("threads:", [(t.name, t.daemon) for t in threading.enumerate()], file=sys.stderr)
        print("cgroup after:", _cg(), file=sys.stderr)
        pstats.Stats(hprof, stream=sys.stderr).sort_stats("tottime").print_stats(35)
    if distributed:
        dist.barrier(group=hg)
    sync()
    el = time.perf_counter() - t0
    assert n_res == a.steps * a.batch
    if distributed:
        t = torch.tensor([el], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX, group=hg)
        el = float(t.item())
    qps = world * a.batch * a.steps / el
    if os.environ.get("LZK_BENCH_STOP_AFTER_HEADLINE") == "1":
        # profiling aid: the timed loop is the trace's last GPU work (a
        # kernel-trace window of ms_per_step x steps is exactly the loop)
        if rank == 0:
            print(json.dumps({"ms_per_step": round(el / a.steps * 1e3, 3), "steps": a.steps, "qps": round(qps, 2)}),
                  flush=True)
        return

    # ---- timed: routed search (every front end's queries spread over ALL
    # ranks' tenants: all-to-all there and back) and global search (each
    # query against every rank's tenant: all-gather + all-to-all + merge) ----
    serving = {}
    svc.embedder = emb
    comm_dev = comm.device

    def gbar():  # a barrier on the RCCL group (bound to this rank's GPU)
        dist.barrier(device_ids=[dev.index]) if dev.type == "cuda" else dist.barrier()

    def timed(n, fn):
        if distributed:
            gbar()
        sync()
        t1 = time.perf_counter()
        for i in range(n):
            fn(i)
        sync()
        if distributed:
            gbar()
        sync()
        e = time.perf_counter() - t1
        if distributed:
            t = torch.tensor([e], device=comm_dev, dtype=torch.float64)
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
            e = float(t.item())
        return e

    rsteps = a.steps if a.routed_steps < 0 else a.routed_steps
    last, gb = {}, {}  # the last routed / global results (cleared before the tenant is freed)
    if rsteps > 0:
        rr = random.Random(77 + rank)
        rusers = [[tenants[rr.randrange(world)] for _ in range(a.batch)] for _ in range(len(pool))]

        def routed_run(i0, n):
            # pipelined like the headline: batch i+1's front-end embed (the
            # receiving rank's encoder replica, no broadcast, C2) runs on a side
            # stream under batch i's routed search
            bs = [(rusers[(i0 + i) % len(pool)], pool[(i0 + i) % len(pool)]) for i in range(n)]
            for (users, texts), hits in zip(bs, svc.search_routed_stream(bs, a.k)):
                last["users"], last["hits"], last["texts"] = users, hits, texts
        routed_run(0, a.warmup)
        el_r = timed(1, lambda _: routed_run(0, rsteps))
        last["Q"] = svc._embed_front(last["texts"])
        remote = sum(svc.owner(u) != rank for u in last["users"])
        # exactness: every rank checks the queries of ALL front ends that hit
        # its own tenant against its store search (the routed rows must be the
        # owner's own top-k); 64 queries per front end
        m = min(64, a.batch)
        Qs = last["Q"][:m].float().contiguous()
        Rs = last["hits"].rows[:m].to(comm_dev).contiguous()
        own = torch.tensor([svc.owner(u) for u in last["users"][:m]], dtype=torch.int64, device=comm_dev)
        if distributed:
            Qs, Rs, own = comm.all_gather_rows(Qs.to(comm_dev)), comm.all_gather_rows(Rs), comm.all_gather_rows(own)
        mine_q = torch.nonzero(own == rank).flatten()
        agree = torch.zeros(2, dtype=torch.int64, device=comm_dev)
        if mine_q.numel():
            _, ref = g.store_search(Qs[mine_q].to(g.device), a.k, "l2")
            kind = g.kind[ref.clamp_min(0)]
            ref = torch.where((ref >= 0) & (kind == 1), ref, torch.full_like(ref, -1))
            agree[0] = int((ref.to(comm_dev) == Rs[mine_q]).all(1).sum())
            agree[1] = int(mine_q.numel())
        if distributed:
            dist.all_reduce(agree)
        serving.update({"routed_qps": round(world * a.batch * rsteps / el_r, 2),
                        "routed_ms_per_step": round(el_r / rsteps * 1e3, 3), "routed_steps": rsteps,
                        "routed_queries_per_rank": a.batch, "routed_remote_frac_rank0": round(remote / a.batch, 3),
                        "routed_exact_check": f"{int(agree[0])}/{int(agree[1])}",
                        "routed_path": "front-end embed -> all_to_all [emb|tenant|limit] -> owner store search "
                                       "(MFMA scan + fp32 re-rank) -> all_to_all [score|row]; "
                                       "DistributedMemoryService.search_routed_stream (batch i+1's embed on a "
                                       "side stream under batch i's routed search)",
                        "collectives": ("rccl (torch.distributed nccl backend, world %d; header over gloo)" % world)
                        if distributed and not a.cpu else ("gloo" if distributed else "none (world 1, no process "
                                                                                       "group)")})
    if a.global_batch > 0:
        gq = [pool[i % len(pool)][: a.global_batch] for i in range(len(pool))]

        def glob(i):
            gb["h"] = svc.search_global_batch(svc._embed_front(gq[i % len(gq)]), a.k)
        for i in range(a.warmup):
            glob(i)
        gsteps = max(1, rsteps if rsteps > 0 else a.steps)
        el_g = timed(gsteps, glob)
        serving.update({"global_qps": round(world * a.global_batch * gsteps / el_g, 2),
                        "global_ms_per_step": round(el_g / gsteps * 1e3, 3), "global_queries_per_rank": a.global_batch,
                        "global_corpus_rows": world * a.rows,
                        "global_path": "all_gather queries -> per-rank store search over its tenant -> all_to_all "
                                       "candidates to the query's origin -> merge (score desc, key asc)"})

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
    t_embed_dev = None
    if dev.type == "cuda" and hasattr(emb, "encoder"):  # the encoder alone (texts tokenised beforehand)
        from lazzaro_amd.core.embedders import EMBED_PARTS
        ids_, lens_ = emb.tok.encode_batch(pool[0], emb.max_len)
        t_embed_dev, _ = timeit(lambda: emb.encoder.forward_streams(ids_, lens_, parts=EMBED_PARTS))
    t_store, (_, rows_e) = timeit(lambda: g.store_search(Qe, a.k, "l2"))
    Xb = bias = q16 = None
    t_kernel = t_lowp = None
    if dev.type == "cuda":  # the bare candidate-scan kernel, for reference
        Xb, bias = g.emb16[: g.n], g.store_bias("l2")
        q16 = g._q16(Qe)
        t_kernel, _ = timeit(lambda: flat_topk(Xb, q16, 16, bias=bias, alpha=2.0))
        if g.emb8 is not None and g.emb8.dtype == torch.int8:  # the store search's int8 candidate pass
            t_lowp, _ = timeit(lambda: g._i8_candidates(Qe, q16, 16, bias, 2.0))
    t_batch, res0 = timeit(lambda: ms.search_memories_batch(pool[0], limit=a.k))
    nr = min(a.recall_queries, a.batch)
    _, truth_e = exact_l2_topk(g, Qe[:nr], a.k)
    api_rows = [[n._r for n in r] for r in res0[:nr]]
    rec_api = recall(api_rows, truth_e)
    gen = torch.Generator(device=dev).manual_seed(999 + rank)
    Qr = torch.randn((nr, a.dim), device=dev, generator=gen)
    Qr /= Qr.norm(dim=1, keepdim=True)
    _, rows_r = g.store_search(Qr, a.k, "l2")
    ts_r, truth_r = exact_l2_topk(g, Qr, a.k)
    rec_rand = recall(rows_r.cpu().tolist(), truth_r)
    miss_r = recall_misses(g, Qr, rows_r.cpu().tolist(), ts_r, truth_r) if rec_rand < 1.0 else []
    S_tok = int(emb.tok.encode_batch(pool[0], emb.max_len)[0].shape[1])
    lens = emb.tok.encode_batch(pool[0], emb.max_len)[1]

    # measured per-rank HBM peak of each section, next to hbm_plan's estimate,
    # and what was still allocated when the section started
    hbm_peak = {}
    hbm_start = {}

    def _release(name):
        # the previous section's tenant is freed before the next one is
        # built: its MemorySystem / graph / store objects hold reference cycles,
        # so dropping the names alone leaves ~54 GB allocated until a gen-2
        # collection happens to run (the sections' measured peaks then counted
        # two tenants)
        import gc as _gc
        _gc.collect()
        if dev.type == "cuda":
            torch.cuda.empty_cache()
            torch.cuda.reset_peak_memory_stats(dev)
            hbm_start[name] = round(torch.cuda.memory_allocated(dev) / 2 ** 30, 2)

    def peak(name):
        if dev.type == "cuda":
            hbm_peak[name] = round(torch.cuda.max_memory_allocated(dev) / 2 ** 30, 2)
            torch.cuda.reset_peak_memory_stats(dev)
    peak("headline")
    if rank == 0:
        print("bench: %s" % "headline done", file=sys.stderr, flush=True)

    # ---- second half of the metric: consolidate turns/sec ----
    consolidate = persistent = None
    if a.consolidate_steps > 0:
        svc.close()
        # every name that still reaches the headline tenant (a ResultBatch
        # holds its graph for lazy node views)
        del ms, g, Xb, bias, q16, Qe, res0, api_rows, svc, res
        last.clear()
        gb.clear()
        if dev.type == "cuda":
            _release("consolidate")
        sys.path.insert(0, os.path.join(ROOT, "bench"))
        from bench_consolidate import run as run_consolidate
        # two untimed warmup batches: the second is the first that takes the
        # stream's prefetched scan (its side-stream buffers are allocated there)
        consolidate = run_consolidate(comm, dev, a.rows, a.consolidate_convs, 8, a.consolidate_steps, 2, emb,
                                      dim=a.dim, stream=a.consolidate_stream)
        peak("consolidate")
        if a.persistent_graph:
            # same pipeline, MemorySystem(prune_threshold=0): the 2 x rows seeded
            # edges are never pruned (decay still scales every edge each
            # conversation), so decay / components / eviction's edge drops run
            # on a graph of tens of millions of edges
            if dev.type == "cuda":
                _release("consolidate_persistent_graph")
            persistent = run_consolidate(comm, dev, a.rows, a.consolidate_convs, 8, a.consolidate_steps, 2, emb,
                                         dim=a.dim, prune_threshold=0.0, stream=a.consolidate_stream)
            peak("consolidate_persistent_graph")
    sharded = None
    if a.sharded_steps > 0:
        # config 4 as ONE buffer row-sharded over the ranks: collectives in
        # every step (fact all-gather, top-3 merge, global eviction,
        # distributed components and k-means)
        if consolidate is None:
            svc.close()
        if dev.type == "cuda":
            _release("consolidate_sharded")
        sys.path.insert(0, os.path.join(ROOT, "bench"))
        from bench_consolidate import run_sharded
        # topic-clustered rows with cluster placement: the exact cone pruning
        # lets each rank skip the facts no cluster it holds can reach, so the
        # per-rank scan stays (own facts) x (own rows) as ranks are added
        sharded = run_sharded(comm, dev, a.rows, a.consolidate_convs, 8, a.sharded_steps, 1, emb, dim=a.dim,
                              clustered=True)
        peak("consolidate_sharded")
    sharded_pg = None
    if a.sharded_persistent_steps > 0:
        # the same buffer with prune_threshold 0: the 2 x rows seeded edges per
        # rank stay (decay-prune across the ranks on a graph of tens of millions
        # of edges); run_consolidation's digest is the incremental one (the
        # batch's stable base all-gathered and labelled once, the volatile
        # edges per point)
        if consolidate is None and sharded is None:
            svc.close()
        if dev.type == "cuda":
            _release("consolidate_sharded_persistent_graph")
        sys.path.insert(0, os.path.join(ROOT, "bench"))
        from bench_consolidate import run_sharded
        sharded_pg = run_sharded(comm, dev, a.rows, a.consolidate_convs, 8, a.sharded_persistent_steps, 1, emb,
                                 dim=a.dim, clustered=True, prune_threshold=0.0)
        peak("consolidate_sharded_persistent_graph")
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
        "dtype": "bf16 encoder; int8 scan -> bf16 re-score -> fp32 re-rank",
        "data": "synthetic (random unit fp32 memory vectors, synthetic query texts, random-init encoder weights)",
        "config": {"model": "%s (d=%d) on-device embed + MemorySystem.search_memories top-%d over a "
                            "%d x %d fp32 tenant per GPU (L2, fp32 re-rank)"
                            % ({"bge-base": "bge-base-en"}.get(a.model, a.model), a.dim, a.k, a.rows, a.dim),
                   "global_batch": world * a.batch, "seq_len": S_tok, "parallelism": "tenant-dp%d" % world},
        "path": "DistributedMemoryService -> owner's MemorySystem.search_memories_stream (pipelined "
                "search_memories_batch); tenants placed by rendezvous hashing, one per GPU",
        "serving": serving,
        "recall_at_10": round(rec_api, 4),
        "recall_at_10_random_queries": round(rec_rand, 4),
        "recall_queries": nr,
        "recall_misses_random": miss_r,
        "recall_truth": "float64 exact L2 over the stored fp32 vectors",
        "breakdown_ms": {"embed": round(t_embed, 3),
                         "embed_encoder_only": None if t_embed_dev is None else round(t_embed_dev, 3),
                         "store_search": round(t_store, 3),
                         "raw_scan_kernel": None if t_kernel is None else round(t_kernel, 3),
                         "i8_candidate_search": None if t_lowp is None else round(t_lowp, 3),
                         "search_memories_batch_unpipelined": round(t_batch, 3)},
        "search_precision": ("int8 MFMA candidate scan (error-model margin) -> exact bf16 re-score above the error "
                             "cut -> fp32 re-rank; recall checked against float64 truth" if t_lowp is not None else
                             "bf16 MFMA candidate scan -> fp32 re-rank; recall checked against float64 truth"),
        "tokens_per_query": {"padded": S_tok, "real_mean": round(float(lens.float().mean()), 2)},
        "load_s": round(t_load, 1),
        "gc_in_timed_loop": {"startup_heap_frozen": bool(a.gc_freeze),
                             **{f"gen{k}": {"passes": v[0], "ms": round(v[1] * 1e3, 2)} for k, v in gc_log.items()}},
        "prewarm_s": round(t_pre, 1),
        "hbm_per_rank": {"peak_gib_measured": hbm_peak, "allocated_gib_at_section_start": hbm_start,
                         "plan": hbm_plan(a.rows, a.dim, a.batch, a.consolidate_convs, world=a.gpus)},
    }
    if consolidate is not None:
        res["consolidate_turns_per_s"] = consolidate["turns_per_s"]
        res["consolidate"] = {k: consolidate[k] for k in ("ms_per_step", "nodes_per_rank", "convs_per_rank_step",
                                                          "facts_per_conv", "per_step_rank0", "nodes_rank0",
                                                          "edges_rank0", "edges_rank0_at_start", "prune_threshold",
                                                          "path", "hierarchical_clustering", "persistence")}
        if consolidate.get("stages_ms"):  # LZK_TRACE=1
            res["consolidate"]["stages_ms"] = consolidate["stages_ms"]
        res["consolidate"]["edge_lifetime_note"] = (
            "reference semantics (prune_threshold 0.5, decay 1%/conversation): a link (w <= 0.8) is pruned within "
            "47 conversations, so the seeded edges are gone after the first step and the steady state holds only "
            "the last conversations' links; see consolidate_persistent_graph for a graph that keeps its edges")
    if persistent is not None:
        res["consolidate_persistent_graph"] = {k: persistent[k] for k in (
            "turns_per_s", "ms_per_step", "per_step_rank0", "nodes_rank0", "edges_rank0_at_start", "edges_rank0",
            "prune_threshold")}
    if sharded is not None:
        res["consolidate_sharded"] = {k: sharded[k] for k in (
            "turns_per_s", "ms_per_step", "buffer_nodes_total", "nodes_per_rank", "convs_per_rank_step", "per_step",
            "scan_facts_x_rows_per_rank_step", "scan_facts_x_rows_unpruned_per_rank_step", "data", "path",
            "gc_in_timed_loop")}
        if sharded.get("stages_p50_ms"):  # LZK_TRACE=1
            res["consolidate_sharded"]["stages_p50_ms"] = sharded["stages_p50_ms"]
    if sharded_pg is not None:
        res["consolidate_sharded_persistent_graph"] = {k: sharded_pg[k] for k in (
            "turns_per_s", "ms_per_step", "buffer_nodes_total", "nodes_per_rank", "per_step", "prune_threshold",
            "edges_total_at_start", "edges_total", "incremental_digest_points", "incremental_digest_base_edges_max",
            "path", "gc_in_timed_loop")}
        if sharded_pg.get("stages_p50_ms"):
            res["consolidate_sharded_persistent_graph"]["stages_p50_ms"] = sharded_pg["stages_p50_ms"]
    from lazzaro_amd.ops import search as _S
    if _S.SPEC_STATS:  # LZK_SPEC_STATS=1 (diagnostic): queries sent to the exact fallback per store search
        res["spec_fallback_queries"] = [int(x) for x in _S.SPEC_STATS[:64]]
    if rank == 0:
        line = json.dumps(res)
        print(line, flush=True)
        if a.json_out:
            with open(a.json_out, "w") as f:
                f.write(line + "\n")
    if distributed:
        dist.barrier(group=hg)
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
