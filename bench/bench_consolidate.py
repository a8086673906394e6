"""Consolidation at scale (BASELINE.json config 4) through the product API.

Each GPU owns one large tenant (``--nodes`` memories, tenant-DP: the
framework's scale-out axis, so per-GPU work is independent of the GPU count)
held by a ``MemorySystem(device=cuda)``. One step = ``--convs`` finished
conversations of that tenant, ``--facts`` extracted facts each, consolidated by
``MemorySystem.consolidate_batch`` -- the batched form of the reference's
``end_conversation`` (memory_system.py:580-649, :651-933), equal to B
sequential calls (tests/unit/test_memory_system.py):

  1. embed the fact texts with the on-device encoder (bge-base, MFMA kernels)
  2. ONE fused scan of the facts against the 10M-row tenant: dedupe top-1,
     within-shard and cross-memory top-3 (bf16 MFMA candidates, float64
     re-rank), plus the in-batch block for earlier conversations
  3. duplicate merges, inserts, chain / similarity links with per-edge decay
     for the conversations that follow them, decay + prune of the whole
     graph by (1-r)^B (``tg_decay_kernel``)
  4. eviction to ``max_buffer_size`` (``tg_importance_kernel`` + select +
     ``tg_flag_remove``): the buffer is full, so every step evicts
  5. ``run_consolidation`` (reference default: every 3 conversations):
     connected components (``cc_hook``/``cc_compress``) + component digest +
     profile, prune
  6. hierarchy_mode="kmeans": the two-level k-means hierarchy (4096 fine /
     64 topic clusters, MFMA argmax assign + sorted segment sums) every
     ``--cluster-every`` steps, inside the timed loop
  7. incremental persistence commit of the changed rows / edges / deletions
     to the columnar store on disk

Fact *texts* are embedded (the cost is paid inside the timed step) but the
vectors ingested are synthetic controlled ones -- perturbations of existing
memories with a fixed duplicate rate -- because random-init encoder weights
map every text to nearly the same vector, which would make dedupe degenerate.

Edge lifetime under the reference semantics: a link starts at w = 0.8*cos <=
0.8, is never re-added by consolidation, and decays by 0.99 per
conversation, so it is pruned (< 0.5) within 46 conversations of its tenant.
With 128 conversations per step the steady-state graph holds the links of the
tenant's last ~46 conversations (plus whatever the initial edges leave).

turns/sec = conversations consolidated per second over all ranks.
"""
from __future__ import annotations

import contextlib
import math
import os
import random
import sys
import tempfile
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

SHARDS = ("work", "personal", "learning", "health", "2026-10")
WORDS = "user likes prefers works lives started visited learned project team python rust garden music".split()


@contextlib.contextmanager
def _ff_timer():
    """Device time of the farthest-first seeding inside the cold cluster pass
    (the ``ff_seed`` tracer stage, index/kmeans.py); the rest of the cold
    pass is the k-means iterations over every row."""
    from lazzaro_amd.utils.tracing import tracer
    was = tracer.enabled
    tracer.enable(True)
    out = {}
    try:
        yield out
    finally:
        st = tracer.summary().get("ff_seed")
        out["ms"] = round(st["total_ms"], 1) if st else None
        if not was:
            tracer.reset()
        tracer.enable(was)


def _unit(x):
    return x / x.norm(dim=1, keepdim=True).clamp_min(1e-30)


def build_tenant(dev, nodes: int, dim: int, encoder, seed: int, db_dir: str, cluster_convs: int, n_fine: int,
                 n_top: int, cluster_iters: int, init_edges: int, prune_threshold: float = 0.5,
                 persist_async: bool = False):
    from bench import populate  # the headline bench's tenant loader
    from lazzaro_amd.core.memory_system import MemorySystem
    from lazzaro_amd.core.providers import HashEmbedder, LocalLLM

    ms = MemorySystem(llm_provider=LocalLLM(), embedding_provider=encoder or HashEmbedder(dim=dim), device=dev,
                      db_dir=db_dir, load_from_disk=False, enable_async=False, max_buffer_size=nodes,
                      prune_threshold=prune_threshold, persist_async=persist_async, hierarchy_mode="kmeans", hierarchy_params={"fine": n_fine, "top": n_top,
                                                                 "every": cluster_convs, "iters": cluster_iters})
    g = ms.graph
    g._set_dim(dim)
    g.reserve(int(nodes * 1.02) + 4096)  # inserts get fresh rows: headroom so the timed steps never re-allocate
    populate(ms, nodes, dim, dev, seed=seed)
    if init_edges:
        gen = torch.Generator(device=dev).manual_seed(seed + 1)
        src = torch.randint(0, nodes, (init_edges,), device=dev, generator=gen)
        dst = torch.randint(0, nodes, (init_edges,), device=dev, generator=gen)
        w = torch.rand(init_edges, device=dev, generator=gen) * 0.5 + 0.5
        g.append_edges(src.int(), dst.int(), w, g.shard[src], g.etype("relates_to"))
    g.clear_tracking(stored=False)  # the synthetic edges are not in the store
    return ms


def synth_facts(convs: int, facts: int, rng):
    """The extraction LLM's output for ``convs`` conversations (fact dicts).
    Generated before the timed loop: it stands in for the LLM, it is not
    engine work."""
    return [[{"content": " ".join(rng.choice(WORDS) for _ in range(12)), "type": "semantic",
              "salience": round(rng.uniform(0.4, 0.95), 3), "topic": rng.choice(SHARDS)} for _ in range(facts)]
            for _ in range(convs)]


def synth_vectors(ms, n: int, dim: int, dup_rate: float, gen):
    """Controlled fact vectors: a duplicate (cos ~0.995) or a related memory
    (cos ~0.64) of a random live row of the tenant's CURRENT graph."""
    g = ms.graph
    dev = g.device
    base_rows = torch.randint(0, g.n, (n,), device=dev, generator=gen)
    base = g.emb32[base_rows].float()
    noise = torch.randn((n, dim), device=dev, generator=gen) / (dim ** 0.5)
    is_dup = torch.rand(n, device=dev, generator=gen) < dup_rate
    return torch.where(is_dup[:, None], _unit(base + 0.1 * noise), _unit(base + 1.2 * noise))



def _sync(dev):
    if dev.type == "cuda":
        torch.cuda.synchronize(dev)


def run(comm, dev, nodes: int, convs: int, facts: int, steps: int, warmup: int, encoder=None, dim: int = 768,
        dup_rate: float = 0.1, seed: int = 7, cluster_every: int = 5, n_fine: int = 4096, n_top: int = 64,
        cluster_iters: int = 2, init_edges: int = None, db_dir: str = None, prune_threshold: float = 0.5,
        persist_async: bool = False, stream: bool = True, lookahead: int = 2):
    """``stream``: the batches go through ``MemorySystem.consolidate_stream``
    (batch i+1's candidate scan under batch i's apply; results identical to
    the per-batch calls, tests/kernels/test_tenant_engine_gpu.py); False:
    one ``consolidate_batch`` call per step."""
    db_dir = db_dir or tempfile.mkdtemp(prefix=f"lzcons{comm.rank}_")
    init_edges = 2 * nodes if init_edges is None else init_edges
    ms = build_tenant(dev, nodes, dim, encoder, seed + 31 * comm.rank, db_dir, cluster_every * convs, n_fine, n_top,
                      cluster_iters, init_edges, prune_threshold, persist_async)
    edges_start = ms.graph.num_edges
    gen = torch.Generator(device=dev).manual_seed(seed + 100 + comm.rank)
    rng = random.Random(seed + comm.rank)
    # the first k-means pass seeds the hierarchy (farthest-first); steady-state
    # passes are warm-started and run inside the timed loop
    _sync(dev)
    t0 = time.perf_counter()
    with _ff_timer() as ff:
        ms.graph.cluster_pass(n_fine, n_top, cluster_iters)
    _sync(dev)
    seed_ms = (time.perf_counter() - t0) * 1e3

    batches = iter([synth_facts(convs, facts, rng) for _ in range(warmup + steps)])

    def make_batch():
        conversations = next(batches)
        V = synth_vectors(ms, convs * facts, dim, dup_rate, gen)
        texts = [f["content"] for c in conversations for f in c]
        from lazzaro_amd.utils.tracing import tracer as _tr
        with _tr.stage("fact_embed", dev):
            ms._batch_embed_any(texts)  # the fact embedding runs (see module doc)
        return conversations, V

    def run_steps(k):
        if stream:
            yield from ms.consolidate_stream((make_batch() for _ in range(k)), lookahead=lookahead)
        else:
            for _ in range(k):
                conversations, V = make_batch()
                yield ms.consolidate_batch(conversations, embeddings=V)

    for _ in run_steps(warmup):
        pass
    _sync(dev)
    comm.barrier()
    prof = None
    if os.environ.get("LZK_PROF_HOST") == "1":  # host-side profile of the timed steps (stderr)
        import cProfile
        prof = cProfile.Profile()
        prof.enable()
    tprof = None
    if os.environ.get("LZK_PROF_OPS") == "1":  # aten ops per Python call site of the timed steps (stderr)
        from torch.profiler import ProfilerActivity, profile
        tprof = profile(activities=[ProfilerActivity.CPU], with_stack=True)
        tprof.__enter__()
    t0 = time.perf_counter()
    agg = {}
    for i, st in enumerate(run_steps(steps)):
        for k, v in st.items():
            agg[k] = agg.get(k, 0) + v
        if comm.rank == 0:  # progress (stderr, one short line per step)
            print(f"consolidate step {i + 1}/{steps} {time.perf_counter() - t0:.2f}s", file=sys.stderr, flush=True)
    ms.flush_persistence()  # write-behind commits of the timed steps land inside the timed region
    _sync(dev)
    if tprof is not None:
        tprof.__exit__(None, None, None)
        ka = tprof.key_averages(group_by_stack_n=3)
        rows = sorted(ka, key=lambda e: -e.count)
        print(f"# aten ops over {steps} steps: {sum(e.count for e in ka if e.key.startswith('aten::'))}",
              file=sys.stderr)
        for e in rows[:120]:
            if not e.key.startswith("aten::") and not e.key.startswith("cuda"):
                continue
            st = " <- ".join(x.split("/")[-1] for x in (e.stack or [])[:3])
            print(f"{e.count / steps:8.1f}/step  {e.self_cpu_time_total / steps / 1e3:8.2f} ms  {e.key:32s} {st}",
                  file=sys.stderr)
    if prof is not None:
        import pstats
        prof.disable()
        pstats.Stats(prof, stream=sys.stderr).sort_stats("tottime").print_stats(30)
        pstats.Stats(prof, stream=sys.stderr).sort_stats("cumulative").print_stats(40)
        # who synchronises: callers of the host-device transfers / syncing ops
        pstats.Stats(prof, stream=sys.stderr).print_callers(r"method 'cpu'|method 'item'|method 'tolist'|"
                                                            r"torch.nonzero|method 'numpy'")
    comm.barrier()
    el = time.perf_counter() - t0
    t = torch.tensor([el], dtype=torch.float64, device=dev if comm.enabled and dev.type == "cuda" else "cpu")
    comm.all_reduce(t, "max")
    el = float(t.item())
    g = ms.graph
    from lazzaro_amd.utils.tracing import tracer
    stages = None
    if tracer.enabled:  # LZK_TRACE=1: per-stage device time (hipEvents), warmup included
        import json as _json
        stages = tracer.summary()
        print(_json.dumps({"stages_ms": stages}), flush=True)
        tracer.reset()
    out = {"turns_per_s": round(convs * comm.world * steps / el, 2), "ms_per_step": round(el / steps * 1e3, 3),
           "nodes_per_rank": nodes, "convs_per_rank_step": convs, "facts_per_conv": facts,
           "prune_threshold": prune_threshold, "edges_rank0_at_start": edges_start,
           "buffer_nodes_total": nodes * comm.world, "nodes_rank0": g.num_nodes(), "edges_rank0": g.num_edges,
           "per_step_rank0": {k: round(v / steps, 1) for k, v in agg.items()},
           # per-rank scan work (facts x rows of the rank's own tenant): no
           # rank ever scans another rank's rows, so it is independent of N
           "scan_facts_x_rows_per_rank_step": int(convs * facts * g.n),
           "path": ("MemorySystem.consolidate_stream (tenant-DP; batch i+1's scan under batch i's apply)" if stream
                    else "MemorySystem.consolidate_batch (tenant-DP)"),
           "hierarchical_clustering": {"mode": "kmeans", "every_steps": cluster_every, "fine": n_fine, "top": n_top,
                                       "iters_per_pass": cluster_iters, "seed_pass_ms": round(seed_ms, 1),
                                       "farthest_first_ms": ff.get("ms")},
           "stages_ms": stages,
           "persistence": "incremental columnar commit per step (db on local disk)" + (
               ", write-behind (persist_async: commits on a writer thread, flushed inside the timed region)"
               if persist_async else "")}
    ms.close()
    return out


def run_sharded(comm, dev, nodes_per_rank: int, convs: int, facts: int, steps: int, warmup: int, encoder=None,
                dim: int = 768, dup_rate: float = 0.1, seed: int = 7, cluster_every: int = 5, n_fine: int = 4096,
                n_top: int = 64, cluster_iters: int = 2, init_edges: int = None, db_dir: str = None,
                clustered: bool = False, topics_per_rank: int = 32, cadence: str = "conversation",
                stream: bool = False, prune_threshold: float = 0.5):
    """BASELINE config 4 as ONE tenant: a ``nodes_per_rank * world``-node
    buffer row-sharded over the ranks (``ShardedMemorySystem``); every step
    each rank brings ``convs`` conversations, the whole batch is consolidated
    over the whole buffer (facts all-gathered, each rank scans them against
    its rows, top-3 lists merged, global eviction, distributed CC, distributed
    k-means hierarchy), each rank commits its rows. Per-rank scan work is
    (world * convs * facts) x nodes_per_rank: the buffer is split N ways,
    every fact is compared with every memory (the reference's semantics).

    ``clustered``: each rank's rows are ``topics_per_rank`` tight topics of
    its own (cos ~0.97 to the topic centre) and new nodes are placed on their
    cluster's home rank (``placement="cluster"``); the exact cone pruning
    then lets a rank skip the facts no cluster it holds can reach, and the
    reported ``scan_facts_x_rows_per_rank_step`` is the measured count
    (``ShardedMemorySystem.last_scan_work``, max over ranks).

    ``cadence``: "conversation" (default, the reference's per-conversation
    eviction / run_consolidation, planned once per batch) or "batch".
    ``stream``: ``ShardedMemorySystem.consolidate_stream`` instead of
    per-batch calls -- off by default: on the clustered buffer a batch's
    victims sit in the next batch's candidate lists, whose facts are then
    re-scanned (profiles/r5/sharded_stream/). ``prune_threshold`` 0: the
    persistent graph (the seeded 2 x rows edges per rank are never pruned;
    run_consolidation's digest takes the incremental form,
    ShardedMemorySystem._dcc_begin)."""
    from lazzaro_amd.core.providers import HashEmbedder, LocalLLM
    from lazzaro_amd.parallel.sharded_memory import ShardedMemorySystem

    world = comm.world
    db_dir = db_dir or tempfile.mkdtemp(prefix=f"lzshc{comm.rank}_")
    init_edges = 2 * nodes_per_rank if init_edges is None else init_edges
    sm = ShardedMemorySystem(comm, "buffer", max_buffer_size=nodes_per_rank * world, llm_provider=LocalLLM(),
                             embedding_provider=encoder or HashEmbedder(dim=dim), db_dir=db_dir, device=dev,
                             hierarchy_params={"fine": n_fine, "top": n_top, "every": cluster_every * convs * world,
                                               "iters": cluster_iters},
                             placement="cluster" if clustered else "origin", prune_threshold=prune_threshold)
    g = sm.g
    g._set_dim(dim)
    g.reserve(int(nodes_per_rank * 1.05) + 65536)
    codes = torch.tensor(sm.register_shards(SHARDS), dtype=torch.int32, device=dev)
    gen = torch.Generator(device=dev).manual_seed(seed + 31 * comm.rank)
    now = time.time()
    chunk = 1 << 20
    t0 = time.perf_counter()
    if clustered:  # every rank draws the same centres; rank r's rows come from topics r*T .. r*T+T-1
        cg = torch.Generator().manual_seed(seed)
        centres = _unit(torch.randn((world * topics_per_rank, dim), generator=cg)).to(dev)
        sigma = math.tan(math.radians(14.0)) / math.sqrt(dim)  # rows at cos ~0.97 to their topic centre
    for r0 in range(0, nodes_per_rank, chunk):  # collective per chunk: global node numbers, rank-major
        r1 = min(nodes_per_rank, r0 + chunk)
        v = torch.randn((r1 - r0, dim), device=dev, generator=gen)
        if clustered:
            t = comm.rank * topics_per_rank + torch.randint(0, topics_per_rank, (r1 - r0,), device=dev, generator=gen)
            v = centres[t] + sigma * v
        v /= v.norm(dim=1, keepdim=True)
        sm.add_memories([f"memory {comm.rank}.{i}" for i in range(r0, r1)], v, salience=0.5, now=now,
                        shard_codes=codes[torch.arange(r0, r1, device=dev) % len(SHARDS)])
    if init_edges:
        src = torch.randint(0, nodes_per_rank, (init_edges,), device=dev, generator=gen)
        dst = torch.randint(0, nodes_per_rank, (init_edges,), device=dev, generator=gen)
        w = torch.rand(init_edges, device=dev, generator=gen) * 0.5 + 0.5
        g.append_edges(src.int(), dst.int(), w, g.shard[src], g.etype("relates_to"))
    g.clear_tracking(stored=False)
    _sync(dev)
    load_s = time.perf_counter() - t0
    edges0 = sm.get_stats()["total_edges"]
    t0 = time.perf_counter()
    with _ff_timer() as ff:
        sm.cluster_pass()
    _sync(dev)
    seed_ms = (time.perf_counter() - t0) * 1e3
    rng = random.Random(seed + comm.rank)
    batches = iter([synth_facts(convs, facts, rng) for _ in range(warmup + steps)])

    def make_batch():
        conversations = next(batches)
        V = synth_vectors(sm.local, convs * facts, dim, dup_rate, gen)
        if encoder is not None:
            from lazzaro_amd.utils.tracing import tracer as _tr
            with _tr.stage("fact_embed", dev):
                sm.local._batch_embed_any([f["content"] for c in conversations for f in c])
        return conversations, V

    def run_steps(k):
        if stream:
            yield from sm.consolidate_stream((make_batch() for _ in range(k)), cadence=cadence)
        else:
            for _ in range(k):
                conversations, V = make_batch()
                yield sm.consolidate_batch(conversations, embeddings=V, cadence=cadence)

    for _ in run_steps(warmup):
        pass
    _sync(dev)
    comm.barrier()
    prof = None
    if os.environ.get("LZK_PROF_HOST") == "1":  # host-side profile of the timed steps (stderr)
        import cProfile
        prof = cProfile.Profile()
        prof.enable()
    import gc
    gcl = [0, 0.0, 0.0]  # passes, seconds, start

    def _gc_cb(phase, info):
        if phase == "start":
            gcl[2] = time.perf_counter()
        else:
            gcl[0] += 1
            gcl[1] += time.perf_counter() - gcl[2]
    gc.callbacks.append(_gc_cb)
    t0 = time.perf_counter()
    agg = {}
    work0 = sm.scan_work
    for i, st in enumerate(run_steps(steps)):
        if comm.rank == 0:  # progress (stderr)
            print(f"sharded consolidate step {i + 1}/{steps}", file=sys.stderr, flush=True)
        for k, v in st.items():
            agg[k] = agg.get(k, 0) + v
    _sync(dev)
    comm.barrier()
    el = time.perf_counter() - t0
    gc.callbacks.remove(_gc_cb)
    if prof is not None:
        import pstats
        prof.disable()
        pstats.Stats(prof, stream=sys.stderr).sort_stats("tottime").print_stats(40)
        pstats.Stats(prof, stream=sys.stderr).sort_stats("cumulative").print_stats(60)
        pstats.Stats(prof, stream=sys.stderr).print_callers(r"method 'cpu'|method 'item'|method 'tolist'|"
                                                            r"torch.nonzero|method 'numpy'")
    t = torch.tensor([el], dtype=torch.float64, device=dev if comm.enabled and dev.type == "cuda" else "cpu")
    comm.all_reduce(t, "max")
    el = float(t.item())
    wk = torch.tensor([(sm.scan_work - work0) / max(steps, 1)], dtype=torch.float64,
                      device=dev if comm.enabled and dev.type == "cuda" else "cpu")
    comm.all_reduce(wk, "max")
    from lazzaro_amd.utils.tracing import tracer
    stages = {k: v["p50_ms"] for k, v in tracer.summary().items()} if tracer.enabled else None
    st = sm.get_stats()
    out = {"turns_per_s": round(convs * world * steps / el, 2), "ms_per_step": round(el / steps * 1e3, 3),
           "prune_threshold": prune_threshold, "edges_total_at_start": edges0,
           "incremental_digest_points": sm.dcc_points, "incremental_digest_base_edges_max": sm.dcc_base_max,
           "buffer_nodes_total": st["total_nodes"], "nodes_per_rank": nodes_per_rank, "edges_total": st["total_edges"],
           "convs_per_rank_step": convs, "facts_per_conv": facts,
           "per_step": {k: round(v / steps, 1) for k, v in agg.items()},
           # measured: facts x live rows this rank's scans compared (max over ranks)
           "scan_facts_x_rows_per_rank_step": int(wk.item()),
           "scan_facts_x_rows_unpruned_per_rank_step": int(world * convs * facts * nodes_per_rank),
           "data": "clustered topics, cluster placement" if clustered else "uniform random rows",
           "path": ("ShardedMemorySystem.%s (one tenant row-sharded over the ranks), cadence=%s"
                    % ("consolidate_stream" if stream else "consolidate_batch", cadence)),
           "hierarchical_clustering": {"mode": "distributed kmeans", "every_steps": cluster_every, "fine": n_fine,
                                       "top": n_top, "iters_per_pass": cluster_iters,
                                       "seed_pass_ms": round(seed_ms, 1), "farthest_first_ms": ff.get("ms")},
           "load_s": round(load_s, 1), "stages_p50_ms": stages,
           "gc_in_timed_loop": {"passes": gcl[0], "ms": round(gcl[1] * 1e3, 2)},
           "persistence": "incremental columnar commit of each rank's rows per step"}
    sm.close()
    return out


if __name__ == "__main__":
    import argparse
    import json

    from lazzaro_amd.parallel import Communicator

    ap = argparse.ArgumentParser()
    ap.add_argument("--nodes", type=int, default=10_000_000)
    ap.add_argument("--convs", type=int, default=128)
    ap.add_argument("--facts", type=int, default=8)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--no-embed", action="store_true")
    ap.add_argument("--cluster-every", type=int, default=5, help="steps between hierarchical clustering passes")
    ap.add_argument("--fine", type=int, default=4096)
    ap.add_argument("--top", type=int, default=64)
    ap.add_argument("--cluster-iters", type=int, default=2)
    ap.add_argument("--dim", type=int, default=768)
    ap.add_argument("--prune-threshold", type=float, default=0.5,
                    help="MemorySystem(prune_threshold=): 0.5 is the reference default; 0 keeps every edge "
                         "(decay still runs on all of them) -- the large-graph variant")
    ap.add_argument("--persist-async", action="store_true", help="MemorySystem(persist_async=True)")
    ap.add_argument("--no-stream", dest="stream", action="store_false",
                    help="one consolidate_batch call per step instead of consolidate_stream")
    ap.add_argument("--init-edges", type=int, default=None, help="seeded edges (default 2 x nodes)")
    ap.add_argument("--sharded", action="store_true",
                    help="config 4 as one tenant row-sharded over the ranks (--nodes per rank)")
    ap.add_argument("--clustered", action="store_true",
                    help="--sharded: per-rank topic clusters + cluster placement (exact scan pruning applies)")
    ap.add_argument("--cadence", default="conversation", choices=["conversation", "batch"],
                    help="--sharded: reference per-conversation cadence or once-per-batch")
    ap.add_argument("--no-incremental-digest", action="store_true",
                    help="--sharded: the full digest at every run_consolidation point (A/B)")
    ap.add_argument("--no-prefetch-under-cluster", action="store_true",
                    help="no batch i+1 scan prefetch past a batch that runs a k-means pass (A/B)")
    ap.add_argument("--eager-node-decay", action="store_true",
                    help="native applier: a node-salience pass per segment instead of the lazy stamps (A/B)")
    ap.add_argument("--lookahead", type=int, default=2,
                    help="consolidate_stream: batches drawn ahead (1 = the next one only; A/B)")
    ap.add_argument("--cluster-inline", action="store_true",
                    help="k-means passes in line instead of in the background (A/B)")
    a = ap.parse_args()
    if a.eager_node_decay:
        from lazzaro_amd.engine import native_apply
        native_apply.LAZY_NODE_DECAY = False
    if a.cluster_inline:
        from lazzaro_amd.core.memory_system import MemorySystem
        MemorySystem.CLUSTER_BACKGROUND = False
    if a.no_prefetch_under_cluster:
        from lazzaro_amd.core.memory_system import MemorySystem
        MemorySystem.PREFETCH_UNDER_CLUSTER = False
    if a.no_incremental_digest:
        from lazzaro_amd.parallel.sharded_memory import ShardedMemorySystem
        ShardedMemorySystem.DIGEST_INCREMENTAL = False
    comm = Communicator.init()
    local = int(os.environ.get("LOCAL_RANK", "0"))
    dev = torch.device("cuda", local) if torch.cuda.is_available() else torch.device("cpu")
    enc = None
    if not a.no_embed and dev.type == "cuda":
        from lazzaro_amd.core.embedders import OnDeviceEmbedder
        enc = OnDeviceEmbedder("bge-base", device=dev, max_len=64)
    fn = run_sharded if a.sharded else run
    res = fn(comm, dev, a.nodes, a.convs, a.facts, a.steps, a.warmup, enc, dim=a.dim, cluster_every=a.cluster_every,
             n_fine=a.fine, n_top=a.top, cluster_iters=a.cluster_iters, init_edges=a.init_edges,
             **({"clustered": a.clustered, "cadence": a.cadence, "stream": a.stream,
                 "prune_threshold": a.prune_threshold} if a.sharded else
                {"prune_threshold": a.prune_threshold, "persist_async": a.persist_async, "stream": a.stream,
                 "lookahead": a.lookahead}))
    if comm.rank == 0:
        print(json.dumps({"metric": "consolidate turns/sec", "n_gpus": comm.world, **res}), flush=True)
    if comm.enabled:
        import torch.distributed as dist
        dist.barrier()
        dist.destroy_process_group()
