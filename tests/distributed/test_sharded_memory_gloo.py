"""Row-sharded tenant (lazzaro_amd/parallel/sharded_memory.py) on CPU with
gloo: ONE tenant's buffer split over 1, 2 and 3 ranks, consolidated batch by
batch, ends in exactly the state a single-process ``MemorySystem`` reaches on
the union of the rows and all ranks' conversations -- the same node ids,
saliences and access counts, the same edges and weights, the same eviction
victims and per-batch counts, the same component digest and profile.

Data: clustered unit vectors (so links clear the 0.5 threshold), facts that
are near-duplicates of stored memories, related memories or new, a buffer
limit that forces eviction every batch, distinct saliences (no importance
ties), and a shard first seen mid-run."""
import functools
import math
import random

import pytest
import torch

from tests.distributed.test_dist_gloo import spawn

DIM = 32
ROWS = 180
LIMIT = 200
STEPS = 4
CONVS = 12
TOPICS = ["work", "personal", "learning"]
QUERIES = ["fact about work", "memory 12", "learning something new", "health and sleep", "personal", "memory 7 x"]


def _unit(x):
    return x / x.norm(dim=-1, keepdim=True)


CPU = {"rows": ROWS, "dim": DIM, "limit": LIMIT, "steps": STEPS, "convs": CONVS, "device": "cpu"}


def _data(cfg=CPU):
    """Union rows + per-step global conversation lists (deterministic)."""
    ROWS, DIM, STEPS, CONVS = cfg["rows"], cfg["dim"], cfg["steps"], cfg["convs"]
    noise = 0.18 * (32 / DIM) ** 0.5 * 1.0
    g = torch.Generator().manual_seed(5)
    centers = _unit(torch.randn(8, DIM, generator=g))
    lab = torch.randint(0, 8, (ROWS,), generator=g)
    X = _unit(centers[lab] + noise * torch.randn(ROWS, DIM, generator=g))
    rng = random.Random(11)
    sal0 = [round(rng.uniform(0.3, 0.95), 6) for _ in range(ROWS)]
    keys0 = [TOPICS[i % 3] for i in range(ROWS)]
    tight = cfg.get("tight", False)
    if tight:  # one tight topic: its super-node's mean is close enough to dedupe facts onto it
        for i in range(2, ROWS, 3):
            X[i] = _unit(centers[0] + noise / 3 * torch.randn(DIM, generator=g))
    steps = []
    for s in range(STEPS):
        convs, vecs = [], []
        for c in range(CONVS):
            facts = []
            for f in range(rng.randint(1, 4)):
                kind = rng.random()
                if tight and 0.8 <= kind < 0.88:
                    v = _unit(centers[0] + noise / 4 * torch.randn(DIM, generator=g))  # onto the tight topic
                    facts.append({"content": f"fact {s}.{c}.{f} about learning", "type": "semantic",
                                  "salience": round(rng.uniform(0.3, 0.95), 6), "topic": "learning"})
                    vecs.append(v)
                    continue
                if kind < 0.2:
                    v = _unit(X[rng.randrange(ROWS)] + noise / 9 * torch.randn(DIM, generator=g))  # duplicate
                elif kind < 0.3 and vecs:
                    v = _unit(vecs[rng.randrange(len(vecs))] + noise / 9 * torch.randn(DIM, generator=g))  # in-batch
                elif kind < 0.8:
                    v = _unit(centers[rng.randrange(8)] + noise * torch.randn(DIM, generator=g))  # related
                else:
                    v = _unit(torch.randn(DIM, generator=g))  # new
                topic = "health" if (s >= 2 and kind > 0.9) else TOPICS[rng.randrange(3)]
                facts.append({"content": f"fact {s}.{c}.{f} about {topic}", "type": "semantic",
                              "salience": round(rng.uniform(0.3, 0.95), 6), "topic": topic})
                vecs.append(v)
            convs.append(facts)
        steps.append((convs, torch.stack(vecs)))
    return X, sal0, keys0, steps


def _seed_edges(cfg):
    """``seed_edges`` random links among the initial rows (weights in [0.55, 1))."""
    g = torch.Generator().manual_seed(17)
    m, R = int(cfg["seed_edges"]), cfg["rows"]
    src = torch.randint(0, R, (m,), generator=g)
    dst = (src + 1 + torch.randint(0, R - 1, (m,), generator=g)) % R
    return src, dst, torch.rand(m, generator=g) * 0.45 + 0.55


def _split(n, world, r, weights=None):
    if weights:
        w = weights[:world]
        per = [n * x // sum(w) for x in w]
        per[0] += n - sum(per)
    else:
        per = [n // world + (1 if i < n % world else 0) for i in range(world)]
    lo = sum(per[:r])
    return lo, lo + per[r]


def _sid(i):
    """Super-node ids without their creation second (the single process's
    batch cadence stamps them with the wall clock)."""
    return i.rsplit("_", 1)[0] if i.startswith("super_") else i


def _graph_state(g):
    from lazzaro_amd.engine.tenant_graph import NODE
    n = g.n
    kind, sal, acc, sh = (g.kind[:n].tolist(), g.sal[:n].tolist(), g.acc[:n].tolist(), g.shard[:n].tolist())
    par, sup = g.parent[:n].tolist(), g.sup[:n].tolist()
    nodes = {_sid(g.ids[r]): (round(sal[r], 5), acc[r], g.shard_names[sh[r]],
                              _sid(g.ids[par[r]]) if par[r] >= 0 else None,
                              (g.content[r], list(g.children.get(r, []))) if sup[r] else None)
             for r in range(n) if kind[r] == NODE}
    e = g.e
    edges = {}
    for s, d, w, m in zip(e["src"].tolist(), e["dst"].tolist(), e["w"].tolist(), e["meta"].tolist()):
        edges[(g.ids[s], g.ids[d])] = (round(w, 5), g.shard_names[m & 0xFFFFFF])
    return nodes, edges


def _now(s):
    return 1.7e9 + 3600.0 * s


def _single(tmp, cfg=CPU):
    """The single-process engine on the union."""
    from lazzaro_amd.core.memory_system import MemorySystem
    from lazzaro_amd.core.providers import HashEmbedder, LocalLLM
    X, sal0, keys0, steps = _data(cfg)
    dev = cfg["device"]
    ms = MemorySystem(llm_provider=LocalLLM(), embedding_provider=HashEmbedder(dim=cfg["dim"]), enable_async=False,
                      db_dir=tmp, user_id="solo", device=dev, max_buffer_size=cfg["limit"],
                      enable_hierarchy=cfg.get("hier", False), super_node_threshold=cfg.get("sthr", 20),
                      load_from_disk=False, enable_caching=False, prune_threshold=cfg.get("prune_thr", 0.5))
    g = ms.graph
    codes = [g.shard_id(k) for k in keys0]
    R = cfg["rows"]
    g.add_nodes([f"node_{i + 1}" for i in range(R)], [f"memory {i + 1}" for i in range(R)], X.to(dev),
                shard=codes, sal=torch.tensor(sal0), now=_now(-1), stored=True)
    ms.node_counter = R
    if cfg.get("seed_edges"):  # a graph that starts with edges (world-1 comparisons only)
        src, dst, w = _seed_edges(cfg)
        g.append_edges(src.to(dev), dst.to(dev), w.to(dev), g.shard[src.to(dev)], g.etype("relates_to"), now=_now(-1))
    stats = []
    for s, (convs, V) in enumerate(steps):
        import lazzaro_amd.engine.tenant_graph as tgm
        real = tgm.time.time
        tgm.time.time = lambda s=s: _now(s)  # the single-process eviction reads the wall clock
        try:
            stats.append(ms.consolidate_batch(convs, embeddings=V.to(dev), now=_now(s),
                                              cadence=cfg.get("cadence", "batch")))
        finally:
            tgm.time.time = real
    nodes, edges = _graph_state(g)
    digest = g.component_digest(3, 0.3, 10)
    contents = [[g.content[r] for r in rows.tolist()] for rows in digest]
    prof = dict(ms.profile.data)
    found = [[n.id for n in res] for res in ms.search_memories_batch(QUERIES, 5)]
    ms.close()
    return stats, nodes, edges, contents, prof, found


def _sharded(comm, cfg=CPU):
    import tempfile

    from lazzaro_amd.core.providers import HashEmbedder, LocalLLM
    from lazzaro_amd.parallel.sharded_memory import ShardedMemorySystem
    X, sal0, keys0, steps = _data(cfg)
    dev = cfg["device"]
    tmp = tempfile.mkdtemp(prefix=f"lzsh{comm.rank}_")
    pruned = cfg.get("pruned", False)
    extra = dict(hierarchy_params={"fine": 12, "top": 4, "every": 10 ** 6, "iters": 3}, placement="cluster",
                 prune=True) if pruned else {}
    if not pruned:
        extra.update(enable_hierarchy=cfg.get("hier", False), super_node_threshold=cfg.get("sthr", 20))
    sm = ShardedMemorySystem(comm, "big", max_buffer_size=cfg["limit"], llm_provider=LocalLLM(),
                             embedding_provider=HashEmbedder(dim=cfg["dim"]), db_dir=tmp, device=dev,
                             force_collectives=cfg.get("force", False), prune_threshold=cfg.get("prune_thr", 0.5),
                             **extra)
    if "dcc_min" in cfg:  # the incremental digest from this many edges (0: every batch with a point)
        sm.DIGEST_INCREMENTAL_MIN = cfg["dcc_min"]
    if cfg.get("dcc_check"):  # every incremental point equals the full replicated digest
        real_inc = sm._digest_incremental
        checked_pts = []

        def inc_checked(min_size, min_avg_w, take):
            a = real_inc(min_size, min_avg_w, take)
            b = sm._digest_replicated(sm._host_ints(sm.g.num_edges)[:, 0].tolist(), min_size, min_avg_w, take)
            assert a == b, (a, b)
            checked_pts.append(len(b))
            return a
        sm._digest_incremental = inc_checked
    if "native_w1" in cfg:  # one rank: the native segment applier on / off
        sm.NATIVE_W1 = bool(cfg["native_w1"])
    if "digest_max" in cfg:  # -1: the boundary-label digest instead of the replicated one
        sm.DIGEST_REPLICATE_MAX = cfg["digest_max"]
    if cfg.get("digest_check"):  # one GPU rank: the row digest equals the replicated one at every point
        real = sm.component_digest
        seen = []

        def checked(min_size=3, min_avg_w=0.3, take=10):
            a = real(min_size, min_avg_w, take)
            b = sm._digest_replicated([sm.g.num_edges], min_size, min_avg_w, take) if sm.g.num_edges else []
            assert a == b, (a, b)
            seen.append(len(a))
            return a
        sm.component_digest = checked
    rebal = cfg.get("rebalance", False)
    lo, hi = _split(cfg["rows"], comm.world, comm.rank, [5, 1, 2] if rebal else None)
    sm.add_memories([f"memory {i + 1}" for i in range(lo, hi)], X[lo:hi].to(dev), keys0[lo:hi],
                    salience=torch.tensor(sal0[lo:hi]), now=_now(-1))
    if cfg.get("seed_edges"):
        assert comm.world == 1, "seeded edges: one rank (every row local)"
        src, dst, w = _seed_edges(cfg)
        g = sm.g
        g.append_edges(src.to(dev), dst.to(dev), w.to(dev), g.shard[src.to(dev)], g.etype("relates_to"), now=_now(-1))
    if pruned:  # pruned scan + cluster placement: the same decisions as the single process
        sm.cluster_pass()
    spread = []
    stats = []

    def part(s, convs, V):
        c0, c1 = _split(len(convs), comm.world, comm.rank)
        f0 = sum(len(c) for c in convs[:c0])
        f1 = f0 + sum(len(c) for c in convs[c0:c1])
        return convs[c0:c1], V[f0:f1].to(dev), _now(s)

    if cfg.get("stream"):  # consolidate_stream: batch i+1 gathered and scanned under batch i's apply
        stats = list(sm.consolidate_stream((part(s, c, V) for s, (c, V) in enumerate(steps)),
                                           cadence=cfg.get("cadence", "batch")))
        steps = []
    for s, (convs, V) in enumerate(steps):
        cv, Vp, t = part(s, convs, V)
        stats.append(sm.consolidate_batch(cv, embeddings=Vp, now=t, cadence=cfg.get("cadence", "batch")))
        if rebal:  # all-to-all re-shard to even shares between batches; decisions must not change
            sm.rebalance()
            cnt = comm.all_gather_object(sm.g.num_nodes())
            spread.append(max(cnt) - min(cnt))
    pf_used = sm.prefetched_batches
    nodes, edges = _graph_state(sm.g)
    parts = comm.all_gather_object((nodes, edges))
    contents = sm.component_digest(3, 0.3, 10)
    prof = dict(sm.profile.data)
    total = sm.num_nodes()
    q0, q1 = _split(len(QUERIES), comm.world, comm.rank)
    found = [[d["id"] for d in res] for res in sm.search_memories_batch(QUERIES[q0:q1], 5)]
    found = [f for part in comm.all_gather_object(found) for f in part]
    sm.close()
    native = sm.native_w1_runs
    dcc = (sm.dcc_points, sm.dcc_base_max, sum(checked_pts) if cfg.get("dcc_check") else 0)
    if comm.rank != 0:
        return {"stats": stats, "prof": prof, "pf_used": pf_used, "native": native, "dcc": dcc}
    nodes_all, edges_all = {}, {}
    for n_, e_ in parts:
        assert not (set(n_) & set(nodes_all)), "a node is live on two ranks"
        nodes_all.update(n_)
        edges_all.update(e_)
    single = _single(tempfile.mkdtemp(prefix="lzsolo_"), cfg)
    return {"stats": stats, "nodes": nodes_all, "edges": edges_all, "contents": contents, "prof": prof,
            "total": total, "found": found, "single": single, "spread": spread, "pf_used": pf_used, "native": native,
            "dcc": dcc}


def check_equivalent(out, world, limit):
    r0 = out[0]
    s_stats, s_nodes, s_edges, s_contents, s_prof, s_found = r0["single"]
    assert r0["stats"] == s_stats, (r0["stats"], s_stats)
    for r in range(world):  # every rank reports the same whole-batch counts and profile
        assert out[r]["stats"] == s_stats
        assert out[r]["prof"] == s_prof
    assert sum(st["evicted"] for st in s_stats) > 0 and sum(st["dup"] for st in s_stats) > 0
    assert sum(st["linked"] for st in s_stats) > 0 and s_edges
    assert r0["nodes"] == s_nodes
    assert r0["total"] == len(s_nodes) == limit
    assert set(r0["edges"]) == set(s_edges)
    for k, (w, sh) in s_edges.items():
        w2, sh2 = r0["edges"][k]
        assert sh2 == sh and math.isclose(w, w2, abs_tol=1e-4)
    assert r0["contents"] == s_contents
    assert r0["found"] == s_found and all(len(f) == 5 for f in s_found)


@pytest.mark.parametrize("world", [1, 2, 3])
def test_sharded_tenant_matches_single_process(world):
    check_equivalent(spawn(world, _sharded), world, LIMIT)


@pytest.mark.parametrize("pruned", [False, True])
def test_sharded_tenant_forced_collectives_world1(pruned):
    """One rank with every exchange forced through the communicator (the
    path bench.py times under a 1-rank torch.distributed.run): the
    single-process state."""
    cfg = dict(CPU, force=True, pruned=pruned)
    check_equivalent(spawn(1, functools.partial(_sharded, cfg=cfg)), 1, LIMIT)


@pytest.mark.parametrize("world", [2, 3])
def test_sharded_tenant_pruned_cluster_placement_matches_single_process(world):
    check_equivalent(spawn(world, functools.partial(_sharded, cfg=dict(CPU, pruned=True))), world, LIMIT)


@pytest.mark.parametrize("world", [2, 3])
def test_sharded_tenant_rebalance_keeps_semantics(world):
    """Uneven initial split (5:1:2) re-sharded to even shares after every
    batch by all-to-all (C3): still the single-process state, shares within 1."""
    out = spawn(world, functools.partial(_sharded, cfg=dict(CPU, rebalance=True)))
    check_equivalent(out, world, LIMIT)
    assert all(s <= 1 for s in out[0]["spread"])


EXACT = dict(CPU, cadence="conversation")


@pytest.mark.parametrize("world", [1, 2, 3, 8])
def test_sharded_tenant_reference_cadence_matches_single_process(world):
    """cadence="conversation" (the default): the reference's per-conversation
    cadence over the row-sharded buffer equals a single process's
    ``consolidate_batch(cadence="conversation")`` on the union -- eviction
    per conversation, run_consolidation at every multiple of 3."""
    out = spawn(world, functools.partial(_sharded, cfg=EXACT))
    check_equivalent(out, world, LIMIT)
    assert sum(st["consolidations"] for st in out[0]["stats"]) == STEPS * CONVS // 3


def test_sharded_tenant_consolidate_stream_cpu():
    """consolidate_stream at 2 gloo ranks: the per-batch calls' state (on the
    CPU nothing is prefetched: the stream plumbing; the prefetched GPU path
    is tests/kernels/test_sharded_memory_gpu.py)."""
    out = spawn(2, functools.partial(_sharded, cfg=dict(EXACT, stream=True)))
    check_equivalent(out, 2, LIMIT)


@pytest.mark.parametrize("world", [2, 3])
def test_sharded_tenant_distributed_digest_matches_single_process(world):
    """The boundary-label component digest (taken above
    DIGEST_REPLICATE_MAX edges) gives the same runs as the replicated one."""
    out = spawn(world, functools.partial(_sharded, cfg=dict(EXACT, digest_max=-1)))
    check_equivalent(out, world, LIMIT)
    assert out[0]["contents"]


@pytest.mark.parametrize("world,prune_thr", [(2, 0.5), (3, 0.5), (2, 0.0), (3, 0.0)])
def test_sharded_tenant_incremental_digest(world, prune_thr):
    """The incremental digest (a batch's stable base all-gathered and
    labelled once, only the volatile edges per point): at every
    run_consolidation point the full replicated digest's lists, and the
    single process's state -- with the default decay-prune and on a
    persistent graph (prune_threshold 0: no edge is ever pruned)."""
    cfg = dict(EXACT, dcc_min=0, dcc_check=True, prune_thr=prune_thr)
    out = spawn(world, functools.partial(_sharded, cfg=cfg))
    check_equivalent(out, world, LIMIT)
    d = [out[r]["dcc"] for r in range(world)]
    assert all(x[0] > 0 for x in d), d  # points served incrementally
    assert max(x[1] for x in d) > 0, d  # with a non-empty stable base
    assert d[0][2] > 0, d  # and qualifying components


def test_sharded_tenant_reference_cadence_forced_world1():
    check_equivalent(spawn(1, functools.partial(_sharded, cfg=dict(EXACT, force=True))), 1, LIMIT)


@pytest.mark.parametrize("world", [2, 3])
def test_sharded_tenant_reference_cadence_pruned_cluster(world):
    check_equivalent(spawn(world, functools.partial(_sharded, cfg=dict(EXACT, pruned=True))), world, LIMIT)


def test_sharded_tenant_reference_cadence_rebalance():
    out = spawn(3, functools.partial(_sharded, cfg=dict(EXACT, rebalance=True)))
    check_equivalent(out, 3, LIMIT)


def _sharded_hierarchy(comm):
    import tempfile

    from lazzaro_amd.core.providers import HashEmbedder, LocalLLM
    from lazzaro_amd.parallel.sharded_memory import ShardedMemorySystem
    X, sal0, keys0, steps = _data()
    sm = ShardedMemorySystem(comm, "big", max_buffer_size=LIMIT, llm_provider=LocalLLM(),
                             embedding_provider=HashEmbedder(dim=DIM), db_dir=tempfile.mkdtemp(), device="cpu",
                             hierarchy_params={"fine": 16, "top": 4, "every": 12, "iters": 3})
    lo, hi = _split(ROWS, comm.world, comm.rank)
    sm.add_memories([f"memory {i + 1}" for i in range(lo, hi)], X[lo:hi], keys0[lo:hi], now=_now(-1))
    convs, V = steps[0]
    c0, c1 = _split(len(convs), comm.world, comm.rank)
    f0 = sum(len(c) for c in convs[:c0])
    f1 = f0 + sum(len(c) for c in convs[c0:c1])
    sm.consolidate_batch(convs[c0:c1], embeddings=V[f0:f1], now=_now(0))
    h = sm.g.hier
    fine = h["fine"][: sm.g.n]
    n_lab = int((fine >= 0).sum())
    tot = torch.tensor([n_lab])
    comm.all_reduce(tot)
    cents = comm.all_gather_object(h["top_c"].tolist())
    out = {"labelled": int(tot), "nodes": sm.num_nodes(), "same_centroids": all(c == cents[0] for c in cents),
           "shape": list(h["fine_c"].shape)}
    sm.close()
    return out


def test_sharded_hierarchy_distributed_kmeans():
    out = spawn(2, _sharded_hierarchy)
    for r in range(2):
        assert out[r]["same_centroids"]  # the topic level is identical on every rank
        assert out[r]["labelled"] == out[r]["nodes"]  # every live node of the tenant has a fine cluster
        assert out[r]["shape"][0] == 16


HIER = dict(EXACT, hier=True, tight=True)


def _check_supers(out):
    nodes = out[0]["nodes"]
    sups = [k for k, v in nodes.items() if v[4] is not None]
    assert sups, "no super-node was created"
    assert sum(1 for v in nodes.values() if v[3] is not None) > 0  # children point at their super-node
    return nodes, sups


@pytest.mark.parametrize("world,sthr", [(1, 20), (2, 20), (3, 62), (8, 62)])
def test_sharded_tenant_reference_hierarchy_matches_single_process(world, sthr):
    """The reference's per-shard mean super-nodes over the row-sharded buffer
    (collective member lists and means): the same super-nodes -- id, summary,
    children, salience, access count -- the same parents, dedupes onto a
    super-node and every other decision as the single process with
    enable_hierarchy=True. sthr=62: shards cross the threshold mid-batch (the
    children are pre-batch rows AND facts of the batch)."""
    out = spawn(world, functools.partial(_sharded, cfg=dict(HIER, sthr=sthr)))
    check_equivalent(out, world, LIMIT)
    nodes, sups = _check_supers(out)
    assert any(nodes[s][1] > 0 for s in sups)  # facts were merged onto a super-node


@pytest.mark.parametrize("world", [2, 3])
def test_sharded_tenant_reference_hierarchy_batch_cadence(world):
    out = spawn(world, functools.partial(_sharded, cfg=dict(CPU, hier=True, tight=True)))
    check_equivalent(out, world, LIMIT)
    _check_supers(out)


def _commit_snaps(comm, cfg):
    """Per-commit graph states of the row-sharded tenant (every rank's part)
    and, on rank 0, of the single process, both with commit="conversation"."""
    import tempfile

    from lazzaro_amd.core.memory_system import MemorySystem
    from lazzaro_amd.core.providers import HashEmbedder, LocalLLM
    from lazzaro_amd.parallel.sharded_memory import ShardedMemorySystem
    snaps = []
    orig = MemorySystem._save_to_persistence

    def rec(self):
        out = orig(self)
        snaps.append(_graph_state(self.graph))
        return out
    MemorySystem._save_to_persistence = rec
    X, sal0, keys0, steps = _data(cfg)
    sm = ShardedMemorySystem(comm, "big", max_buffer_size=cfg["limit"], llm_provider=LocalLLM(),
                             embedding_provider=HashEmbedder(dim=cfg["dim"]), db_dir=tempfile.mkdtemp(), device="cpu",
                             enable_hierarchy=True, super_node_threshold=cfg["sthr"])
    lo, hi = _split(cfg["rows"], comm.world, comm.rank)
    sm.add_memories([f"memory {i + 1}" for i in range(lo, hi)], X[lo:hi], keys0[lo:hi],
                    salience=torch.tensor(sal0[lo:hi]), now=_now(-1))
    for s, (convs, V) in enumerate(steps):
        c0, c1 = _split(len(convs), comm.world, comm.rank)
        f0 = sum(len(c) for c in convs[:c0])
        f1 = f0 + sum(len(c) for c in convs[c0:c1])
        snaps.append("batch")
        sm.consolidate_batch(convs[c0:c1], embeddings=V[f0:f1], now=_now(s), commit="conversation")
    sm.close()
    parts = comm.all_gather_object(snaps)
    if comm.rank != 0:
        return None
    single = []
    ms = MemorySystem(llm_provider=LocalLLM(), embedding_provider=HashEmbedder(dim=cfg["dim"]), enable_async=False,
                      db_dir=tempfile.mkdtemp(), user_id="solo", device="cpu", max_buffer_size=cfg["limit"],
                      enable_hierarchy=True, super_node_threshold=cfg["sthr"], load_from_disk=False,
                      enable_caching=False)
    g = ms.graph
    g.add_nodes([f"node_{i + 1}" for i in range(cfg["rows"])], [f"memory {i + 1}" for i in range(cfg["rows"])], X,
                shard=[g.shard_id(k) for k in keys0], sal=torch.tensor(sal0), now=_now(-1), stored=True)
    ms.node_counter = cfg["rows"]
    snaps.clear()
    import lazzaro_amd.engine.tenant_graph as tgm
    for s, (convs, V) in enumerate(steps):
        real = tgm.time.time
        tgm.time.time = lambda s=s: _now(s)
        try:
            snaps.append("batch")
            ms.consolidate_batch(convs, embeddings=V, now=_now(s), commit="conversation")
        finally:
            tgm.time.time = real
        single = list(snaps)
    ms.close()
    MemorySystem._save_to_persistence = orig
    return parts, single


@pytest.mark.parametrize("world", [2, 3])
def test_sharded_tenant_commit_per_conversation(world):
    """commit="conversation" on the row-sharded tenant: every rank commits
    after each conversation of the batch, and the union of the ranks' k-th
    commits is the single process's k-th commit (commit="conversation",
    reference hierarchy) -- a crash loses at most the conversation in flight."""
    cfg = dict(HIER, sthr=62, steps=2)
    parts, single = spawn(world, functools.partial(_commit_snaps, cfg=cfg))[0]
    n_commits = [len(p) for p in parts]
    assert len(set(n_commits)) == 1 and n_commits[0] == len(single)
    assert sum(1 for x in single if x != "batch") >= 2 * CONVS  # one per conversation (+ the batch ends)
    for k, want in enumerate(single):
        if want == "batch":
            assert all(p[k] == "batch" for p in parts)
            continue
        nodes, edges = {}, {}
        for p in parts:
            nodes.update(p[k][0])
            edges.update(p[k][1])
        assert nodes == want[0], k
        assert set(edges) == set(want[1]), k
