"""Exact cross-rank pruning of the row-sharded consolidation scan
(parallel/sharded_memory.py ``prune`` / ``placement``).

Each rank bounds, per fine k-means cluster it holds, the angle between the
cluster's centroid and its farthest member; a fact is scanned on a rank only
if some cluster there can reach cos > LINK_THRESHOLD (every decision reads
only entries above it). On clustered data homed one topic per rank, the
8-rank gloo run must reach exactly the state of the unpruned run (nodes,
saliences, access counts, edges, per-batch counts), while each rank's
facts x rows counter falls."""
import random
import tempfile

import torch

from tests.distributed.test_dist_gloo import spawn

DIM = 48
WORLD = 8
PER_RANK = 60
STEPS = 3
CONVS = 3


def _unit(x):
    return x / x.norm(dim=-1, keepdim=True)


def _data():
    g = torch.Generator().manual_seed(3)
    centers = _unit(torch.randn(WORLD, DIM, generator=g))
    rows = [_unit(centers[r] + 0.02 * torch.randn(PER_RANK, DIM, generator=g)) for r in range(WORLD)]
    rng = random.Random(4)
    steps = []
    for s in range(STEPS):
        per_rank = []
        for r in range(WORLD):
            convs, vecs = [], []
            for c in range(CONVS):
                facts = []
                for f in range(rng.randint(1, 3)):
                    kind = rng.random()
                    base = rows[r][rng.randrange(PER_RANK)]
                    if kind < 0.25:
                        v = _unit(base + 0.002 * torch.randn(DIM, generator=g))  # duplicate of a stored row
                    elif kind < 0.85:
                        v = _unit(base + 0.12 * torch.randn(DIM, generator=g))  # related: links
                    else:
                        v = _unit(torch.randn(DIM, generator=g))  # unrelated
                    facts.append({"content": f"fact {s}.{r}.{c}.{f}", "type": "semantic",
                                  "salience": round(rng.uniform(0.3, 0.95), 6), "topic": ("work", "life")[f % 2]})
                    vecs.append(v)
                convs.append(facts)
            per_rank.append((convs, torch.stack(vecs)))
        steps.append(per_rank)
    return rows, steps


def _state(g):
    from lazzaro_amd.engine.tenant_graph import NODE
    n = g.n
    kind, sal, acc = g.kind[:n].tolist(), g.sal[:n].tolist(), g.acc[:n].tolist()
    nodes = {g.ids[r]: (sal[r], acc[r]) for r in range(n) if kind[r] == NODE}
    e = g.e
    edges = {(g.ids[s], g.ids[d]): w for s, d, w in zip(e["src"].tolist(), e["dst"].tolist(), e["w"].tolist())}
    return nodes, edges


def _run(comm, prune):
    from lazzaro_amd.core.providers import HashEmbedder, LocalLLM
    from lazzaro_amd.parallel.sharded_memory import ShardedMemorySystem
    rows, steps = _data()
    ShardedMemorySystem.FAR_MAX = 64
    sm = ShardedMemorySystem(comm, "pr", max_buffer_size=WORLD * PER_RANK + 10, llm_provider=LocalLLM(),
                             embedding_provider=HashEmbedder(dim=DIM), db_dir=tempfile.mkdtemp(), device="cpu",
                             hierarchy_params={"fine": 16, "top": 8, "every": 10 ** 6, "iters": 4},
                             prune=prune, placement="cluster")
    r = comm.rank
    sm.add_memories([f"memory {r}.{i}" for i in range(PER_RANK)], rows[r], ["work"] * PER_RANK, now=1.7e9)
    sm.cluster_pass()
    stats = []
    for s, per_rank in enumerate(steps):
        convs, V = per_rank[r]
        stats.append(sm.consolidate_batch(convs, embeddings=V, now=1.7e9 + 3600 * (s + 1)))
    nodes, edges = _state(sm.g)
    work = sm.scan_work
    parts = comm.all_gather_object((nodes, edges, work))
    sm.close()
    nodes_all, edges_all = {}, {}
    for n_, e_, _ in parts:
        nodes_all.update(n_)
        edges_all.update(e_)
    return {"stats": stats, "nodes": nodes_all, "edges": edges_all, "work": [p[2] for p in parts]}


def _both(comm):
    return {"pruned": _run(comm, True), "full": _run(comm, False)}


def test_pruned_scan_is_exact_and_cheaper_8_ranks():
    out = spawn(WORLD, _both)
    a, b = out[0]["pruned"], out[0]["full"]
    assert a["stats"] == b["stats"]
    assert sum(s["linked"] for s in b["stats"]) > 0 and sum(s["dup"] for s in b["stats"]) > 0
    assert a["nodes"] == b["nodes"] and len(a["nodes"]) >= WORLD * PER_RANK
    assert a["edges"] == b["edges"] and a["edges"]
    for r in range(WORLD):
        assert out[r]["pruned"]["stats"] == a["stats"]
    # every rank scanned every fact unpruned; pruned, a rank scans mostly its own topic's facts
    assert max(a["work"]) * 3 < min(b["work"]), (a["work"], b["work"])
