"""Behavioural tests of the orchestrator against the reference semantics
(SURVEY.md App. A/B/C): consolidation, linking, eviction, hierarchy, async
mode, multi-tenancy, snapshots."""
import json

import numpy as np
import pytest

from lazzaro_amd.core.memory_system import MemorySystem
from lazzaro_amd.core.providers import HashEmbedder, LocalLLM, ScriptedLLM
from lazzaro_amd.models.graph import Edge, Node


class VecEmbedder:
    """Maps text -> preset vector (unit axis or given list) for exact control."""

    def __init__(self, table, dim=8):
        self.table, self.dim = table, dim

    def _v(self, t):
        v = self.table.get(t)
        if v is None:
            v = [0.0] * self.dim
            v[hash(t) % self.dim] = 1.0
        return list(v)

    def embed(self, t):
        return self._v(t)

    def batch_embed(self, ts):
        return [self._v(t) for t in ts]


def facts_json(*facts):
    return json.dumps({"memories": [dict(content=c, type="semantic", salience=s, topic=tp) for c, s, tp in facts]})


def test_chain_and_similarity_links_then_prune():
    a = [1, 0, 0, 0, 0, 0, 0, 0]
    b = [0.9, 0.43589, 0, 0, 0, 0, 0, 0]  # cos(a,b)=0.9
    emb = VecEmbedder({"User likes tea": a, "User likes green tea": b})
    llm = ScriptedLLM([facts_json(("User likes tea", 0.6, "personal"), ("User likes green tea", 0.6, "personal"))])
    ms = MemorySystem(llm_provider=llm, embedding_provider=emb, enable_async=False, load_from_disk=False,
                      max_buffer_size=100)
    ms.start_conversation()
    ms.add_to_short_term("I like tea")
    res = ms.end_conversation()
    assert "Auto-pruned 1 weak edges" in res  # chain edge 0.5 -> 0.495 < 0.5
    assert ms.buffer.size() == (2, 0)
    ms.close()


def test_within_shard_links_to_existing():
    v = {f"User fact {i}": [1.0 if j == i else 0.0 for j in range(8)] for i in range(3)}
    v["User new fact"] = [0.8, 0.6, 0, 0, 0, 0, 0, 0]
    emb = VecEmbedder(v)
    llm = ScriptedLLM([facts_json(*[(f"User fact {i}", 0.9, "work") for i in range(3)]),
                       facts_json(("User new fact", 0.9, "work"))])
    ms = MemorySystem(llm_provider=llm, embedding_provider=emb, enable_async=False, load_from_disk=False,
                      max_buffer_size=100, auto_prune=False)
    for _ in range(2):
        ms.start_conversation()
        ms.add_to_short_term("x")
        ms.end_conversation()
    sh = ms.shards["work"]
    new_id = [n.id for n in sh.nodes.values() if n.content == "User new fact"][0]
    w = {k: e.weight for k, e in sh.edges.items() if k[0] == new_id}
    # cos 0.8 and 0.6 to facts 0 and 1 (> 0.5) -> weights 0.8*cos, decayed once
    assert len(w) == 2
    assert sorted(round(x, 4) for x in w.values()) == sorted(round(0.8 * c * 0.99, 4) for c in (0.8, 0.6))
    assert [n.content for n in ms.get_connected_memories(new_id)] in (["User fact 0", "User fact 1"],
                                                                      ["User fact 1", "User fact 0"])
    ms.close()


def test_buffer_limit_evicts_least_important():
    ms = MemorySystem(llm_provider=LocalLLM(), embedding_provider=HashEmbedder(), enable_async=False,
                      load_from_disk=False, max_buffer_size=2)
    for i, s in enumerate([0.9, 0.1, 0.5]):
        n = Node(id=f"node_{i}", content=f"c{i}", embedding=[float(i + 1)] * 4, salience=s)
        ms._get_or_create_shard("default").add_node(n)
    ms.store.add_nodes([n.to_dict() for n in ms.shards["default"].nodes.values()], ms.user_id)
    ms._enforce_buffer_limit()
    assert set(ms.buffer.nodes) == {"node_0", "node_2"}
    assert "node_1" not in ms.store.search_nodes([2.0] * 4, ms.user_id, limit=3)
    ms.close()


def test_super_nodes_and_hierarchical_retrieval():
    ms = MemorySystem(llm_provider=LocalLLM(), embedding_provider=HashEmbedder(dim=64), enable_async=False,
                      load_from_disk=False, max_buffer_size=1000, super_node_threshold=5)
    emb = HashEmbedder(dim=64)
    for i in range(7):
        txt = f"User works on project alpha task {i}"
        ms._get_or_create_shard("work").add_node(Node(id=f"node_{i+1}", content=txt, embedding=emb.embed(txt)))
    ms.node_counter = 7
    ms._create_super_nodes_for_shard("work")
    assert len(ms.super_nodes) == 1
    sup = next(iter(ms.super_nodes.values()))
    assert sup.is_super_node and len(sup.child_ids) == 7
    assert np.allclose(sup.embedding, np.mean([n.embedding for n in ms.shards["work"].nodes.values()], axis=0))
    ms._create_super_nodes_for_shard("work")  # one per shard
    assert len(ms.super_nodes) == 1
    ids = ms._optimized_retrieval(emb.embed("project alpha task"), "project alpha task")
    assert len(ids) == 5 and all(i in ms.shards["work"].nodes for i in ids)
    ms.close()


def test_async_consolidation_and_flush():
    ms = MemorySystem(llm_provider=LocalLLM(), embedding_provider=HashEmbedder(), enable_async=True,
                      load_from_disk=False, max_buffer_size=100)
    ms.start_conversation()
    ms.chat("I started a new job at a robotics company today.")
    r = ms.end_conversation()
    assert "consolidation queued" in r
    ms.flush()
    assert ms.buffer.size()[0] >= 1 and ms.metrics["consolidation_times"]
    ms.close()


def test_switch_user_isolates_tenants():
    ms = MemorySystem(llm_provider=LocalLLM(), embedding_provider=HashEmbedder(), enable_async=False,
                      user_id="alice", max_buffer_size=100)
    ms.start_conversation()
    ms.chat("My favorite color is green and I love sailing.")
    ms.end_conversation()
    n_alice = ms.buffer.size()[0]
    assert n_alice >= 1
    ms.switch_user("bob")
    assert ms.buffer.size()[0] == 0 and ms.user_id == "bob"
    assert ms.search_memories("sailing") == []
    ms.switch_user("alice")
    assert ms.buffer.size()[0] == n_alice
    assert sorted(ms.get_all_users()) == ["alice"]
    assert ms.search_memories("sailing green")
    ms.close()


def test_save_load_state_roundtrip(tmp_path):
    ms = MemorySystem(llm_provider=LocalLLM(), embedding_provider=HashEmbedder(), enable_async=False,
                      load_from_disk=False)
    ms._get_or_create_shard("work").add_node(Node(id="node_1", content="a", embedding=[1.0, 0.0]))
    ms._get_or_create_shard("work").add_node(Node(id="node_2", content="b", embedding=[0.0, 1.0]))
    ms.shards["work"].add_edge(Edge(source="node_1", target="node_2", weight=0.7))
    ms.profile.update_domain("preferences", "tea")
    ms.max_buffer_size = 42
    p = str(tmp_path / "s.json")
    ms.save_state(p)
    ms2 = MemorySystem(llm_provider=LocalLLM(), embedding_provider=HashEmbedder(), load_from_disk=False)
    assert ms2.load_state(p) == f"✓ State loaded from {p}"
    assert ms2.buffer.get_node("node_2").content == "b" and ms2.max_buffer_size == 42
    assert ms2.buffer.get_neighbors("node_1") == ["node_2"] and ms2.profile.data["preferences"] == "tea"
    assert ms2.load_state(str(tmp_path / "missing.json")).startswith("⚠ File")
    ms.close()
    ms2.close()


def test_merge_modes():
    def build(mode):
        ms = MemorySystem(llm_provider=LocalLLM(), embedding_provider=HashEmbedder(), enable_async=False,
                          load_from_disk=False, merge_mode=mode)
        sh = ms._get_or_create_shard("default")
        for i, v in enumerate([[1, 0], [1, 0.001], [0, 1], [1, 0]]):
            sh.add_node(Node(id=f"node_{i}", content=f"c{i}", embedding=list(map(float, v)), access_count=1))
        sh.add_edge(Edge(source="node_1", target="node_2", weight=0.9))
        return ms
    ms = build("reference")
    assert ms._merge_similar_nodes() == 0  # reference no-op (indentation bug preserved)
    ms = build("pairwise")
    assert ms._merge_similar_nodes() == 2
    n0 = ms.buffer.get_node("node_0")
    assert n0.content == "c0 | c1 | c3" and n0.access_count == 3
    assert ms.buffer.get_neighbors("node_0") == ["node_2"]


def test_stats_and_exports():
    ms = MemorySystem(llm_provider=LocalLLM(), embedding_provider=HashEmbedder(), enable_async=False,
                      load_from_disk=False)
    ms.start_conversation()
    ms.chat("I am learning Japanese from a book.")
    ms.chat("I am learning Japanese from a book.")
    s = ms.get_stats()
    assert set(s) >= {"buffer_nodes", "buffer_edges", "num_shards", "num_super_nodes", "short_term_memories",
                      "conversation_active", "conversation_count", "profile_domains_filled", "auto_consolidate",
                      "vector_store", "performance"}
    assert s["performance"]["cache_hit_rate"].endswith("%") and s["short_term_memories"] == 4
    assert "SCALABLE MEMORY SYSTEM STATS" in ms.display_stats()
    ms.end_conversation()
    md = ms.export_observations()
    assert md.startswith("# Memory Observations for default")
    assert isinstance(json.loads(ms.export_observations("json")), list)
    assert ms.get_insights()
    assert "User Profile" in ms.display_profile()
    ms.close()


def test_run_consolidation_fallback_profile_from_contents():
    ms = MemorySystem(llm_provider=LocalLLM(), embedding_provider=HashEmbedder(), enable_async=False,
                      load_from_disk=False)
    for i, c in enumerate(["User loves jazz music.", "User prefers tea over coffee.", "User has 5 years of "
                           "experience in Rust."]):
        ms._get_or_create_shard("default").add_node(Node(id=f"n{i}", content=c, embedding=[1.0, float(i)]))
    r = ms.run_consolidation()
    assert "Updated profile domains" in r and ms.profile.data["preferences"]
    ms.close()


def test_config_and_tracing(monkeypatch):
    from lazzaro_amd.config import MemoryConfig
    from lazzaro_amd.utils.tracing import tracer
    monkeypatch.setenv("LZK_MAX_BUFFER_SIZE", "77")
    monkeypatch.setenv("LZK_ENABLE_ASYNC", "false")
    monkeypatch.setenv("LZK_HIERARCHY_MODE", "kmeans")
    monkeypatch.setenv("LZK_HIERARCHY_EVERY", "7")
    cfg = MemoryConfig.from_env(load_from_disk=False, merge_mode="pairwise")
    assert cfg.max_buffer_size == 77 and cfg.enable_async is False
    assert set(cfg.reference_kwargs()) >= {"max_buffer_size", "db_dir", "user_id"}
    ms = MemorySystem.from_config(cfg, llm_provider=LocalLLM(), embedding_provider=HashEmbedder())
    assert ms.max_buffer_size == 77 and ms.merge_mode == "pairwise" and not ms.enable_async
    assert ms.hierarchy_mode == "kmeans" and ms.hierarchy_params["every"] == 7
    tracer.enable(True)
    tracer.reset()
    try:
        ms.start_conversation()
        ms.chat("I enjoy long walks on the beach.")
        ms.search_memories("beach")
        ms.end_conversation()
        s = tracer.summary()
        assert {"embed_query", "retrieve", "llm", "search", "ingest"} <= set(s)
        assert s["retrieve"]["calls"] == 1
    finally:
        tracer.enable(False)
    ms.close()


def test_concurrent_chat_and_background_consolidation():
    """Readers (chat/search) and the async consolidation writer share the
    graph under the graph lock: no torn reads, no lost memories."""
    import threading

    ms = MemorySystem(llm_provider=LocalLLM(), embedding_provider=HashEmbedder(), enable_async=True,
                      load_from_disk=False, max_buffer_size=1000, consolidate_every=1000)
    errors = []
    stop = threading.Event()

    def reader():
        try:
            while not stop.is_set():
                ms.search_memories("hobby music city")
                ms.get_stats()
        except Exception as e:  # pragma: no cover - the failure we guard against
            import traceback
            errors.append("".join(traceback.format_exception(e)))

    t = threading.Thread(target=reader)
    t.start()
    try:
        for i in range(12):
            ms.start_conversation()
            ms.chat(f"I moved to city number {i} and I love music genre {i}.")
            ms.end_conversation()
    finally:
        ms.flush()
        stop.set()
        t.join()
    assert not errors, errors
    assert ms.consolidation_queue == [] and ms.buffer.size()[0] >= 12
    ms.close()


def test_search_memories_stream_matches_batch(tmp_path):
    from lazzaro_amd.core.providers import HashEmbedder, LocalLLM
    ms = MemorySystem(llm_provider=LocalLLM(), embedding_provider=HashEmbedder(dim=32), enable_async=False,
                      db_dir=str(tmp_path), load_from_disk=False, max_buffer_size=10 ** 6)
    g = ms.graph
    rng = np.random.default_rng(0)
    X = rng.standard_normal((500, 32)).astype(np.float32)
    g.add_nodes([f"node_{i + 1}" for i in range(500)], [f"m{i}" for i in range(500)], X.tolist(),
                shard=g.shard_id("work"), stored=True)
    batches = [[f"q {b} {j}" for j in range(7)] for b in range(4)]
    want = [[[n.id for n in r] for r in ms.search_memories_batch(qs, limit=5)] for qs in batches]
    got = [[[n.id for n in r] for r in res] for res in ms.search_memories_stream(batches, limit=5)]
    assert got == want and all(len(r) == 5 for b in got for r in b)
    assert [[n.id for n in ms.search_memories(q, limit=5)] for q in batches[0]] == want[0]
    ms.close()


@pytest.mark.parametrize("device", ["cpu", pytest.param("cuda", marks=pytest.mark.gpu)])
@pytest.mark.parametrize("ne,seed", [(300, 3), (1500, 4), (120, 5)])
def test_component_digest_matches_materialised_components(ne, seed, device):
    """run_consolidation's device digest == the per-component reference logic
    (size >= 3, mean edge weight > 0.3, first 10 live shard-node rows), for
    many small components, one giant component and a sparse graph (GPU: the
    digest.hip keyed-reduction kernels)."""
    import torch

    from lazzaro_amd.engine.tenant_graph import NODE, TenantGraph
    rng = np.random.default_rng(seed)
    g = TenantGraph(device=device, dim=8)
    n = 400
    codes = [g.shard_id(f"s{i}") for i in range(4)]
    g.add_nodes([f"node_{i}" for i in range(n)], [f"c{i}" for i in range(n)],
                rng.standard_normal((n, 8)).astype(np.float32).tolist(), shard=[codes[i % 4] for i in range(n)],
                sup=[1 if i % 97 == 0 else 0 for i in range(n)])
    s = torch.as_tensor(rng.integers(0, n, ne), dtype=torch.int32)
    d = torch.as_tensor(rng.integers(0, n, ne), dtype=torch.int32)
    g.append_edges(s, d, torch.as_tensor(rng.uniform(0.1, 1.0, ne), dtype=torch.float32),
                   torch.as_tensor([codes[int(x) % 4] for x in s], dtype=torch.int32))
    g.remove_nodes([5, 6, 7, 50])  # ghosts that are still edge endpoints
    comps = g.components()
    ws, wc = g.component_edge_stats(comps)
    kind, sup = g.mirror("kind"), g.mirror("sup")
    want = []
    for i, c in enumerate(comps):
        if c.size < 3 or not wc[i] or not ws[i] / wc[i] > 0.3:
            continue
        rows = [r for r in c.tolist() if kind[r] == NODE and not sup[r]][:10]
        if rows:
            want.append(rows)
    got = [r.tolist() for r in g.component_digest(3, 0.3, 10)]
    assert got == want and len(want) >= 1


def _batch_scenario(seed=0, n_conv=7, per=5, dim=16):
    rng = np.random.default_rng(seed)
    centers = rng.standard_normal((4, dim))
    pool = []
    convs = []
    for c in range(n_conv):
        fs = []
        for j in range(per):
            r = rng.random()
            if pool and r < 0.25:  # near-duplicate of an earlier fact (cos > 0.95)
                base = pool[rng.integers(len(pool))][1]
                v = base + 0.02 * rng.standard_normal(dim)
            else:  # related to a topic centre (links with cos > 0.5)
                v = centers[rng.integers(4)] + 0.6 * rng.standard_normal(dim)
            v = v / np.linalg.norm(v)
            content = f"fact {c}.{j} about things"
            topic = ["work", "personal", "learning"][rng.integers(3)]
            fs.append({"content": content, "type": "semantic", "salience": float(rng.uniform(0.3, 0.9)),
                       "topic": topic})
            pool.append((content, v))
        convs.append(fs)
    return convs, {c: v.tolist() for c, v in pool}


def _graph_state(ms):
    nodes = {n.content: (n.shard_key, n.salience, n.access_count) for n in ms.buffer.nodes.values()}
    edges = {}
    for sk, sh in ms.shards.items():
        for (s, t), e in sh.edges.items():
            edges[(sk, ms.buffer.get_node(s).content, ms.buffer.get_node(t).content)] = (round(e.weight, 6),
                                                                                         e.co_occurrence)
    return nodes, edges




@pytest.mark.parametrize("seed", [0, 1, 2, 3])
def test_consolidate_batch_equals_sequential_end_conversations(tmp_path, seed):
    """B conversations through consolidate_batch == B sequential
    end_conversation calls (dedupe incl. earlier conversations of the batch,
    within-shard + cross links, decay + prune in closed form)."""
    convs, table = _batch_scenario(seed)
    seed = [[{"content": f"seed memory {i}", "type": "semantic", "salience": 0.7,
              "topic": ["work", "personal", "learning"][i % 3]} for i in range(6)]]
    rng = np.random.default_rng(9)
    for i in range(6):
        v = rng.standard_normal(16)
        table[f"seed memory {i}"] = (v / np.linalg.norm(v)).tolist()
    kw = dict(enable_async=False, load_from_disk=False, max_buffer_size=10 ** 6, consolidate_every=10 ** 6,
              super_node_threshold=10 ** 6)
    # sequential reference
    seq = MemorySystem(llm_provider=ScriptedLLM([json.dumps({"memories": f}) for f in seed + convs]),
                       embedding_provider=VecEmbedder(table, 16), db_dir=str(tmp_path / "a"), **kw)
    for _ in range(len(seed) + len(convs)):
        seq.start_conversation()
        seq.add_to_short_term("conversation text")
        seq.end_conversation()
    # batched: the seed conversation sequentially, then one batch
    bat = MemorySystem(llm_provider=ScriptedLLM([json.dumps({"memories": f}) for f in seed]),
                       embedding_provider=VecEmbedder(table, 16), db_dir=str(tmp_path / "b"), **kw)
    bat.start_conversation()
    bat.add_to_short_term("conversation text")
    bat.end_conversation()
    flat = [f for c in convs for f in c]
    st = bat.consolidate_batch(convs, embeddings=np.asarray([table[f["content"]] for f in flat], np.float32))
    a, b = _graph_state(seq), _graph_state(bat)
    assert st["dup"] > 0 and st["linked"] > 0 and st["inserted"] + st["dup"] == len(flat)
    assert a[0].keys() == b[0].keys()
    for k in a[0]:
        assert a[0][k][0] == b[0][k][0] and a[0][k][2] == b[0][k][2] and abs(a[0][k][1] - b[0][k][1]) < 1e-5, k
    assert a[1].keys() == b[1].keys() and len(a[1]) > 0
    for k in a[1]:
        assert abs(a[1][k][0] - b[1][k][0]) < 1e-5 and a[1][k][1] == b[1][k][1], k
    assert seq.conversation_count == bat.conversation_count
    seq.close()
    bat.close()


def test_kmeans_hierarchy_mode_clusters_and_retrieves(tmp_path):
    """hierarchy_mode="kmeans": a two-level k-means pass over the tenant after
    every `every` conversations; retrieval's hierarchical step returns members
    of the query's topic cluster (reference super-node step, :464-482)."""
    rng = np.random.default_rng(4)
    dim = 16
    centers = rng.standard_normal((4, dim))
    centers /= np.linalg.norm(centers, axis=1, keepdims=True)
    convs, vecs = [], []
    for c in range(12):
        fs = []
        for j in range(5):
            k = (c * 5 + j) % 4
            v = centers[k] + 0.15 * rng.standard_normal(dim)
            vecs.append(v / np.linalg.norm(v))
            fs.append({"content": f"cluster {k} fact {c}.{j}", "salience": 0.6, "topic": "work"})
        convs.append(fs)
    ms = MemorySystem(llm_provider=LocalLLM(), embedding_provider=VecEmbedder({}, dim), enable_async=False,
                      load_from_disk=False, db_dir=str(tmp_path), max_buffer_size=10 ** 6, consolidate_every=10 ** 6,
                      hierarchy_mode="kmeans", hierarchy_params={"fine": 8, "top": 4, "every": 5, "iters": 4})
    ms.consolidate_batch(convs, embeddings=np.asarray(vecs, np.float32))
    g = ms.graph
    assert g.hier and g.hier["top_c"].shape[0] == 4 and ms.get_stats()["num_super_nodes"] == 0
    # the last pass ran at conversation 10 (every 5, exact cadence): it covers
    # the rows that existed then
    tops = g.hier["top"][: g.n].tolist()
    # facts of one generating centre share a topic cluster
    by_center = {}
    for r in range(len(tops)):
        if g.kind_h(r) == 1:
            by_center.setdefault(g.content[r].split()[1], set()).add(tops[r])
    assert all(len(v) == 1 for v in by_center.values()) and len({min(v) for v in by_center.values()}) == 4
    q = centers[2]
    ids = ms._optimized_retrieval(q.tolist(), "a query near centre 2")
    assert len(ids) == 5 and all(ms.buffer.get_node(i).content.startswith("cluster 2") for i in ids)
    ms.close()


def test_ordered_node_rows_dev_matches_host():
    import torch

    from lazzaro_amd.engine.tenant_graph import TenantGraph
    g = TenantGraph(device="cpu", dim=4)
    codes = [g.shard_id(f"s{i}") for i in range(3)]
    rng = np.random.default_rng(1)
    n = 300
    g.add_nodes([f"n{i}" for i in range(n)], [""] * n, rng.standard_normal((n, 4)).astype(np.float32).tolist(),
                shard=[codes[int(x)] for x in rng.integers(0, 3, n)], sup=[1 if i % 50 == 7 else 0 for i in range(n)])
    g.remove_nodes([3, 4, 100])
    assert g.ordered_node_rows_dev().tolist() == g.ordered_node_rows().tolist()
    host = g.ordered_node_rows()
    assert g.ordered_node_rows_dev(super_=False).tolist() == host[g.mirror("sup")[host] == 0].tolist()


def test_evict_select_matches_full_sort_with_ties():
    """Eviction's radix-select + top-k path == the full (importance, shard,
    row) order, with heavy score ties (reference :541-578 victim order)."""
    import torch

    from lazzaro_amd.engine.tenant_graph import TenantGraph
    from lazzaro_amd.ops import tenant_ops as T
    rng = np.random.default_rng(2)
    n = 20000
    g = TenantGraph(device="cpu", dim=4)
    codes = [g.shard_id(f"s{i}") for i in range(4)]
    sh = rng.integers(0, 4, n)
    g.add_nodes([f"n{i}" for i in range(n)], [""] * n, rng.standard_normal((n, 4)).astype(np.float32).tolist(),
                shard=[codes[int(x)] for x in sh], sal=rng.choice([0.3, 0.5, 0.7], n).astype(np.float32),
                acc=rng.integers(0, 3, n), last=np.full(n, 1000.0), sup=[1 if i % 997 == 0 else 0 for i in range(n)])
    now = 5000.0
    score = T.importance(g.sal[:n], g.acc[:n], g.last[:n], g.kind[:n], g.sup[:n], now).numpy()
    okey = np.asarray(g.shard[:n]).astype(np.int64) * (1 << 32) + np.arange(n)
    excess = 150
    want = np.lexsort((okey, score))[:excess].tolist()
    got = g.evict(g.num_nodes() - excess, now=now)
    assert got == want


def test_kmeans_minibatch_sample_matches_quality():
    """kmeans(sample=...): refinement steps on a random subset, last step on
    all rows -- every masked-in row labelled, clusters recovered."""
    import torch
    from lazzaro_amd.index.kmeans import kmeans
    g = torch.Generator().manual_seed(0)
    C, per, d = 8, 400, 32
    cen = torch.nn.functional.normalize(torch.randn(C, d, generator=g), dim=1)
    X = torch.nn.functional.normalize(cen.repeat_interleave(per, 0) + 0.05 * torch.randn(C * per, d, generator=g), dim=1)
    mask = torch.rand(C * per, generator=g) > 0.05
    c32, _, lab = kmeans(X, C, iters=4, seed=1, mask=mask, sample=500)
    assert bool((lab[mask] >= 0).all()) and bool((lab[~mask] == -1).all())
    pure = sum(len(set(lab[j * per:(j + 1) * per][mask[j * per:(j + 1) * per]].tolist())) == 1 for j in range(C))
    assert pure >= C - 1


def test_two_level_assign_matches_full_on_separated_topics():
    """assign_two_level (fine clusters searched under the nearest topic only)
    equals the full assign when topics are well separated."""
    import torch
    from lazzaro_amd.index.kmeans import assign, assign_two_level
    g = torch.Generator().manual_seed(3)
    d, T, per = 32, 4, 6
    tops = torch.nn.functional.normalize(torch.randn(T, d, generator=g), dim=1)
    fine = torch.nn.functional.normalize(tops.repeat_interleave(per, 0) + 0.2 * torch.randn(T * per, d, generator=g),
                                         dim=1)
    top_of = torch.arange(T).repeat_interleave(per)
    X = torch.nn.functional.normalize(fine[torch.randint(0, T * per, (3000,), generator=g)]
                                      + 0.05 * torch.randn(3000, d, generator=g), dim=1)
    l_full, _ = assign(X, fine)
    l_two, _ = assign_two_level(X, fine, tops, top_of)
    assert (l_full.long() == l_two.long()).float().mean() > 0.99


def test_get_stats_engine_block():
    """get_stats keeps the reference's keys and adds the engine metrics
    (device, HBM bytes of the tenant graph, search throughput)."""
    ms = MemorySystem(llm_provider=LocalLLM(), embedding_provider=HashEmbedder(dim=32), enable_async=False,
                      load_from_disk=False)
    ms.start_conversation()
    ms.chat("I like sailing and my sister lives in Porto.")
    ms.end_conversation()
    ms.search_memories_batch(["sailing", "Porto", "sister"], limit=2)
    s = ms.get_stats()
    assert {"buffer_nodes", "buffer_edges", "performance"} <= set(s)
    e = s["engine"]
    assert e["search_queries"] == 3 and e["hbm_graph_bytes"] > 0 and e["search_qps"] > 0
    ms.close()


def test_ivfpq_index_under_the_tenant_graph(tmp_path):
    """MemorySystem(index="ivfpq"): a tenant above ivf_min_rows is searched
    through IVF-PQ candidates re-ranked exactly on the graph's fp32 rows --
    removed rows never come back, fresh rows are indexed on the next search."""
    import torch
    g0 = torch.Generator().manual_seed(0)
    C, per, d = 20, 200, 32
    cen = torch.nn.functional.normalize(torch.randn(C, d, generator=g0), dim=1)
    X = torch.nn.functional.normalize(cen.repeat_interleave(per, 0) + 0.3 * torch.randn(C * per, d, generator=g0), dim=1)
    ms = MemorySystem(llm_provider=LocalLLM(), embedding_provider=HashEmbedder(dim=d), enable_async=False,
                      load_from_disk=False, db_dir=str(tmp_path), index="ivfpq",
                      index_params={"nlist": 16, "nprobe": 16, "pq_m": 8, "ivf_min_rows": 1000})
    g = ms.graph
    g.add_nodes([f"m{i}" for i in range(len(X))], [f"c{i}" for i in range(len(X))], X, shard=g.shard_id("w"),
                stored=True)
    q = X[:40] + 0.01 * torch.randn(40, d, generator=g0)
    s, rows = g.store_search(q, 5, "l2")
    assert g._ann is not None and g._ann_covered == len(X)
    truth = torch.topk(-torch.cdist(q, X), 5, dim=1).indices
    hit = sum(len(set(a.tolist()) & set(b.tolist())) for a, b in zip(rows, truth)) / truth.numel()
    assert hit > 0.95
    g.remove_nodes([0], unstore=True)
    _, rows = g.store_search(X[:1], 3, "l2")
    assert 0 not in rows[0].tolist()
    g.add_nodes(["fresh"], ["f"], X[5:6] * 1.0, shard=g.shard_id("w"), stored=True)
    _, rows = g.store_search(X[5:6], 2, "l2")
    assert g._ann_covered == g.n and set(rows[0].tolist()) == {5, g.n - 1}
    ms.close()


@pytest.mark.parametrize("fail", [False, True])
def test_write_behind_persistence_equals_sync(tmp_path, fail):
    """persist_async=True: commits run on the writer thread, in order; what a
    fresh MemorySystem reloads equals the synchronous run's store. With an
    injected commit failure the snapshot is kept and retried before the next
    one, so nothing is lost."""
    from lazzaro_amd.utils.faults import injector

    convs, table = _batch_scenario(5, n_conv=6)
    kw = dict(enable_async=False, max_buffer_size=20, consolidate_every=2, super_node_threshold=10 ** 6)

    def run(db, persist_async):
        ms = MemorySystem(llm_provider=ScriptedLLM([json.dumps({"memories": f}) for f in convs]),
                          embedding_provider=VecEmbedder(table, 16), db_dir=db, load_from_disk=False,
                          persist_async=persist_async, **kw)
        for i in range(len(convs)):
            if fail and persist_async and i == 2:
                injector.arm("store.commit", 1)
            ms.start_conversation()
            ms.add_to_short_term("conversation text")
            ms.end_conversation()
        ms.close()
        injector.disarm()
        back = MemorySystem(llm_provider=LocalLLM(), embedding_provider=VecEmbedder(table, 16), db_dir=db,
                            load_from_disk=True, **kw)
        st = _graph_state(back)
        back.close()
        return st, ms.metrics.get("persist_failures", 0)

    (a, _), (b, nfail) = run(str(tmp_path / "sync"), False), run(str(tmp_path / "wb"), True)
    assert a[0].keys() == b[0].keys() and len(a[0]) > 0
    for k in a[0]:
        assert a[0][k][0] == b[0][k][0] and abs(a[0][k][1] - b[0][k][1]) < 1e-6, k
    assert a[1] == b[1]
    assert nfail == (1 if fail else 0)


def test_first_shard_rows_fast_path_matches_topk(monkeypatch):
    """first_node_rows_dev(super_=False) on a large tenant walks the shards in
    code order through growing row windows (host shard counts); it must equal
    the one-pass top-k over every row, after removals and with super-nodes."""
    import torch

    from lazzaro_amd.engine.tenant_graph import TenantGraph
    rng = np.random.default_rng(7)
    g = TenantGraph(device="cpu", dim=4)
    codes = [g.shard_id(f"s{i}") for i in range(5)]
    n = 3000
    sh = rng.choice([codes[1], codes[3], codes[4]], n, p=[0.01, 0.5, 0.49]).tolist()
    g.add_nodes([f"node_{i}" for i in range(n)], [f"c{i}" for i in range(n)],
                rng.standard_normal((n, 4)).astype(np.float32).tolist(), shard=sh,
                sup=(rng.random(n) < 0.05).astype(np.int64).tolist())
    g.remove_nodes(rng.choice(n, 400, replace=False).tolist())
    monkeypatch.setattr(TenantGraph, "FIRST_ROWS_WINDOW", 64)
    for k in (1, 10, 40):
        fast = g._first_shard_rows(k).tolist()
        monkeypatch.setattr(TenantGraph, "FIRST_ROWS_WINDOW", 1 << 30)
        ref = g.first_node_rows_dev(k, super_=False).tolist()
        monkeypatch.setattr(TenantGraph, "FIRST_ROWS_WINDOW", 64)
        assert fast == ref and len(ref) == k
        assert g.first_node_rows_dev(k, super_=False).tolist() == ref


def test_farthest_first_large_sample_path():
    """A tenant larger than 4x the farthest-first sample draws it without a
    permutation of every row: deterministic, distinct seeds, unit rows."""
    import torch

    from lazzaro_amd.index.kmeans import _farthest_first
    X = torch.randn(200_000, 16, generator=torch.Generator().manual_seed(0))
    X /= X.norm(dim=1, keepdim=True)
    a, b = _farthest_first(X, 64, seed=1), _farthest_first(X, 64, seed=1)
    assert a.shape == (64, 16) and torch.equal(a, b)
    assert torch.unique(a, dim=0).shape[0] == 64
