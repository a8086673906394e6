"""``MemorySystem.consolidate_batch`` equals B sequential ``end_conversation``
calls at the reference's cadence: a buffer limit that
evicts in most conversations, ``run_consolidation`` every 3 conversations,
super-nodes created mid-batch, duplicates against the graph and against
earlier conversations of the batch, links, decay + prune. The whole graph
(nodes with salience / access / timestamps / parents, ghost rows, edges with
weights), the profile and the evicted ids must be identical, bit for bit."""
import hashlib
import json

import numpy as np
import pytest
import torch

DIM = 32
TOPICS = ("work", "personal", "learning", "health")


class TopicEmbedder:
    """text -> unit vector: its topic's centre + seeded noise (same-topic facts
    have cosine ~0.7, so they link; a repeated text is an exact duplicate)."""
    centres = {t: np.random.default_rng(i + 5).standard_normal(DIM) for i, t in enumerate(TOPICS)}

    def _v(self, text):
        topic = next((t for t in TOPICS if t in text), "work")
        c = self.centres[topic] / np.linalg.norm(self.centres[topic])
        seed = int.from_bytes(hashlib.md5(text.encode()).digest()[:4], "little")
        n = np.random.default_rng(seed).standard_normal(DIM)
        v = c + 0.1 * n
        return (v / np.linalg.norm(v)).astype(np.float32).tolist()

    def embed(self, t):
        return self._v(t)

    def batch_embed(self, ts):
        return [self._v(t) for t in ts]


class ScriptLLM:
    """Extraction: the facts the conversation's single turn carries as JSON;
    profile: a summary that depends on the memories' topics and count only."""

    def completion(self, messages, response_format=None):
        sysmsg = messages[0]["content"]
        if sysmsg.startswith("Extract distinct"):
            mems = []
            for m in json.loads(messages[1]["content"]):
                if m["content"].startswith("FACTS:"):
                    mems += json.loads(m["content"][6:])
            return json.dumps({"memories": mems})
        if sysmsg.startswith("Analyze these related memories"):
            lines = [l[2:] for l in messages[1]["content"].split("\n")[1:]]
            topics = "/".join(sorted({t for l in lines for t in TOPICS if t in l}))
            return json.dumps({"preferences": f"Likes {topics}", "knowledge_domains": f"{len(lines)} memories"})
        return "ok"


def conversations(B, seed=3):
    rng = np.random.default_rng(seed)
    pool = [f"User {t} fact {k}" for t in TOPICS for k in range(6)]
    out = []
    for c in range(B):
        facts = []
        for _ in range(int(rng.integers(1, 5))):
            base = pool[int(rng.integers(len(pool)))]
            text = base if rng.random() < 0.35 else f"{base} variant {c}.{len(facts)}"
            h = int(rng.integers(1 << 30))
            topic = next(t for t in TOPICS if t in text)
            facts.append({"content": text, "type": ("semantic", "episodic", "procedural")[h % 3],
                          "salience": round(0.3 + (h % 60) / 100.0, 2), "topic": topic})
        out.append(facts)
    return out


def _system(tmp, device, **kw):
    from lazzaro_amd.core.memory_system import MemorySystem
    cfg = dict(max_buffer_size=18, super_node_threshold=5, consolidate_every=3)
    cfg.update(kw)
    return MemorySystem(llm_provider=ScriptLLM(), embedding_provider=TopicEmbedder(), enable_async=False,
                        load_from_disk=False, db_dir=str(tmp), device=device, enable_caching=False, **cfg)


def _state(ms):
    g = ms.graph
    n = g.n
    cols = {k: getattr(g, k)[:n].cpu().numpy().tolist() for k in ("sal", "acc", "last", "kind", "sup", "shard",
                                                                    "parent", "stored")}
    e = {k: v.cpu().numpy().tolist() for k, v in g.e.items()}
    return {"ids": g.ids[:n], "content": g.content[:n], "types": g.types[:n], "cols": cols, "edges": e,
            "children": {g.ids[r]: list(v) for r, v in g.children.items()}, "profile": dict(ms.profile.data),
            "count": ms.conversation_count, "counter": ms.node_counter,
            "shards": {k: g.shard_count[c] for k, c in g.shard_code.items()}}


def _run_pair(tmp_path, monkeypatch, device, B, **kw):
    import time as _time
    monkeypatch.setattr(_time, "time", lambda: 1_900_000_000.0)
    convs = conversations(B)
    seq = _system(tmp_path / "seq", device, **kw)
    for facts in convs:
        seq.start_conversation()
        seq.add_to_short_term("FACTS:" + json.dumps(facts), "episodic", 0.7)
        seq.end_conversation()
    bat = _system(tmp_path / "bat", device, **kw)
    half = B // 2  # two batches: the second starts from a graph with evictions, supers and edges
    s1 = bat.consolidate_batch(convs[:half], now=1_900_000_000.0)
    s2 = bat.consolidate_batch(convs[half:], now=1_900_000_000.0)
    return _state(seq), _state(bat), (s1, s2)


@pytest.mark.parametrize("B,kw", [(24, {}), (30, {"max_buffer_size": 10, "super_node_threshold": 20}),
                                  (21, {"prune_threshold": 0.3, "consolidate_every": 2}),
                                  (18, {"auto_prune": False})])
def test_batch_equals_sequential_cpu(tmp_path, monkeypatch, B, kw):
    a, b, (s1, s2) = _run_pair(tmp_path, monkeypatch, "cpu", B, **kw)
    assert s1["evicted"] + s2["evicted"] > 0 and s1["dup"] + s2["dup"] > 0
    assert s1["consolidations"] + s2["consolidations"] == B // kw.get("consolidate_every", 3)
    for k in a:
        assert a[k] == b[k], k


def test_batch_equals_sequential_with_supers_and_links(tmp_path, monkeypatch):
    a, b, (s1, s2) = _run_pair(tmp_path, monkeypatch, "cpu", 27, max_buffer_size=40, super_node_threshold=4)
    assert any(a["cols"]["sup"]) and s1["linked"] + s2["linked"] > 0
    for k in a:
        assert a[k] == b[k], k


def test_batch_plan_pool_retry_is_exact(tmp_path, monkeypatch):
    """A pool far smaller than the victims it must hold: the planner detects
    it (PoolTooSmall) and the retry with a larger pool is still exact."""
    from lazzaro_amd.core import consolidation as C
    orig = C.ConsolidationMixin._plan_inputs

    def small(self, *a, **k):
        out = orig(self, *a, **k)
        out["P0"] = min(out["P0"], 2)
        return out
    monkeypatch.setattr(C.ConsolidationMixin, "_plan_inputs", small)
    a, b, (s1, s2) = _run_pair(tmp_path, monkeypatch, "cpu", 24, max_buffer_size=12)
    assert s1.get("pool_retries", 0) + s2.get("pool_retries", 0) > 0
    for k in a:
        assert a[k] == b[k], k


def test_batch_plan_list_fallback_is_exact(tmp_path, monkeypatch):
    """Candidate lists of 2 rows run out as the batch evicts their rows: the
    planner recomputes them exactly over the rows still present."""
    from lazzaro_amd.core import consolidation as C
    monkeypatch.setattr(C.ConsolidationMixin, "BATCH_LIST_K", 2)
    a, b, (s1, s2) = _run_pair(tmp_path, monkeypatch, "cpu", 30, max_buffer_size=9, super_node_threshold=50)
    assert s1["fallbacks"] + s2["fallbacks"] > 0
    for k in a:
        assert a[k] == b[k], k


def test_batch_pairwise_merge_mode_is_sequential(tmp_path, monkeypatch):
    """merge_mode="pairwise" changes the graph inside run_consolidation: the
    batch then runs the sequential bodies one by one (still equal)."""
    a, b, _ = _run_pair(tmp_path, monkeypatch, "cpu", 12, merge_mode="pairwise")
    for k in a:
        assert a[k] == b[k], k


@pytest.mark.gpu
@pytest.mark.parametrize("native", ["lazy", "eager", False])
@pytest.mark.parametrize("B,kw", [(30, {"max_buffer_size": 16, "super_node_threshold": 5}), (24, {}),
                                  (30, {"max_buffer_size": 10, "super_node_threshold": 20}),
                                  (21, {"prune_threshold": 0.3, "consolidate_every": 2}),
                                  (27, {"max_buffer_size": 40, "super_node_threshold": 4})])
def test_batch_equals_sequential_gpu(tmp_path, monkeypatch, native, B, kw):
    """The GPU batch path -- through the native segment applier
    (csrc/kernels/apply.hip, engine/native_apply.py; its node-salience decay
    lazy (per-row stamps, one pass per run) or eager (a pass per segment))
    and through the per-segment Python path -- equals the sequential
    end_conversation run."""
    from lazzaro_amd.core import consolidation as C
    from lazzaro_amd.engine import native_apply as NA
    monkeypatch.setattr(C.ConsolidationMixin, "NATIVE_APPLY", bool(native))
    monkeypatch.setattr(NA, "LAZY_NODE_DECAY", native == "lazy")
    runs = []
    orig = C.ConsolidationMixin._native_run

    def counted(self, segs, *a, **k):
        runs.append(len(segs))
        return orig(self, segs, *a, **k)
    monkeypatch.setattr(C.ConsolidationMixin, "_native_run", counted)
    a, b, (s1, s2) = _run_pair(tmp_path, monkeypatch, "cuda", B, **kw)
    assert s1["evicted"] + s2["evicted"] > 0
    assert (sum(runs) > 0) == bool(native)  # the native applier ran (and only when enabled)
    for k in a:
        assert a[k] == b[k], k


def test_batch_commit_per_conversation(tmp_path, monkeypatch):
    """commit="conversation": a segment per conversation, each committed as it
    is applied -- every commit sees the graph the sequential run persisted
    after the same end_conversation (a crash loses at most the conversation
    in flight, as in the reference)."""
    import time as _time

    from lazzaro_amd.core.memory_system import MemorySystem
    monkeypatch.setattr(_time, "time", lambda: 1_900_000_000.0)
    snaps = {"seq": [], "bat": []}
    orig = MemorySystem._save_to_persistence

    def rec(self):  # the state each commit leaves (stored / dirty bits included)
        out = orig(self)
        snaps[self._tag].append(_state(self))
        return out
    monkeypatch.setattr(MemorySystem, "_save_to_persistence", rec)
    B = 15
    convs = conversations(B)
    seq = _system(tmp_path / "seq", "cpu")
    seq._tag = "seq"
    for facts in convs:
        seq.start_conversation()
        seq.add_to_short_term("FACTS:" + json.dumps(facts), "episodic", 0.7)
        seq.end_conversation()
    bat = _system(tmp_path / "bat", "cpu")
    bat._tag = "bat"
    st = bat.consolidate_batch(convs, now=1_900_000_000.0, commit="conversation")
    assert st["evicted"] > 0 and st["consolidations"] == B // 3
    assert len(snaps["bat"]) == B + 1  # + the batch-end commit (nothing left to write)
    # the sequential end_conversation commits twice (reference :785 inside the
    # consolidation, :648 after it); the second is the conversation's state
    assert len(snaps["seq"]) == 2 * B
    for c in range(B):
        a, b = snaps["seq"][2 * c + 1], snaps["bat"][c]
        for k in a:
            if k == "shards":  # the batch registers its shards up front (empty ones are not persisted)
                a[k], b[k] = ({s: n for s, n in x[k].items() if n} for x in (a, b))
            assert a[k] == b[k], (c, k)
    with pytest.raises(ValueError):
        bat.consolidate_batch(convs[:1], commit="sometimes")


@pytest.mark.parametrize("lookahead", [1, 2, 5])
def test_consolidate_stream_equals_sequential_cpu(tmp_path, monkeypatch, lookahead):
    """``consolidate_stream`` over three batches is the sequential run (on the
    CPU the next batch's scan is not prefetched: the stream plumbing only;
    the prefetched GPU path is tests/kernels/test_tenant_engine_gpu.py::
    test_consolidate_stream_matches_batches_gpu), however many batches it
    draws ahead (``lookahead`` 5 > the stream's length)."""
    import time as _time
    monkeypatch.setattr(_time, "time", lambda: 1_900_000_000.0)
    B = 24
    convs = conversations(B)
    seq = _system(tmp_path / "seq", "cpu")
    for facts in convs:
        seq.start_conversation()
        seq.add_to_short_term("FACTS:" + json.dumps(facts), "episodic", 0.7)
        seq.end_conversation()
    st = _system(tmp_path / "st", "cpu")
    embs = [None] * 3  # the embedder runs per batch
    parts = [convs[:8], convs[8:16], convs[16:]]
    drawn = []

    def gen():
        for p, e in zip(parts, embs):
            drawn.append(len(drawn))
            yield p, e, 1_900_000_000.0
    it = st.consolidate_stream(gen(), lookahead=lookahead)
    first = next(it)
    # before batch 1's counts are handed back, exactly `lookahead` batches
    # past batch 0 were drawn (bounded by the stream's length)
    assert len(drawn) == min(3, 1 + lookahead)
    stats = [first] + list(it)
    assert len(stats) == 3 and sum(s["conversations"] for s in stats) == B
    a, b = _state(seq), _state(st)
    for k in a:
        assert a[k] == b[k], k
