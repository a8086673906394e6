"""One scripted scenario driven through either the REFERENCE MemorySystem
(/root/reference/src/lazzaro, pure Python; ``lancedb`` / ``openai`` replaced by
stubs that are never called, an in-memory Store injected through ``store=``,
as the SURVEY [probe] did) or ``lazzaro_amd.MemorySystem`` (its own HBMStore
on the CPU). Prints the final state as JSON. Run as a subprocess by
``test_reference_differential.py`` so the stubs never leak into the suite.

    python _differential_scenario.py ref|ours <db_dir>

Deterministic inputs shared by both sides:
* a clock: ``time.time`` returns a strictly increasing fake time (+1 ms per
  call), so creation order decides the eviction tie-breaks in both systems;
* an embedder: text -> unit vector = topic centre + seeded noise (facts of one
  topic have cosine ~0.7, so links form; a repeated fact text is an exact
  duplicate, so dedupe fires);
* an LLM that answers the extraction prompt from the ``FACTS:`` user turns in
  the conversation JSON, the profile prompt with an order-independent
  summary, and chat with a fixed reply.
"""
import hashlib
import json
import os
import sys
import types

import numpy as np

DIM = 48
TOPICS = ("work", "personal", "learning", "health", "other")
_T = [1_800_000_000.0]


def fake_time():
    _T[0] += 0.001
    return _T[0]


def _h(s: str) -> int:
    return int.from_bytes(hashlib.md5(s.encode()).digest()[:8], "little")


def _topic(text: str) -> str:
    for t in TOPICS:
        if f"[{t}]" in text:
            return t
    return "other"


class Embedder:
    centres = {t: np.random.default_rng(i + 1).standard_normal(DIM) for i, t in enumerate(TOPICS)}

    def _v(self, text):
        c = self.centres[_topic(text)]
        c = c / np.linalg.norm(c)
        noise = np.random.default_rng(_h(text) % (1 << 32)).standard_normal(DIM)
        v = c + 0.09 * noise
        return (v / np.linalg.norm(v)).astype(np.float64).tolist()

    def embed(self, text):
        return self._v(text)

    def batch_embed(self, texts):
        return [self._v(t) for t in texts]


class LLM:
    def completion(self, messages, response_format=None):
        sysmsg = messages[0]["content"] if messages and messages[0]["role"] == "system" else ""
        if sysmsg.startswith("Extract distinct, atomic facts"):
            mems = []
            for m in json.loads(messages[1]["content"]):
                c = m.get("content", "")
                if not c.startswith("FACTS:"):
                    continue
                for f in c[len("FACTS:"):].split("|"):
                    f = f.strip()
                    h = _h(f)
                    mems.append({"content": f, "type": ("semantic", "episodic", "procedural")[h % 3],
                                 "salience": round(0.35 + (h >> 8) % 60 / 100.0, 2), "topic": _topic(f)})
            return json.dumps({"memories": mems})
        if sysmsg.startswith("Analyze these related memories"):
            # a function of the topics and the count only: the reference picks
            # a component's first 10 contents in set-iteration order (string
            # hashing), so any 10 of a larger component must give one answer
            lines = [l[2:] for l in messages[1]["content"].split("\n")[1:]]
            topics = "/".join(sorted({_topic(l) for l in lines}))
            return json.dumps({"preferences": f"Likes {topics}", "knowledge_domains": f"{len(lines)} memories",
                               "key_experiences": f"Talked about {topics}"})
        return "Noted."

    def completion_stream(self, messages, response_format=None):
        yield self.completion(messages, response_format)


class MemStore:
    """In-memory Store protocol (reference interfaces.py:55-102) with a flat
    L2 search like LanceDB's default (ties by insertion order)."""

    def __init__(self):
        self.nodes, self.edges, self.profiles, self.version = {}, {}, {}, 0

    def add_nodes(self, nodes, user_id="default"):
        for n in nodes:
            self.nodes[(user_id, n["id"])] = dict(n, user_id=user_id)
        self.version += 1

    def get_nodes(self, user_id="default"):
        return [dict(v, vector=v.get("embedding")) for (u, _), v in self.nodes.items() if u == user_id]

    def search_nodes(self, query_vector, user_id="default", limit=5):
        rows = [(k[1], v) for k, v in self.nodes.items() if k[0] == user_id and v.get("embedding")]
        if not rows:
            return []
        q = np.asarray(query_vector, np.float64)
        d = [float(((np.asarray(v["embedding"], np.float64) - q) ** 2).sum()) for _, v in rows]
        order = np.argsort(np.asarray(d), kind="stable")[:limit]
        return [rows[i][0] for i in order]

    def delete_nodes(self, node_ids, user_id="default"):
        if not node_ids:
            self.nodes = {k: v for k, v in self.nodes.items() if k[0] != user_id}
        else:
            for i in node_ids:
                self.nodes.pop((user_id, i), None)
        self.version += 1

    def get_latest_version(self):
        return self.version

    def add_edges(self, edges, user_id="default"):
        for e in edges:
            src, tgt = e.get("source") or e.get("source_id"), e.get("target") or e.get("target_id")
            self.edges[(user_id, src, tgt)] = dict(e, user_id=user_id, source_id=src, target_id=tgt)

    def delete_edges(self, source_id=None, user_id="default"):
        self.edges = {k: v for k, v in self.edges.items() if k[0] != user_id or (source_id and k[1] != source_id)}

    def get_edges(self, user_id="default"):
        return [v for k, v in self.edges.items() if k[0] == user_id]

    def save_profile(self, profile_data, user_id="default"):
        self.profiles[user_id] = profile_data

    def load_profile(self, user_id="default"):
        return self.profiles.get(user_id)

    def close(self):
        pass


FACTS = {
    "work": ["User leads the [work] robotics project", "User meets the [work] client on Mondays",
             "User ships [work] releases every sprint", "User reviews [work] pull requests daily",
             "User mentors two [work] interns", "User owns the [work] deployment pipeline"],
    "personal": ["User has a [personal] dog named Rex", "User sails on [personal] weekends",
                 "User cooks [personal] Sunday dinners", "User visits [personal] family in Lisbon"],
    "learning": ["User studies [learning] Japanese grammar", "User reads a [learning] book on compilers",
                 "User takes a [learning] course on GPUs", "User practices [learning] piano scales"],
    "health": ["User runs [health] five kilometres", "User sleeps [health] eight hours",
               "User tracks [health] protein intake"],
}


def conversations(n=24):
    rng = np.random.default_rng(2024)
    topics = list(FACTS)
    out = []
    for c in range(n):
        turns = []
        for _ in range(2):
            t = topics[int(rng.integers(len(topics)))]
            k = int(rng.integers(1, 4))
            facts = []
            for _ in range(k):
                base = FACTS[t][int(rng.integers(len(FACTS[t])))]
                # half the facts repeat an earlier text (duplicates), half are new variants
                facts.append(base if rng.random() < 0.5 else f"{base} (note {c}.{len(facts)})")
            turns.append("FACTS: " + " | ".join(facts))
        out.append(turns)
    return out


# "pressure": a buffer that evicts every conversation, small shards get
# super-nodes, auto-consolidation every 3 conversations; "defaults": the
# reference's own constructor defaults (max_buffer_size=10, threshold 20)
CONFIGS = {"pressure": dict(max_buffer_size=26, super_node_threshold=6, consolidate_every=3),
           "defaults": dict()}


def state(ms):
    nodes, edges = {}, {}
    for key, sh in ms.shards.items():
        for nid, n in sh.nodes.items():
            nodes[nid] = {"content": n.content, "type": n.type, "salience": round(float(n.salience), 5),
                          "access_count": int(n.access_count), "shard": key, "parent": n.parent_id or ""}
        for (s, t), e in sh.edges.items():
            edges[f"{s}->{t}@{key}"] = round(float(e.weight), 5)
    sup = sorted([n.shard_key, sorted(n.child_ids)] for n in ms.super_nodes.values())
    return {"nodes": nodes, "edges": edges, "super": sup, "profile": dict(ms.profile.data),
            "conversation_count": ms.conversation_count, "node_counter": ms.node_counter}


def run(which, db):
    import time
    time.time = fake_time
    if which == "ref":
        for name, attr in (("openai", "OpenAI"), ("lancedb", "connect")):
            m = types.ModuleType(name)

            def _never(*a, **k):
                raise RuntimeError("stub: never called")
            setattr(m, attr, _never)
            sys.modules[name] = m
        sys.path.insert(0, "/root/reference/src")
        from lazzaro.core.memory_system import MemorySystem
        kw = dict(store=MemStore())
    else:
        from lazzaro_amd.core.memory_system import MemorySystem
        kw = dict(db_dir=db, device=os.environ.get("LZK_DIFF_DEVICE", "cpu"))
    # enable_caching=False: the reference never invalidates cached retrieval
    # results (a repeated query text returns the ids of its first retrieval,
    # even after consolidation changed the graph); lazzaro_amd drops cached
    # results whenever the tenant's index changes (docs/INVENTORY.md,
    # deliberate differences). Without the cache both recompute every time.
    ms = MemorySystem(llm_provider=LLM(), embedding_provider=Embedder(), enable_async=False, load_from_disk=False,
                      **CONFIGS[os.environ.get("LZK_DIFF_CFG", "pressure")],
                      enable_caching=os.environ.get("LZK_DIFF_CACHE") == "1", **kw)
    snaps = []
    trace = []
    if os.environ.get("LZK_DIFF_TRACE"):
        orig = ms._optimized_retrieval

        def traced(q, text):
            r = orig(q, text)
            trace.append([text[:40], list(r)])
            return r
        ms._optimized_retrieval = traced
    for c, turns in enumerate(conversations()):
        ms.start_conversation()
        for t in turns:
            ms.chat(t)
        ms.end_conversation()
        if c % 6 == 5 or os.environ.get("LZK_DIFF_EVERY"):
            snaps.append(state(ms))
    out = state(ms)
    out["snapshots"] = snaps
    out["trace"] = trace
    out["search"] = [[n.id for n in ms.search_memories(q, limit=4)]
                     for q in ("robotics project", "[health] running", "[learning] Japanese")]
    return out


if __name__ == "__main__":
    import contextlib
    import io
    buf = io.StringIO()
    with contextlib.redirect_stdout(buf):  # the reference prints progress lines
        res = run(sys.argv[1], sys.argv[2])
    print(json.dumps(res))
