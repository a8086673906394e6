"""MemorySystem: the agent-memory orchestrator (reference
``src/lazzaro/core/memory_system.py:21-1550``).

Public API, constructor kwargs and defaults are the reference's (SURVEY.md
App. A/B) so existing code switches by changing the import. The engine under
it is MI355X-first:

* vectors live in per-tenant HBM arenas (``HBMStore``); search, dedupe, super
  node scoring and linking are batched device/host GEMMs with fused top-k
  (``lazzaro_amd.ops``), never per-pair Python loops;
* persistence is the native versioned columnar store;
* embeddings can run on-device (``core.embedders.OnDeviceEmbedder``: BERT-family
  encoders on hand-written MFMA GEMM / attention / LayerNorm kernels);
* background consolidation is serialised against the caller with a graph lock.

Constructor additions (all keyword, all optional): ``device``, ``metric``
(store search metric, default "l2" like LanceDB), ``merge_mode``
("reference" | "pairwise"), ``verbose`` (print status lines like the reference).
"""
from __future__ import annotations

import json
import logging
import os
import threading
import time
from concurrent.futures import ThreadPoolExecutor
from typing import Dict, List, Optional

import numpy as np

from ..models.graph import Edge, Node
from . import providers as _providers
from .buffer_graph import BufferGraph
from .consolidation import ConsolidationMixin
from .interfaces import EmbeddingProvider, LLMProvider, Store
from .memory_shard import MemoryShard
from .profile import EMPTY_CONTEXT, Profile
from .providers import HashEmbedder, LocalLLM, OpenAIEmbedder, OpenAILLM, cosine
from .query_cache import QueryCache
from .similarity import EmbeddingCache, topk_cosine
from .vector_store import HBMStore
from ..utils.faults import StoreError, degenerate_embedding, fault_point
from ..utils.tracing import tracer

# kept for parity with code/tests that patch `...memory_system.openai`
openai = _providers.openai

log = logging.getLogger("lazzaro_amd")

SYSTEM_PROMPT = ("You are a helpful assistant with access to the user's profile and past memories. "
                 "Use the provided context ONLY if it is relevant to the user's current query. "
                 "Do not force the information if it doesn't fit naturally.")
SHARD_KEYWORDS = {
    "work": ["work", "project", "meeting", "deadline", "client", "colleague"],
    "personal": ["family", "friend", "hobby", "home", "personal"],
    "learning": ["learn", "study", "course", "book", "tutorial", "practice"],
    "health": ["health", "exercise", "diet", "sleep", "medical", "fitness"],
}
HISTORY_WINDOW = 10
SUPER_MATCH = 0.4
SUPER_CHILDREN = 10
RESULT_LIMIT = 5


class MemorySystem(ConsolidationMixin):
    def __init__(
        self,
        openai_api_key: Optional[str] = None,
        model: str = "gpt-4o-mini",
        enable_sharding: bool = True,
        enable_hierarchy: bool = True,
        enable_caching: bool = True,
        enable_async: bool = True,
        max_shard_size: int = 500,
        super_node_threshold: int = 20,
        auto_consolidate: bool = True,
        consolidate_every: int = 3,
        auto_prune: bool = True,
        prune_threshold: float = 0.5,
        max_buffer_size: int = 10,
        load_from_disk: bool = True,
        llm_provider: Optional[LLMProvider] = None,
        embedding_provider: Optional[EmbeddingProvider] = None,
        db_dir: str = "db",
        user_id: str = "default",
        store: Optional[Store] = None,
        *,
        device=None,
        metric: str = "l2",
        merge_mode: str = "reference",
        verbose: bool = False,
        strict_errors: bool = False,
        max_consolidation_retries: int = 3,
        index: str = "flat",
        index_params: Optional[Dict] = None,
    ):
        self.model = model
        self.user_id = user_id
        self.verbose = verbose
        key = openai_api_key or os.environ.get("OPENAI_API_KEY")
        if llm_provider is not None:
            self.llm = llm_provider
        elif key:
            self.llm = OpenAILLM(api_key=key, model=model)
        else:
            self.llm = LocalLLM()
        if embedding_provider is not None:
            self.embedder = embedding_provider
        elif key:
            self.embedder = OpenAIEmbedder(api_key=key)
        else:
            self.embedder = _default_local_embedder()

        self.shards: Dict[str, MemoryShard] = {}
        self.super_nodes: Dict[str, Node] = {}
        self.buffer = BufferGraph(self.shards, self.super_nodes)
        self.profile = Profile()
        self.store = store if store is not None else HBMStore(db_dir=db_dir, device=device, metric=metric,
                                                              index=index, **(index_params or {}))
        self.vector_store = self.store
        self._device = getattr(self.store, "device", None)
        if isinstance(self._device, str):
            import torch
            self._device = torch.device(self._device)

        self.enable_sharding = enable_sharding
        self.enable_hierarchy = enable_hierarchy
        self.enable_caching = enable_caching
        self.enable_async = enable_async
        self.max_shard_size = max_shard_size  # accepted for parity; unused (as in the reference)
        self.super_node_threshold = super_node_threshold
        self.auto_consolidate = auto_consolidate
        self.consolidate_every = consolidate_every
        self.auto_prune = auto_prune
        self.prune_threshold = prune_threshold
        self.max_buffer_size = max_buffer_size
        self.merge_mode = merge_mode
        # failure policy: strict -> typed errors propagate;
        # otherwise failures are counted in metrics and work is retried
        self.strict_errors = strict_errors
        self.max_consolidation_retries = max_consolidation_retries
        self._persist_pending = False

        self.query_cache = QueryCache(max_size=1000) if enable_caching else None
        self.consolidation_queue: List[Dict] = []
        # one worker: consolidations of a tenant are applied in order
        self.background_executor = ThreadPoolExecutor(max_workers=1) if enable_async else None
        self._pending = []
        self._queue_lock = threading.Lock()
        self._graph_lock = threading.RLock()
        self._emb_cache = EmbeddingCache()

        self.conversation_active = False
        self.short_term_memory: List[Dict] = []
        self.conversation_history: List[Dict] = []
        self.node_counter = 0
        self.conversation_count = 0
        self.metrics = {"embedding_calls": 0, "llm_calls": 0, "retrieval_times": [],
                        "consolidation_times": [], "consolidation_failures": 0, "dropped_batches": 0,
                        "persist_failures": 0, "rejected_embeddings": 0}
        if load_from_disk:
            self._load_from_persistence()

    @classmethod
    def from_config(cls, cfg=None, **kw) -> "MemorySystem":
        """Build from a :class:`lazzaro_amd.config.MemoryConfig` (env-aware)."""
        from ..config import MemoryConfig

        cfg = cfg or MemoryConfig.from_env()
        emb = kw.pop("embedding_provider", None)
        if emb is None and cfg.embed_model:
            from .embedders import OnDeviceEmbedder
            emb = OnDeviceEmbedder(cfg.embed_model, device=cfg.device, weights=cfg.embed_weights)
        kw.setdefault("index", cfg.index)
        kw.setdefault("index_params", {"nlist": cfg.nlist, "nprobe": cfg.nprobe, "pq_m": cfg.pq_m,
                                       "ivf_min_rows": cfg.ivf_min_rows})
        return cls(**cfg.reference_kwargs(), embedding_provider=emb, device=cfg.device, metric=cfg.metric,
                   merge_mode=cfg.merge_mode, verbose=cfg.verbose, **kw)

    # ------------------------------------------------------------ helpers
    def _say(self, msg: str) -> None:
        log.info(msg)
        if self.verbose:
            print(msg)

    def _generate_node_id(self) -> str:
        self.node_counter += 1
        return f"node_{self.node_counter}"

    def _infer_shard_key(self, content: str) -> str:
        if not self.enable_sharding:
            return "default"
        low = content.lower()
        for key, terms in SHARD_KEYWORDS.items():
            if any(t in low for t in terms):
                return key
        return time.strftime("%Y-%m")

    def _get_or_create_shard(self, shard_key: str) -> MemoryShard:
        sh = self.shards.get(shard_key)
        if sh is None:
            sh = self.shards[shard_key] = MemoryShard(shard_key)
        return sh

    def _get_embedding(self, text: str) -> List[float]:
        self.metrics["embedding_calls"] += 1
        if self.query_cache:
            hit = self.query_cache.get_embedding(text)
            if hit:
                return hit
        fault_point("provider.embed")
        emb = self.embedder.embed(text)
        if self.query_cache and not degenerate_embedding(emb):
            self.query_cache.set_embedding(text, emb)
        return emb

    def _batch_embed(self, texts: List[str]) -> List[List[float]]:
        if not texts:
            return []
        self.metrics["embedding_calls"] += 1
        fault_point("provider.embed")
        return self.embedder.batch_embed(texts)

    def _cosine_similarity(self, v1, v2) -> float:
        return cosine(v1, v2)

    def _call_llm(self, messages: List[Dict], response_format: Dict = None) -> str:
        self.metrics["llm_calls"] += 1
        fault_point("provider.llm")
        return self.llm.completion(messages, response_format)

    def _search_batch(self, embs: List[List[float]], k: int) -> List[List[str]]:
        fn = getattr(self.vector_store, "search_nodes_batch", None)
        if fn is not None:
            return fn(embs, user_id=self.user_id, limit=k)
        return [self.vector_store.search_nodes(e, user_id=self.user_id, limit=k) for e in embs]

    # ------------------------------------------------------------ conversation
    def start_conversation(self) -> str:
        self.conversation_active = True
        self.short_term_memory = []
        self.conversation_history = []
        return "✓ Conversation started"

    def add_to_short_term(self, content: str, memory_type: str = "semantic", salience: float = 0.5):
        if not self.conversation_active:
            raise RuntimeError("No active conversation")
        self.short_term_memory.append({"content": content, "type": memory_type, "salience": salience,
                                       "timestamp": time.time()})
        self._auto_save_if_needed()

    def _auto_save_if_needed(self):
        pass  # persistence happens at end of conversation / consolidation (reference :238-240)

    # ------------------------------------------------------------ retrieval
    def _boost_neighbors(self, retrieved_ids: List[str]):
        neigh = []
        seen = set()
        for nid in retrieved_ids:
            for nb in self.buffer.get_neighbors(nid):
                if nb not in seen:
                    seen.add(nb)
                    neigh.append(nb)
        count = 0
        now = time.time()
        for nid in neigh:
            if nid in retrieved_ids:
                continue
            n = self.buffer.get_node(nid)
            if n is not None:
                n.last_accessed = now
                n.salience = min(1.0, n.salience + 0.02)
                count += 1
        if count:
            self._say(f"   (Graph: Boosted {count} neighbor nodes via association)")

    def _optimized_retrieval(self, query_emb: List[float], query_text: str) -> List[str]:
        if self.query_cache:
            cached = self.query_cache.get_results(query_text)
            if cached:
                return cached
        retrieved: List[str] = []
        if self.enable_hierarchy and self.super_nodes:
            sup = list(self.super_nodes.values())
            q = np.asarray(query_emb, dtype=np.float64)
            qn = np.linalg.norm(q)
            qu = q / qn if qn > 0 else q
            S = self._emb_cache.matrix(sup, dim=qu.shape[0])
            sims, idx = topk_cosine(qu[None, :], S, 1)
            if idx[0, 0] >= 0 and sims[0, 0] > SUPER_MATCH:
                best = sup[idx[0, 0]]
                for cid in best.child_ids[:SUPER_CHILDREN]:
                    c = self.buffer.get_node(cid)
                    if c is not None and not c.is_super_node:
                        retrieved.append(cid)
                if len(retrieved) >= RESULT_LIMIT:
                    if self.query_cache:
                        self.query_cache.set_results(query_text, retrieved[:RESULT_LIMIT])
                    return retrieved[:RESULT_LIMIT]
        limit = 10 if not retrieved else 5
        vec_ids = self.vector_store.search_nodes(query_emb, user_id=self.user_id, limit=limit)
        seen_ids = set(retrieved)
        seen_content = set()
        final = []
        for rid in retrieved:
            n = self.buffer.get_node(rid)
            if n is not None:
                seen_content.add(n.content)
                final.append(rid)
        for rid in vec_ids:
            if rid in seen_ids:
                continue
            n = self.buffer.get_node(rid)
            if n is not None and n.content not in seen_content:
                seen_content.add(n.content)
                final.append(rid)
                seen_ids.add(rid)
        final = final[:RESULT_LIMIT]
        if self.query_cache:
            self.query_cache.set_results(query_text, final)
        return final

    def _build_messages(self, retrieved_ids: List[str]) -> List[Dict]:
        parts = []
        pc = self.profile.get_context()
        if pc and pc != EMPTY_CONTEXT:
            parts.append(f"User Profile:\n{pc}\n")
        if retrieved_ids:
            texts = []
            for nid in retrieved_ids:
                n = self.buffer.get_node(nid)
                if n is not None:
                    texts.append(f"- {n.content}")
                    self.buffer.update_access(nid)
            if texts:
                parts.append("Relevant Information from Past Conversations (Use if relevant to the query):\n"
                             + "\n".join(texts) + "\n")
        msgs = [{"role": "system", "content": SYSTEM_PROMPT}]
        if parts:
            msgs.append({"role": "system", "content": "\n".join(parts)})
        msgs.extend(self.conversation_history[-HISTORY_WINDOW:])
        return msgs

    def _retrieve_for(self, user_message: str):
        if not self.conversation_active:
            self._say(self.start_conversation())
        t0 = time.time()
        self.add_to_short_term(user_message, "episodic", salience=0.7)
        self.conversation_history.append({"role": "user", "content": user_message})
        with tracer.stage("embed_query", self._device):
            q = self._get_embedding(user_message)
        # readers and the background consolidation writer serialise on the
        # graph lock (the reference mutates the graph from two worker threads
        # with no lock at all); the writer holds it only for
        # the on-device ingest, never across the LLM call
        with self._graph_lock:
            with tracer.stage("retrieve", self._device):
                ids = self._optimized_retrieval(q, user_message)
            with tracer.stage("boost", self._device):
                self._boost_neighbors(ids)
        return ids, (time.time() - t0) * 1000.0

    @staticmethod
    def _timing_line(ms: float, n: int) -> str:
        emoji = "⚡" if ms < 100 else ("✓" if ms < 200 else "⏱")
        return f"[{emoji} Retrieval: {ms:.0f}ms, Retrieved: {n} nodes]"

    def _node_lines(self, ids: List[str]) -> List[str]:
        out = []
        for nid in ids:
            n = self.buffer.get_node(nid)
            if n is not None:
                snip = n.content[:60] + "..." if len(n.content) > 60 else n.content
                out.append(f"   • [{nid}] ({n.shard_key}) {snip}")
        return out

    def chat(self, user_message: str) -> str:
        ids, ms = self._retrieve_for(user_message)
        self.metrics["retrieval_times"].append(ms)
        with self._graph_lock:
            msgs = self._build_messages(ids)
            node_lines = self._node_lines(ids)
        with tracer.stage("llm", "cpu"):
            response = self._call_llm(msgs)
        self.add_to_short_term(response, "semantic", salience=0.5)
        self.conversation_history.append({"role": "assistant", "content": response})
        self._say(self._timing_line(ms, len(ids)))
        if ids:
            self._say("   Retrieved Nodes:")
            for line in node_lines:
                self._say(line)
        return response

    def chat_stream(self, user_message: str):
        ids, ms = self._retrieve_for(user_message)
        with self._graph_lock:
            node_lines = self._node_lines(ids)
            msgs = self._build_messages(ids)
        yield {"type": "info", "content": self._timing_line(ms, len(ids))}
        if ids:
            yield {"type": "info", "content": "   Retrieved Nodes:"}
            for line in node_lines:
                yield {"type": "info", "content": line}
        if hasattr(self.llm, "completion_stream"):
            full = ""
            for chunk in self.llm.completion_stream(msgs):
                full += chunk
                yield {"type": "token", "content": chunk}
            self.add_to_short_term(full, "semantic", salience=0.5)
            self.conversation_history.append({"role": "assistant", "content": full})
        else:
            resp = self.llm.completion(msgs)
            self.add_to_short_term(resp, "semantic", salience=0.5)
            self.conversation_history.append({"role": "assistant", "content": resp})
            yield {"type": "token", "content": resp}

    def _get_relevant_shards(self, query: str, max_shards: int = 3) -> List[str]:
        """Recency/size shard ranking (present but unused in the reference, :516-533)."""
        if not self.enable_sharding or not self.shards:
            return ["default"]
        if len(self.shards) <= 5:
            return list(self.shards.keys())
        now = time.time()
        scored = []
        for k, sh in self.shards.items():
            rec = 1.0 / (1.0 + (now - sh.last_accessed) / 3600.0)
            scored.append((k, 0.7 * rec + 0.3 * min(1.0, len(sh.nodes) / 100)))
        scored.sort(key=lambda x: x[1], reverse=True)
        return [k for k, _ in scored[:max_shards]]

    # ------------------------------------------------------------ queries
    def get_connected_memories(self, node_id: str) -> List[Node]:
        with self._graph_lock:
            return self._connected(node_id)

    def _connected(self, node_id: str) -> List[Node]:
        ids = []
        seen = set()
        for sh in list(self.shards.values()):
            for s, t in sh.edges.incident(node_id):
                o = t if s == node_id else s
                if o not in seen:
                    seen.add(o)
                    ids.append(o)
        return [n for n in (self.buffer.get_node(i) for i in ids) if n is not None]

    def search_memories(self, query: str, limit: int = 5) -> List[Node]:
        with tracer.stage("embed_query", self._device):
            q = self._get_embedding(query)
        with tracer.stage("search", self._device):
            ids = self.vector_store.search_nodes(q, user_id=self.user_id, limit=limit)
        with self._graph_lock:
            return [n for n in (self.buffer.get_node(i) for i in ids) if n is not None]

    def search_memories_batch(self, queries: List[str], limit: int = 5) -> List[List[Node]]:
        """Batched search: one embedding call and one fused top-k launch."""
        embs = self._batch_embed(list(queries))
        res = self._search_batch(embs, limit)
        with self._graph_lock:
            return [[n for n in (self.buffer.get_node(i) for i in ids) if n is not None] for ids in res]

    # ------------------------------------------------------------ stats / display
    def get_stats(self) -> Dict:
        with self._graph_lock:
            return self._stats()

    def _stats(self) -> Dict:
        nodes, edges = self.buffer.size()
        rt = self.metrics["retrieval_times"]
        ct = self.metrics["consolidation_times"]
        avg_r = float(np.mean(rt)) if rt else 0.0
        p95_r = float(np.percentile(rt, 95)) if rt else 0.0
        avg_c = float(np.mean(ct)) if ct else 0.0
        hit = self.query_cache.get_hit_rate() if self.query_cache else 0.0
        return {
            "buffer_nodes": nodes,
            "buffer_edges": edges,
            "num_shards": len(self.shards),
            "num_super_nodes": len(self.super_nodes),
            "short_term_memories": len(self.short_term_memory),
            "conversation_active": self.conversation_active,
            "conversation_count": self.conversation_count,
            "profile_domains_filled": sum(1 for v in self.profile.data.values() if v),
            "auto_consolidate": self.auto_consolidate,
            "vector_store": f"{type(self.vector_store).__name__} (Active)" if self.vector_store is not None else "None",
            "performance": {
                "avg_retrieval_ms": f"{avg_r:.1f}",
                "p95_retrieval_ms": f"{p95_r:.1f}",
                "avg_consolidation_s": f"{avg_c:.2f}",
                "cache_hit_rate": f"{hit:.1%}",
                "llm_calls": self.metrics["llm_calls"],
                "embedding_calls": self.metrics["embedding_calls"],
            },
        }

    def display_stats(self) -> str:
        s = self.get_stats()
        p = s["performance"]
        nxt = self.consolidate_every - (self.conversation_count % self.consolidate_every)
        onoff = lambda b: "ON" if b else "OFF"  # noqa: E731
        return f"""
📊 SCALABLE MEMORY SYSTEM STATS:
STORAGE:
  • Buffer nodes: {s["buffer_nodes"]} / {self.max_buffer_size} max
  • Buffer edges: {s["buffer_edges"]}
  • Shards: {s["num_shards"]}
  • Super-nodes: {s["num_super_nodes"]}
  • STM: {s["short_term_memories"]}
  • Conversations: {s["conversation_count"]}
  • Profile domains: {s["profile_domains_filled"]}/5

⚡ PERFORMANCE:
  • Avg retrieval: {p["avg_retrieval_ms"]}ms
  • P95 retrieval: {p["p95_retrieval_ms"]}ms
  • Avg consolidation: {p["avg_consolidation_s"]}s
  • Cache hit rate: {p["cache_hit_rate"]}
  • LLM calls: {p["llm_calls"]}
  • Embedding calls: {p["embedding_calls"]}

⚙️ AUTO-MANAGEMENT:
  • Auto-consolidate: {onoff(s["auto_consolidate"])} (every {self.consolidate_every})
    → Next in: {nxt} conversation(s)
  • Auto-prune: {onoff(self.auto_prune)} (threshold: {self.prune_threshold})
  • Max buffer: {self.max_buffer_size} nodes
  • Sharding: {onoff(self.enable_sharding)}
  • Hierarchy: {onoff(self.enable_hierarchy)}
  • Caching: {onoff(self.enable_caching)}
  • Async: {onoff(self.enable_async)}
"""

    def display_memories(self, limit: int = 10) -> str:
        if not self.buffer.nodes:
            return "No memories stored yet."
        nodes = self.buffer.get_all_nodes_summary()
        out = [f"\n💭 Stored Memories (showing {min(limit, len(nodes))} of {len(nodes)}):"]
        for i, n in enumerate(nodes[:limit], 1):
            out.append(f"\n{i}. [{n['type']}] 📦 {n['shard']} (salience: {n['salience']:.2f}, "
                       f"accessed: {n['access_count']}x)")
            out.append(f"   {n['content']}")
        return "\n".join(out)

    def display_profile(self) -> str:
        return f"\n👤 User Profile:\n{self.profile.get_context()}\n"

    # ------------------------------------------------------------ JSON snapshot
    _SETTINGS = ("auto_consolidate", "consolidate_every", "auto_prune", "prune_threshold", "max_buffer_size")

    def save_state(self, filename: str = "memory_state.json") -> str:
        state = {
            "shards": {k: {"nodes": [n.to_dict() for n in sh.nodes.values()],
                           "edges": [e.to_dict() for e in sh.edges.values()]}
                       for k, sh in self.shards.items()},
            "super_nodes": [n.to_dict() for n in self.super_nodes.values()],
            "profile": self.profile.to_dict(),
            "node_counter": self.node_counter,
            "conversation_count": self.conversation_count,
            "settings": {k: getattr(self, k) for k in self._SETTINGS},
        }
        with open(filename, "w") as f:
            json.dump(state, f, indent=2)
        return f"✓ State saved to {filename}"

    def load_state(self, filename: str = "memory_state.json") -> str:
        try:
            with open(filename) as f:
                state = json.load(f)
        except FileNotFoundError:
            return f"⚠ File {filename} not found"
        with self._graph_lock:
            shards: Dict[str, MemoryShard] = {}
            for k, d in state.get("shards", {}).items():
                sh = MemoryShard(k)
                for nd in d.get("nodes", []):
                    sh.add_node(Node.from_dict(nd))
                for ed in d.get("edges", []):
                    sh.add_edge(Edge.from_dict(ed))
                shards[k] = sh
            self.shards = shards
            self.super_nodes = {n["id"]: Node.from_dict(n) for n in state.get("super_nodes", [])}
            self.buffer = BufferGraph(self.shards, self.super_nodes)  # reference forgets this
            pd = state.get("profile", {})
            self.profile.data = pd.get("data", self.profile.data)
            self.profile.last_updated = pd.get("last_updated", time.time())
            self.node_counter = state.get("node_counter", 0)
            self.conversation_count = state.get("conversation_count", 0)
            for k, v in state.get("settings", {}).items():
                if hasattr(self, k):
                    setattr(self, k, v)
        return f"✓ State loaded from {filename}"

    # ------------------------------------------------------------ store sync
    def _save_to_persistence(self):
        """Write the tenant's graph to the store (reference memory_system.py:
        1275-1302). With a native store the rewrite is one atomic version per
        table. A failed commit leaves the in-memory graph authoritative: it is
        counted, logged, and the next save rewrites everything again
        (``strict_errors`` raises :class:`StoreError` instead)."""
        with self._graph_lock:
            nodes = [n.to_dict() for n in self.buffer.nodes.values()]
            edges = [e.to_dict() for sh in self.shards.values() for e in sh.edges.values()]
            try:
                if hasattr(self.store, "replace_user_nodes"):
                    self.store.replace_user_nodes(nodes, user_id=self.user_id)
                    self.store.replace_user_edges(edges, user_id=self.user_id)
                else:  # third-party Store protocol: the reference's delete + add
                    self.store.delete_nodes([], user_id=self.user_id)
                    self.store.delete_edges(user_id=self.user_id)
                    if nodes:
                        self.store.add_nodes(nodes, user_id=self.user_id)
                    if edges:
                        self.store.add_edges(edges, user_id=self.user_id)
                self.store.save_profile(self.profile.to_dict(), user_id=self.user_id)
            except Exception as e:
                self.metrics["persist_failures"] = self.metrics.get("persist_failures", 0) + 1
                self._persist_pending = True
                log.warning("persistence failed for %s: %s", self.user_id, e)
                self._say(f"⚠ Persistence failed for user {self.user_id}: {e}")
                if self.strict_errors:
                    raise StoreError(str(e)) from e
                return
            self._persist_pending = False
            try:
                # our own write is not an "update from elsewhere" (reference
                # re-loads after its own saves)
                self._last_nodes_version = self.store.get_latest_version()
            except Exception:
                pass
            if self.query_cache:
                self.query_cache.invalidate_results()
        self._say(f"✓ State persisted for user: {self.user_id}")

    def _load_from_persistence(self):
        self._say(f"🔄 Loading state for user: {self.user_id}...")
        with self._graph_lock:
            rows = self.store.get_nodes(user_id=self.user_id)
            shards: Dict[str, MemoryShard] = {}
            supers: Dict[str, Node] = {}
            for nd in rows:
                nd = dict(nd)
                if "vector" in nd:
                    v = nd.pop("vector")
                    nd["embedding"] = v.tolist() if hasattr(v, "tolist") else list(v)
                if isinstance(nd.get("child_ids"), str):
                    try:
                        nd["child_ids"] = json.loads(nd["child_ids"])
                    except json.JSONDecodeError:
                        nd["child_ids"] = []
                n = Node.from_dict(nd)
                if n.is_super_node:
                    supers[n.id] = n
                else:
                    sh = shards.get(n.shard_key)
                    if sh is None:
                        sh = shards[n.shard_key] = MemoryShard(n.shard_key)
                    sh.add_node(n)
            edge_rows = self.store.get_edges(user_id=self.user_id) if rows else []
            for ed in edge_rows:
                ed = dict(ed)
                if "source_id" in ed:
                    ed["source"] = ed.pop("source_id")
                if "target_id" in ed:
                    ed["target"] = ed.pop("target_id")
                if "type" in ed and "edge_type" not in ed:
                    ed["edge_type"] = ed.pop("type")
                e = Edge.from_dict(ed)
                src = supers.get(e.source)
                if src is None:
                    for sh in shards.values():
                        if e.source in sh.nodes:
                            src = sh.nodes[e.source]
                            break
                if src is not None and src.shard_key in shards:
                    shards[src.shard_key].add_edge(e)
            prof = self.store.load_profile(user_id=self.user_id) if rows else None
            self.shards = shards
            self.super_nodes = supers
            self.buffer = BufferGraph(self.shards, self.super_nodes)
            self.profile = Profile.from_dict(prof) if prof else Profile()
            try:
                self._last_nodes_version = self.store.get_latest_version()
            except Exception:
                self._last_nodes_version = 0
            mx = 0
            for nid in self.buffer.nodes:
                if nid.startswith("node_"):
                    try:
                        mx = max(mx, int(nid.split("_")[1]))
                    except ValueError:
                        pass
            if rows:
                self.node_counter = mx
            if self.query_cache:
                self.query_cache.invalidate_results()
        if rows:
            self._say(f"✓ Restored state ({len(self.buffer.nodes)} nodes, {len(edge_rows)} edges)")
        else:
            self._say("ℹ No saved state found.")

    def check_for_updates(self) -> bool:
        try:
            v = self.store.get_latest_version()
            if not hasattr(self, "_last_nodes_version") or v > self._last_nodes_version:
                self._say(f"🔄 Store updated (v{v}), reloading...")
                self._load_from_persistence()
                return True
        except Exception:
            pass
        return False

    def get_all_users(self) -> List[str]:
        fn = getattr(self.store, "list_users", None)
        if fn is None:
            return [self.user_id]
        users = fn()
        return users if users else [self.user_id]

    def switch_user(self, new_user_id: str):
        if self.conversation_active:
            self.end_conversation()
            self.flush()
        else:
            self._save_to_persistence()
        self.user_id = new_user_id
        self._load_from_persistence()
        self._say(f"👤 Switched context to user: {new_user_id}")

    # ------------------------------------------------------------ export
    def export_observations(self, format: str = "markdown") -> str:
        with self._graph_lock:
            return self._export(format)

    def _export(self, format: str) -> str:
        nodes = [n for sh in self.shards.values() for n in sh.nodes.values() if not n.is_super_node]
        nodes.sort(key=lambda n: (n.salience, n.last_accessed), reverse=True)
        if format == "json":
            return json.dumps([n.to_dict() for n in nodes[:50]], indent=2)
        lines = [f"# Memory Observations for {self.user_id}", ""]
        for n in nodes[:50]:
            lines += [f"### {n.type.capitalize()} Memory ({n.shard_key})",
                      f"- **Content**: {n.content}",
                      f"- **Salience**: {n.salience:.2f}",
                      f"- **Last Accessed**: {time.ctime(n.last_accessed)}", ""]
        return "\n".join(lines)

    def get_insights(self) -> str:
        obs = self.export_observations(format="json")
        sys_prompt = f"""Analyze these atomic memories for user '{self.user_id}' and provide a comprehensive psychological and knowledge profile.
Identify long-term patterns, core beliefs, persistent interests, and significant life events reflected in the data.

Structure your response as:
1. **Personality Traits**: Key characteristics detected.
2. **Core Interests & Knowledge**: What the user knows and cares about.
3. **Behavioral Patterns**: How the user typically interacts or works.
4. **Recent Focus**: Most salient topics from recent memories.

Be clinical yet insightful. Do not include conversational filler."""
        return self._call_llm([{"role": "system", "content": sys_prompt},
                               {"role": "user", "content": f"User Observations:\n{obs}"}])

    def close(self):
        if self.background_executor:
            self.background_executor.shutdown(wait=True)
        if hasattr(self, "store") and self.store is not None:
            self.store.close()


def _default_local_embedder() -> EmbeddingProvider:
    """Offline default: on-device encoder when weights are configured
    (``LZK_ENCODER_WEIGHTS``), else the lexical hash embedder."""
    w = os.environ.get("LZK_ENCODER_WEIGHTS")
    if w:
        from .embedders import OnDeviceEmbedder
        return OnDeviceEmbedder(os.environ.get("LZK_ENCODER_MODEL", "minilm-l6"), weights=w)
    return HashEmbedder()
