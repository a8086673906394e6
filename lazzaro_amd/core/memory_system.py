"""MemorySystem: the agent-memory orchestrator (reference
``src/lazzaro/core/memory_system.py:21-1550``).

Public API, constructor kwargs and defaults are the reference's (SURVEY.md
App. A/B) so existing code switches by changing the import. Underneath, the
tenant's memory graph is a :class:`~lazzaro_amd.engine.TenantGraph`: node
and edge columns in HBM (``device=cuda``) or host memory (``device=cpu``),
and every graph operation -- dedupe, linking, decay/prune, eviction, neighbour
boost, components, super-node centroids, the store's vector search -- is a
HIP kernel or a batched tensor op on it (see :mod:`lazzaro_amd.engine`).
``shards`` / ``super_nodes`` / ``buffer`` and the ``Node`` / ``Edge`` objects
they hand out are façades over those columns (:mod:`lazzaro_amd.engine.views`).

* The default store (``HBMStore``) serves this tenant's vector search from the
  graph's own rows (one copy of the vectors in HBM) and persists changes
  incrementally: each commit writes the rows and edges that changed, plus
  deletions, instead of the reference's delete-all + add-all per save
  (:1275-1302). Temporal decay is not a row change: each row records the
  decay clock at which it was written and a reload replays the decay since.
* Embeddings can run on-device (``core.embedders.OnDeviceEmbedder``) and stay
  device tensors into the graph.
* Background consolidation is serialised against the caller with a graph lock.

Constructor additions (all keyword, all optional): ``device``, ``metric``
(store search metric, default "l2" like LanceDB), ``merge_mode``
("reference" | "pairwise"), ``verbose`` (print status lines like the reference).
"""
from __future__ import annotations

import collections
import contextlib
import gc
import json
import logging
import math
import os
import re
import threading
import time
from concurrent.futures import ThreadPoolExecutor
from typing import Dict, Iterable, List, Optional, Tuple

import numpy as np
import torch

from ..engine.tenant_graph import NODE, TYPE_MASK, TenantGraph
from ..engine.views import GraphBuffer, NodeView, ResultBatch, ShardView, ShardsMap, SuperNodesMap, import_edges, import_nodes
from ..models.graph import Edge, Node
from . import providers as _providers
from .consolidation import ConsolidationMixin
from .interfaces import EmbeddingProvider, LLMProvider, Store
from .memory_shard import MemoryShard
from .profile import EMPTY_CONTEXT, Profile
from .providers import HashEmbedder, LocalLLM, OpenAIEmbedder, OpenAILLM, cosine
from .query_cache import QueryCache
from .vector_store import HBMStore
from ..utils.faults import StoreError, degenerate_embedding, fault_point
from ..utils.tracing import tracer

# search_memories_stream: run each batch's store search on the graph's stream
# without the caller's stream waiting for it, so the next batch's embed
# overlaps the scan (SEARCH_OVERLAP = False joins the streams after each search;
# bench.py on one MI355X: 13.9 -> 13.3 ms per 1024-query step)
SEARCH_OVERLAP = True
# batches search_memories_stream keeps in flight behind the one the host maps
# (2: a host stall of up to a step -- tokenizer, result mapping, a collector
# pass -- is absorbed by queued device work instead of idling the GPU)
STREAM_DEPTH = 1
# result events the host waits on sleep instead of spin (BLOCKING_EVENTS = False: spin)
BLOCKING_EVENTS = True

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
SALIENCE_FLOOR = 0.2
_NODE_ID = re.compile(r"^node_(\d+)$")


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
        hierarchy_mode: str = "reference",
        hierarchy_params: Optional[Dict] = None,
        persist_async: bool = False,
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

        self.profile = Profile()
        # a store passed in may be shared by many tenants (the service's
        # factory): close() then only unbinds this tenant's graph from it
        self._owns_store = store is None
        self.store = store if store is not None else HBMStore(db_dir=db_dir, device=device, metric=metric,
                                                              index=index, **(index_params or {}))
        self.vector_store = self.store
        dev = device if device is not None else getattr(self.store, "device", None)
        self._device = torch.device(dev) if dev is not None else torch.device("cpu")
        # one lock serialises every reader and writer of the tenant graph --
        # the caller, the background consolidation worker and the store's
        # search over the bound graph (TenantGraph.lock is this lock)
        self._graph_lock = threading.RLock()
        self.graph = self._new_graph()

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
        # "reference": one mean super-node per shard once it passes
        # super_node_threshold (memory_system.py:893-933); "kmeans": a
        # two-level k-means hierarchy over the whole tenant, re-clustered every
        # hierarchy_params["every"] conversations (TenantGraph.cluster_pass)
        if hierarchy_mode not in ("reference", "kmeans"):
            raise ValueError("hierarchy_mode must be 'reference' or 'kmeans'")
        self.hierarchy_mode = hierarchy_mode
        self.hierarchy_params = {"fine": 4096, "top": 64, "every": 50, "iters": 2, **(hierarchy_params or {})}
        # failure policy: strict -> typed errors propagate;
        # otherwise failures are counted in metrics and work is retried
        self.strict_errors = strict_errors
        self.max_consolidation_retries = max_consolidation_retries
        self._persist_pending = False
        # write-behind persistence (opt-in): a save snapshots the changed
        # rows on the caller's thread and one writer thread commits the
        # snapshots in order, so the store I/O overlaps the next device work
        self.persist_async = bool(persist_async)
        self._writer = ThreadPoolExecutor(max_workers=1) if self.persist_async else None
        self._writes: List = []
        self._unwritten: List = []  # snapshots whose commit failed, retried first
        self._wb_lock = threading.Lock()

        self.query_cache = QueryCache(max_size=1000) if enable_caching else None
        self.consolidation_queue: List[Dict] = []
        # one worker: consolidations of a tenant are applied in order
        self.background_executor = ThreadPoolExecutor(max_workers=1) if enable_async else None
        self._pending = []
        self._queue_lock = threading.Lock()

        self.conversation_active = False
        self.short_term_memory: List[Dict] = []
        self.conversation_history: List[Dict] = []
        self.node_counter = 0
        self.conversation_count = 0
        self.metrics = {"embedding_calls": 0, "llm_calls": 0, "retrieval_times": [],
                        "consolidation_times": [], "consolidation_failures": 0, "dropped_batches": 0,
                        "persist_failures": 0, "rejected_embeddings": 0, "search_queries": 0,
                        "search_batches": 0, "search_ms": 0.0}
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
        kw.setdefault("hierarchy_mode", cfg.hierarchy_mode)
        kw.setdefault("hierarchy_params", {"fine": cfg.hierarchy_fine, "top": cfg.hierarchy_top,
                                           "every": cfg.hierarchy_every})
        kw.setdefault("strict_errors", cfg.strict_errors)
        return cls(**cfg.reference_kwargs(), embedding_provider=emb, device=cfg.device, metric=cfg.metric,
                   merge_mode=cfg.merge_mode, verbose=cfg.verbose, **kw)

    # ------------------------------------------------------------ graph + views
    def _new_graph(self) -> TenantGraph:
        g = TenantGraph(device=self._device)
        g.lock = self._graph_lock
        attach = getattr(self.store, "attach", None)
        if attach is not None:
            attach(self.user_id, g)
        return g

    @property
    def shards(self) -> ShardsMap:
        return ShardsMap(self.graph)

    @shards.setter
    def shards(self, value: Dict[str, MemoryShard]) -> None:
        with self._graph_lock:
            self._replace_graph()
            for k, sh in value.items():
                self.shards[k] = sh

    @property
    def super_nodes(self) -> SuperNodesMap:
        return SuperNodesMap(self.graph)

    @super_nodes.setter
    def super_nodes(self, value: Dict[str, Node]) -> None:
        with self._graph_lock:
            sm = self.super_nodes
            for k in list(sm):
                del sm[k]
            for k, n in value.items():
                sm[k] = n

    @property
    def buffer(self) -> GraphBuffer:
        return GraphBuffer(self.graph)

    def _replace_graph(self) -> None:
        detach = getattr(self.store, "detach", None)
        if detach is not None:
            detach(self.user_id)
        self.graph = self._new_graph()

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
        return ShardView(self.graph, self.graph.shard_id(shard_key))

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

    def _batch_embed_any(self, texts: List[str]):
        """Batch embedding as a device tensor when the provider can produce
        one (on-device encoder: no host round trip), else the protocol's lists."""
        # a class-level method only (a MagicMock provider answers every getattr)
        if getattr(type(self.embedder), "batch_embed_tensor", None) is None or not texts:
            return self._batch_embed(texts)
        self.metrics["embedding_calls"] += 1
        fault_point("provider.embed")
        return self.embedder.batch_embed_tensor(texts)

    def _cosine_similarity(self, v1, v2) -> float:
        return cosine(v1, v2)

    def _call_llm(self, messages: List[Dict], response_format: Dict = None) -> str:
        self.metrics["llm_calls"] += 1
        fault_point("provider.llm")
        return self.llm.completion(messages, response_format)

    def _search_batch(self, embs, k: int) -> List[List[str]]:
        fn = getattr(self.vector_store, "search_nodes_batch", None)
        if fn is not None:
            return fn(embs, user_id=self.user_id, limit=k)
        return [self.vector_store.search_nodes(e, user_id=self.user_id, limit=k) for e in embs]

    def _store_delete(self, ids: List[str], graph_unstored: bool = False) -> None:
        """``graph_unstored``: the rows' stored bits are already cleared in
        the bound graph (segment ends), so the bound store skips that step."""
        if ids:
            if graph_unstored and self._store_binds_graph():
                self.vector_store.delete_nodes(ids, user_id=self.user_id, graph_unstored=True)
            else:
                self.vector_store.delete_nodes(ids, user_id=self.user_id)

    def _store_add_rows(self, rows: List[int], dicts: List[Dict]) -> None:
        """Re-add rows to the store (merge): the bound store only flags them;
        a third-party store gets the reference's add_nodes."""
        if self._store_binds_graph():
            self.graph.mark_stored(rows)
        else:
            self.vector_store.add_nodes(dicts, user_id=self.user_id)

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
        """Reference :242-260 on the device graph: one ``tg_boost_kernel``
        launch over the visible-arc CSR of the retrieved rows."""
        g = self.graph
        rows = g.node_rows_of(retrieved_ids, include_super=False)
        count = g.boost(rows)
        if count:
            self._say(f"   (Graph: Boosted {count} neighbor nodes via association)")

    def _super_best(self, query_emb) -> int:
        """Row of the super-node most similar to the query (float64 cosine,
        first on ties), or -1 when none beats SUPER_MATCH (reference :464-472)."""
        g = self.graph
        srows = g.node_rows_where(super_=True)
        if srows.size == 0 or g.dim is None:
            return -1
        q = torch.as_tensor(np.asarray(query_emb, dtype=np.float64)) if not torch.is_tensor(query_emb) \
            else query_emb.double()
        if q.numel() != g.dim:
            return -1
        with g.on_stream():
            rt = torch.as_tensor(srows, dtype=torch.long).to(g.device)
            X = g.emb32[rt].double()
            nx = g.sqn[rt].double().sqrt()
            qd = q.to(g.device).reshape(-1)
            nq = qd.norm()
            s = (X @ qd) / torch.where(nx * nq > 0, nx * nq, torch.ones_like(nx))
            s = torch.where((nx > 0) & (nq > 0), s, torch.zeros_like(s))
            j = int(torch.argmax(s))  # first maximum
            best = float(s[j])
        return int(srows[j]) if best > SUPER_MATCH else -1

    def _optimized_retrieval(self, query_emb, query_text: str) -> List[str]:
        if self.query_cache:
            cached = self.query_cache.get_results(query_text)
            if cached:
                return cached
        g = self.graph
        retrieved: List[str] = []
        if self.enable_hierarchy and self.hierarchy_mode == "kmeans":
            q = query_emb if torch.is_tensor(query_emb) else torch.as_tensor(np.asarray(query_emb, np.float64))
            if g.dim is not None and q.numel() == g.dim:
                retrieved = [g.ids[r] for r in g.hier_children(q, SUPER_MATCH, SUPER_CHILDREN)]
                if len(retrieved) >= RESULT_LIMIT:
                    if self.query_cache:
                        self.query_cache.set_results(query_text, retrieved[:RESULT_LIMIT])
                    return retrieved[:RESULT_LIMIT]
        elif self.enable_hierarchy and g.n_super:
            sr = self._super_best(query_emb)
            if sr >= 0:
                kids = [(cid, g.row_of.get(cid)) for cid in g.children.get(sr, [])[:SUPER_CHILDREN]]
                kids = [(cid, r) for cid, r in kids if r is not None]
                kind, sup = g.flags_of([r for _, r in kids])
                retrieved += [cid for (cid, _), k, sp in zip(kids, kind, sup) if k == NODE and not sp]
                if len(retrieved) >= RESULT_LIMIT:
                    if self.query_cache:
                        self.query_cache.set_results(query_text, retrieved[:RESULT_LIMIT])
                    return retrieved[:RESULT_LIMIT]
        limit = 10 if not retrieved else 5
        vec_ids = self.vector_store.search_nodes(query_emb, user_id=self.user_id, limit=limit)
        vrows = [g.row_of.get(rid, -1) for rid in vec_ids]
        vkind = dict(zip(vrows, g.flags_of([r for r in vrows if r >= 0])[0])) if vrows else {}
        seen_ids = set(retrieved)
        seen_content = set()
        final = []
        for rid in retrieved:
            seen_content.add(g.content[g.row_of[rid]])
            final.append(rid)
        for rid in vec_ids:
            if rid in seen_ids:
                continue
            r = g.row_of.get(rid)
            if r is not None and vkind.get(r) == NODE and g.content[r] not in seen_content:
                seen_content.add(g.content[r])
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
            g = self.graph
            rows = g.node_rows_of(retrieved_ids)
            texts = [f"- {g.content[r]}" for r in rows if r >= 0]
            g.touch(rows)  # update_access for each retrieved node (buffer_graph.py:79-85)
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
        g = self.graph
        out = []
        rows = g.node_rows_of(ids)
        live = [r for r in rows if r >= 0]
        sh = {}
        if live:  # the shard codes of these rows only (a turn must not mirror a 10M-row column)
            with g.on_stream():
                codes = g.shard[torch.as_tensor(live, dtype=torch.long).to(g.device)].cpu().tolist()
            sh = dict(zip(live, codes))
        for nid, r in zip(ids, rows):
            if r >= 0:
                c = g.content[r]
                snip = c[:60] + "..." if len(c) > 60 else c
                out.append(f"   • [{nid}] ({g.shard_names[sh[r]] if sh[r] >= 0 else 'default'}) {snip}")
        return out

    def chat(self, user_message: str) -> str:
        ids, ms = self._retrieve_for(user_message)
        self.metrics["retrieval_times"].append(ms)
        with self._graph_lock:
            node_lines = self._node_lines(ids)
            msgs = self._build_messages(ids)
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
        if not self.enable_sharding or not len(self.shards):
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
        """Other endpoints of every edge touching the node, any shard, in the
        reference's order (shards in order, edges in order; :1441-1458)."""
        g = self.graph
        r = g.row_of.get(node_id)
        if r is None:
            return []
        idx = g.edges_incident(r)
        with g.on_stream():
            sh = (g.e["meta"][idx] & 0xFFFFFF).long()
            o = torch.sort(sh, stable=True).indices
            idx = idx[o]
            s, d = g.e["src"][idx].tolist(), g.e["dst"][idx].tolist()
        out, seen = [], set()
        for a, b in zip(s, d):
            o_ = b if a == r else a
            if o_ not in seen:
                seen.add(o_)
                out.append(o_)
        kind = g.flags_of(out)[0]
        return [NodeView.of(g, x) for x, k in zip(out, kind) if k == NODE]

    def search_memories(self, query: str, limit: int = 5) -> List[Node]:
        with tracer.stage("embed_query", self._device):
            q = self._get_embedding(query)
        with self._graph_lock:
            with tracer.stage("search", self._device):
                ids = self.vector_store.search_nodes(q, user_id=self.user_id, limit=limit)
            return [n for n in (self.buffer.get_node(i) for i in ids) if n is not None]

    def search_memories_batch(self, queries: List[str], limit: int = 5) -> List[List[Node]]:
        """Batched ``search_memories`` (reference :1460-1472 per query): one
        embedding call (a device tensor when the encoder is on-device), one
        store search -- the fused MFMA candidate scan plus an fp32 re-rank
        over the tenant's HBM rows -- and one row -> Node mapping."""
        t0 = time.perf_counter()
        out = self._search_finish(self._search_submit(queries, limit))
        self._count_search(len(out), (time.perf_counter() - t0) * 1e3)
        return out

    def _count_search(self, n: int, ms: float) -> None:
        m = self.metrics
        m["search_queries"] = m.get("search_queries", 0) + n
        m["search_batches"] = m.get("search_batches", 0) + 1
        m["search_ms"] = m.get("search_ms", 0.0) + ms

    def search_memories_stream(self, batches: Iterable[List[str]], limit: int = 5):
        """Pipelined ``search_memories_batch`` for serving loops: batches i+1 ..
        i+STREAM_DEPTH are tokenised and their embed + scan enqueued on the
        device BEFORE the host waits for batch i and maps its rows to Nodes,
        so host work (tokenizer, result mapping) hides under device work.
        Yields one result list per input batch, in order; results equal
        ``search_memories_batch``."""
        pending = collections.deque()
        for qs in batches:
            pending.append(self._search_submit(qs, limit))
            if len(pending) > STREAM_DEPTH:
                yield self._search_finish(pending.popleft())
        while pending:
            yield self._search_finish(pending.popleft())

    def _search_submit(self, queries, limit: int):
        """Enqueue embed + store search; returns a handle for _search_finish.
        With the graph-bound store the result rows stay on the device and come
        back with one async copy into pinned memory (no host sync here)."""
        queries = list(queries)
        with tracer.stage("embed_query", self._device):
            embs = self._batch_embed_any(queries)
        with self._graph_lock:
            g = self.graph
            if (torch.is_tensor(embs) and self._store_binds_graph() and g.dim is not None
                    and embs.shape[-1] == g.dim and len(queries)):
                overlap = SEARCH_OVERLAP and embs.is_cuda and g.on_gpu
                if overlap:
                    # the search and its result copy run on the graph's stream
                    # and the caller's stream does NOT wait for them: the next
                    # batch's embed overlaps this batch's scan
                    cur = torch.cuda.current_stream(g.device)
                    g.stream.wait_stream(cur)
                    embs.record_stream(g.stream)
                    ctx = torch.cuda.stream(g.stream)
                else:
                    ctx = contextlib.nullcontext()
                with ctx:
                    with tracer.stage("search", self._device):
                        # rows the graph does not hold as nodes are skipped (reference
                        # :1467-1472): marked on the device (by the re-rank kernel), so
                        # mapping needs no mirror
                        _, rows = g.store_search(embs, int(limit), getattr(self.store, "metric", "l2"),
                                                 node_rows=True)
                    if rows.is_cuda:
                        # the rows stay on the device until _search_finish copies them to
                        # pageable host memory on a stream that waits for THIS search only
                        # (host reads of a pinned buffer the device just wrote ran at
                        # ~16 MB/s in the serving loop: 5-7 ms per 1024 x 10 batch)
                        ev = torch.cuda.Event(blocking=BLOCKING_EVENTS)
                        ev.record()
                        return ("rows_dev", g, rows, ev)
                    return ("rows", g, rows, None)
        with tracer.stage("search", self._device):
            return ("ids", None, self._search_batch(embs, limit), None)

    def _search_finish(self, h) -> List[List[Node]]:
        kind_, g0, data, ev = h
        if kind_ == "rows_dev":
            st = getattr(self, "_result_stream", None)
            if st is None:
                st = self._result_stream = torch.cuda.Stream(data.device)
            with torch.cuda.stream(st):
                st.wait_event(ev)
                data = data.to("cpu")  # pageable; waits for this search's event only
            kind_, ev = "rows", None
        if ev is not None:
            ev.synchronize()
        with self._graph_lock:
            g = self.graph
            if kind_ == "rows" and g is g0:  # non-node rows were set to -1 on the device
                # lazy per-row views: no Python object per result row until read
                return ResultBatch(g, data.numpy() if not data.is_cuda else data.cpu().numpy())
            if kind_ == "rows":  # the tenant was switched while the search ran
                data = [[g0.ids[r] for r in row if r >= 0] for row in data.tolist()]
            out = []
            for ids in data:
                rows = [r for r in (g.row_of.get(i, -1) for i in ids) if r >= 0]
                kind = g.flags_of(rows)[0]
                out.append([NodeView.of(g, r) for r, k in zip(rows, kind) if k == NODE])
            return out

    # ------------------------------------------------------------ stats / display
    def get_stats(self) -> Dict:
        with self._graph_lock:
            return self._stats()

    def _stats(self) -> Dict:
        g = self.graph
        nodes, edges = g.num_nodes(), g.num_edges
        rt = self.metrics["retrieval_times"]
        ct = self.metrics["consolidation_times"]
        avg_r = float(np.mean(rt)) if rt else 0.0
        p95_r = float(np.percentile(rt, 95)) if rt else 0.0
        avg_c = float(np.mean(ct)) if ct else 0.0
        hit = self.query_cache.get_hit_rate() if self.query_cache else 0.0
        return {
            "buffer_nodes": nodes,
            "buffer_edges": edges,
            "num_shards": len(g.live_shards()),
            "num_super_nodes": g.n_super,
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
            # engine metrics: the device, the tenant graph's HBM
            # footprint, search throughput of search_memories[_batch]
            "engine": self._engine_brief(),
        }

    def _engine_brief(self) -> Dict:
        g, m = self.graph, self.metrics
        sq, sms = m.get("search_queries", 0), m.get("search_ms", 0.0)
        return {"device": str(self._device), "graph_rows": g.n, "hbm_graph_bytes": self._graph_bytes(),
                "search_queries": sq, "search_qps": round(sq / (sms / 1e3), 1) if sms > 0 else 0.0,
                "avg_search_batch_ms": round(sms / m["search_batches"], 3) if m.get("search_batches") else 0.0}

    def _graph_bytes(self) -> int:
        g = self.graph
        return int(sum(t.numel() * t.element_size() for t in
                       [g.emb32, g.emb16, g.emb8, g.rs8, g.sqn] + [getattr(g, c) for c, _, _ in TenantGraph.NODE_COLS]
                       + list(g.e.values()) if t is not None))

    def engine_stats(self) -> Dict:
        """Engine-level metrics beyond the reference's ``get_stats`` (SURVEY.md
        §5 metrics row): device, HBM bytes held by the tenant graph, rows,
        edges, per-stage timings from the tracer when enabled."""
        g = self.graph
        return {"device": str(self._device), "rows": g.n, "capacity": g.cap, "nodes": g.num_nodes(),
                "edges": g.num_edges, "graph_bytes": self._graph_bytes(), "dim": g.dim,
                "decay_clock": g.decay_log, "stages": tracer.summary(), **self._engine_brief()}

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
        if self.graph.num_nodes() == 0:
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
        with self._graph_lock:
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
            self._replace_graph()
            g = self.graph
            for k, d in state.get("shards", {}).items():
                g.shard_id(k)
                nodes = [Node.from_dict(nd) for nd in d.get("nodes", [])]
                import_nodes(g, nodes, [k] * len(nodes), supers=[False] * len(nodes))
                edges = [Edge.from_dict(ed) for ed in d.get("edges", [])]
                import_edges(g, edges, [k] * len(edges))
            sups = [Node.from_dict(n) for n in state.get("super_nodes", [])]
            import_nodes(g, sups, [n.shard_key or "default" for n in sups], supers=[True] * len(sups))
            pd_ = state.get("profile", {})
            self.profile.data = pd_.get("data", self.profile.data)
            self.profile.last_updated = pd_.get("last_updated", time.time())
            self.node_counter = state.get("node_counter", 0)
            self.conversation_count = state.get("conversation_count", 0)
            for k, v in state.get("settings", {}).items():
                if hasattr(self, k):
                    setattr(self, k, v)
        return f"✓ State loaded from {filename}"

    # ------------------------------------------------------------ store sync
    def _profile_blob(self) -> Dict:
        d = self.profile.to_dict()
        d["_engine"] = {"decay_clock": self.graph.decay_log, "node_counter": self.node_counter,
                        "max_node_id": getattr(self, "_max_node_id", 0)}
        return d

    def _save_to_persistence(self):
        """Persist the tenant (reference memory_system.py:1275-1302).

        With the default store (graph-bound ``HBMStore``) this is ONE
        incremental commit per table: rows and edges changed since the last
        commit are upserted, removed ones deleted -- O(changes), not O(graph).
        A third-party ``Store`` gets the reference's delete-all + add-all.
        A failed commit leaves the graph authoritative and the change set
        pending (it is retried by the next save); ``strict_errors`` raises
        :class:`StoreError` instead."""
        if self._writer is not None and self._store_binds_graph():
            self._save_write_behind()
            return
        with self._graph_lock:
            try:
                with tracer.stage("persist", "cpu"):
                    if self._store_binds_graph():
                        self._commit_incremental()
                    else:
                        self._rewrite_all()
                    with tracer.stage("persist_profile", "cpu"):
                        self.store.save_profile(self._profile_blob(), user_id=self.user_id)
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

    def _snapshot_incremental(self):
        """Take the change set (dirty rows / edges, deletions) and export it
        as store columns. Returns (tracking, commit_tenant arguments)."""
        g = self.graph
        rows = g.take_dirty_rows()
        eidx = g.take_dirty_edges()
        del_ids, del_edges = g.take_deleted()
        try:
            if rows.size:  # kind of the dirty rows only (no mirror of the whole column)
                with g.on_stream():
                    k = g.kind[torch.as_tensor(rows).to(g.device)].cpu().numpy()
                rows = rows[k == NODE]
            with tracer.stage("persist_export", "cpu"):
                node_cols = export_node_columns(g, rows)
                edge_cols = export_edge_columns(g, eidx)
            # largest node_<n> id ever committed (O(changed rows)): a reload
            # restores node_counter from it without scanning every id
            self._max_node_id = max(getattr(self, "_max_node_id", 0), _max_node_num(node_cols.get("id", [])))
        except Exception:
            g.restore_tracking(rows, eidx, del_ids, del_edges)
            raise
        return (rows, eidx, del_ids, del_edges), (self.user_id, node_cols, del_ids, edge_cols,
                                                   [f"{s}_{t}" for s, t in del_edges])

    def _commit_incremental(self) -> None:
        tracking, args = self._snapshot_incremental()
        if getattr(self, "_commit_retry", False):
            # the previous commit failed part way (e.g. nodes written, edges
            # not): rows it reported fresh may be in the table now, so every
            # row goes through the keyed upsert -- a retry never duplicates
            args[1].pop("fresh", None)
        try:
            with tracer.stage("persist_write", "cpu"):
                self.store.commit_tenant(*args)
        except Exception:
            self.graph.restore_tracking(*tracking)
            self._commit_retry = True
            raise
        self._commit_retry = False
        self._mark_committed(tracking[0], tracking[2])

    def _mark_committed(self, rows, del_ids) -> None:
        g = self.graph
        g.mark_stored(rows)
        # ids deleted from the table leave the searchable set too
        gone = [i for i in del_ids if g.node_row(i) < 0]
        if gone:
            g.unstore(gone)

    # ------------------------------------------------------------ write-behind
    def _save_write_behind(self) -> None:
        """``persist_async``: snapshot on this thread (under the graph lock),
        commit on the writer thread. The rows are searchable from now on, as
        after a synchronous save; a commit that fails keeps its snapshot and
        is retried before the next one (upserts / deletes by id, in order)."""
        with self._graph_lock:
            with tracer.stage("persist", "cpu"):
                try:
                    tracking, args = self._snapshot_incremental()
                except Exception as e:
                    self._persist_failed(e)
                    return
                self._mark_committed(tracking[0], tracking[2])
                prof = self._profile_blob()
                self._writes = [f for f in self._writes if not f.done()]
                self._writes.append(self._writer.submit(self._write_job, args, prof))
            if self.query_cache:
                self.query_cache.invalidate_results()

    def _write_job(self, args, prof) -> None:
        with self._wb_lock:
            queue, self._unwritten = self._unwritten + [(args, prof)], []
            for i, (a, p) in enumerate(queue):
                try:
                    with tracer.stage("persist_write", "cpu"):
                        self.store.commit_tenant(*a)
                        self.store.save_profile(p, user_id=a[0])
                except Exception as e:
                    self._unwritten = queue[i:]
                    for a_, _ in self._unwritten:  # retried by key: the failed write may have landed in part
                        a_[1].pop("fresh", None)
                    self.metrics["persist_failures"] = self.metrics.get("persist_failures", 0) + 1
                    log.warning("write-behind commit failed for %s: %s", a[0], e)
                    return
            try:
                self._last_nodes_version = self.store.get_latest_version()
            except Exception:
                pass

    def flush_persistence(self) -> None:
        """Wait for the write-behind commits; retry any failed snapshot once
        more (``strict_errors``: raise :class:`StoreError` if it still fails)."""
        if self._writer is None:
            return
        pend, self._writes = self._writes, []
        for f in pend:
            f.result()
        if self._unwritten:
            with self._wb_lock:
                args, prof = self._unwritten.pop()
            self._writer.submit(self._write_job, args, prof).result()
            if self._unwritten and self.strict_errors:
                raise StoreError(f"write-behind commit failed for {self.user_id}")

    def _persist_failed(self, e) -> None:
        self.metrics["persist_failures"] = self.metrics.get("persist_failures", 0) + 1
        self._persist_pending = True
        log.warning("persistence failed for %s: %s", self.user_id, e)
        if self.strict_errors:
            raise StoreError(str(e)) from e

    def _rewrite_all(self) -> None:
        self._max_node_id = max(getattr(self, "_max_node_id", 0), _max_node_num(self.graph.ids))
        nodes = [n.to_dict() for n in self.buffer.nodes.values()]
        edges = [e.to_dict() for sh in self.shards.values() for e in sh.edges.values()]
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
        self.graph.clear_tracking()

    def _load_from_persistence(self):
        """Rebuild the tenant graph from the store (reference :1304-1410):
        columns go straight into the graph (vectors: one host->device copy),
        no per-row ``Node`` objects; decay since each row was written is
        replayed from the persisted decay clock."""
        if getattr(self, "_writer", None) is not None:
            self.flush_persistence()  # our own queued commits land before we read
        self._say(f"🔄 Loading state for user: {self.user_id}...")
        # a 10M-row tenant creates tens of millions of objects: the cyclic GC
        # would re-scan the heap many times over (none of them form cycles)
        gc_was = gc.isenabled()
        gc.disable()
        try:
            self._load_columns()
        finally:
            if gc_was:
                gc.enable()

    def _load_columns(self):
        with self._graph_lock:
            loader = getattr(self.store, "load_tenant", None)
            if loader is not None:
                ncols, ecols = loader(self.user_id)
            else:
                ncols, ecols = _rows_to_columns(self.store.get_nodes(user_id=self.user_id)), None
            n_rows = len(ncols.get("id", [])) if ncols else 0
            if ecols is None and n_rows:
                ecols = _edge_rows_to_columns(self.store.get_edges(user_id=self.user_id))
            prof = self.store.load_profile(user_id=self.user_id) if n_rows else None
            self._replace_graph()
            self._max_node_id = 0
            eng = (prof or {}).get("_engine", {}) if isinstance(prof, dict) else {}
            clock = float(eng.get("decay_clock", 0.0))
            n_edges = 0
            if n_rows:
                bulk_load(self.graph, ncols, ecols, clock)
                n_edges = self.graph.num_edges
            self.profile = Profile.from_dict(prof) if prof else Profile()
            try:
                self._last_nodes_version = self.store.get_latest_version()
            except Exception:
                self._last_nodes_version = 0
            if n_rows:
                if "max_node_id" in eng:  # written by this engine: no per-id scan
                    mx = max(int(eng.get("node_counter", 0)), int(eng["max_node_id"]))
                else:  # a store written elsewhere: the largest node_<n> id
                    mx = max(int(eng.get("node_counter", 0)), _max_node_num(ncols["id"]))
                self._max_node_id = mx
                self.node_counter = mx
            if self.query_cache:
                self.query_cache.invalidate_results()
            del ncols, ecols
        if n_rows:
            self._say(f"✓ Restored state ({self.graph.num_nodes()} nodes, {n_edges} edges)")
        else:
            self._say("ℹ No saved state found.")

    def check_for_updates(self) -> bool:
        self.flush_persistence()
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
        self.flush_persistence()
        with self._graph_lock:
            detach = getattr(self.store, "detach", None)
            if detach is not None:
                detach(self.user_id)
            self.user_id = new_user_id
            self._load_from_persistence()
        self._say(f"👤 Switched context to user: {new_user_id}")

    # ------------------------------------------------------------ export
    def graph_json(self) -> Dict:
        """The dashboard's ``/api/graph`` payload (reference dashboard/api.py:
        71-112: shard nodes and each shard's edges in shard order, then the
        super-nodes under shard "global"), built from the graph columns in one
        pass under the graph lock (a background consolidation may be writing)."""
        with self._graph_lock:
            g = self.graph
            rows = g.ordered_node_rows()
            sup, sh = g.mirror("sup"), g.mirror("shard")
            sal, acc = g.mirror("sal"), g.mirror("acc")
            nodes, supers = [], []
            names, ids, content, types = g.shard_names, g.ids, g.content, g.types
            for r in rows.tolist():
                if sup[r]:
                    supers.append({"id": ids[r], "content": content[r], "type": "super_node",
                                   "salience": float(sal[r]), "shard": "global", "is_super_node": True})
                else:
                    nodes.append({"id": ids[r], "content": content[r], "type": types[r], "salience": float(sal[r]),
                                  "shard": names[sh[r]], "access_count": int(acc[r]), "is_super_node": False})
            links = []
            if g.num_edges:
                with g.on_stream():
                    meta = g.e["meta"].cpu().numpy()
                    s, d, w = g.e["src"].cpu().numpy(), g.e["dst"].cpu().numpy(), g.e["w"].cpu().numpy()
                es = meta & 0xFFFFFF
                live = np.asarray(g.shard_live, dtype=bool)[es]
                order = np.argsort(es, kind="stable")
                order = order[live[order]]
                et = g.etype_names
                links = [{"source": ids[s[i]], "target": ids[d[i]], "weight": float(w[i]),
                          "type": et[(meta[i] >> 24) & TYPE_MASK]} for i in order.tolist()]
            return {"nodes": nodes + supers, "links": links}

    def export_observations(self, format: str = "markdown") -> str:
        with self._graph_lock:
            return self._export(format)

    def _top_observations(self, k: int = 50) -> List[NodeView]:
        """Top ``k`` shard nodes by (salience, last_accessed) descending
        (reference :1505-1512), selected on the device."""
        g = self.graph
        rows = g.ordered_node_rows()
        rows = rows[g.mirror("sup")[rows] == 0]
        if rows.size == 0:
            return []
        sal, last = g.mirror("sal")[rows].astype(np.float64), g.mirror("last")[rows]
        o = np.lexsort((-last, -sal), axis=0) if rows.size else rows
        return [NodeView.of(g, int(r)) for r in rows[o][:k]]

    def _export(self, format: str) -> str:
        nodes = self._top_observations(50)
        if format == "json":
            return json.dumps([n.to_dict() for n in nodes], indent=2)
        lines = [f"# Memory Observations for {self.user_id}", ""]
        for n in nodes:
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

    # ------------------------------------------------------------ live migration (C3)
    def export_state(self) -> Tuple[Dict, torch.Tensor]:
        """The tenant's graph as (JSON-able metadata, fp32 vector rows on the
        device) -- what :meth:`import_state` on another rank rebuilds it from
        without touching the store (``DistributedMemoryService.migrate``)."""
        with self._graph_lock:
            g = self.graph
            rows = g.node_rows_where()
            nc = export_node_columns(g, rows, device_vectors=True)
            vec = nc.pop("vector", None)
            nc.pop("fresh", None)
            if vec is None:
                vec = torch.zeros((0, g.dim or 0), device=g.device)
            nc.pop("count", None)
            rl = rows.tolist()
            nc["_has"] = g.has_emb[torch.as_tensor(rows, dtype=torch.long).to(g.device)].bool().cpu().tolist() \
                if rows.size else []
            nc["_odd"] = {str(j): g.odd_emb[r] for j, r in enumerate(rl) if r in g.odd_emb}
            ec = export_edge_columns(g, np.arange(g.num_edges))
            ec.pop("count", None)
            meta = {"nodes": _jsonable_cols(nc), "edges": _jsonable_cols(ec), "profile": self._profile_blob(),
                    "conversation_count": self.conversation_count}
            return meta, vec.reshape(len(rl), -1)

    def import_state(self, meta: Dict, vectors: torch.Tensor) -> None:
        """Replace this tenant's graph by an :meth:`export_state` image."""
        with self._graph_lock:
            self._replace_graph()
            nc = dict(meta["nodes"])
            if nc.get("id"):
                for k in ("timestamp", "access_count", "last_accessed", "salience", "is_super_node", "decay_clock"):
                    if k in nc:
                        nc[k] = np.asarray(nc[k])
                nc["_odd"] = {int(j): v for j, v in nc.get("_odd", {}).items()}
                nc["vector"] = vectors
                ec = dict(meta["edges"]) if meta["edges"].get("id") else None
                if ec is not None:
                    for k in ("weight", "co_occurrence", "last_updated", "decay_clock"):
                        if k in ec:
                            ec[k] = np.asarray(ec[k])
                prof = meta.get("profile") or {}
                eng = prof.get("_engine", {})
                bulk_load(self.graph, nc, ec, float(eng.get("decay_clock", 0.0)))
                self.node_counter = max(int(eng.get("node_counter", 0)), int(eng.get("max_node_id", 0)))
                self._max_node_id = int(eng.get("max_node_id", 0))
                self.profile = Profile.from_dict(prof)
            self.conversation_count = int(meta.get("conversation_count", 0))
            if self.query_cache:
                self.query_cache.invalidate_results()

    def close(self):
        if self.background_executor:
            self.background_executor.shutdown(wait=True)
        g = getattr(self, "graph", None)
        if g is not None and hasattr(g, "cluster_join"):
            g.cluster_join()  # a background k-means pass ends before the store closes
        if self._writer is not None:
            self.flush_persistence()
            self._writer.shutdown(wait=True)
        if getattr(self, "store", None) is None:
            return
        detach = getattr(type(self.store), "detach", None)
        if getattr(self, "_owns_store", True) or detach is None:
            self.store.close()  # reference :1545-1550 (a third-party store is closed as there)
        elif self.store.bound_graph(self.user_id) is self.graph:
            self.store.detach(self.user_id)


# ---------------------------------------------------------------- columnar I/O
def export_node_columns(g: TenantGraph, rows: np.ndarray, device_vectors: bool = False) -> Dict:
    """Store columns (SURVEY.md App. D + ``decay_clock``) of graph rows.
    ``device_vectors``: the vector column stays a device tensor (migration
    over the interconnect) instead of a host array. ``fresh``: rows never
    committed (the store cannot hold their ids: no delete needed).

    Every per-row column is built by C-level loops (``map`` over the lists,
    object-array indexing) and the sparse ones (children, parents, odd
    vectors) are patched from their few entries: a 10M-row commit used to
    spend ~20 s in per-row ``json.dumps`` / list comprehensions."""
    rows = np.asarray(rows, dtype=np.int64)
    n = rows.size
    D = g.dim or 0
    if n == 0:
        return {"id": [], "count": 0}
    with g.on_stream():
        rt = torch.as_tensor(rows).to(g.device)
        if device_vectors:
            vec = g.emb32[rt].clone() if g.dim is not None else torch.zeros((n, 0), device=g.device)
        else:
            vec = g.emb32[rt].cpu().numpy() if g.dim is not None else np.zeros((n, 0), dtype=np.float32)
        cols = {k: getattr(g, c)[rt].cpu().numpy() for k, c in
                (("timestamp", "ts"), ("access_count", "acc"), ("last_accessed", "last"), ("salience", "sal"),
                 ("is_super_node", "sup"), ("parent", "parent"), ("shard", "shard"), ("stored", "stored"))}
    rl = rows.tolist()
    # position of each exported row (for the sparse patches below)
    sparse = [r for r in g.odd_emb] + list(g.children.keys())
    pos = {}
    if sparse:
        rmap = np.full(max(g.n, int(rows.max()) + 1), -1, dtype=np.int64)
        rmap[rows] = np.arange(n)
        pos = {r: int(rmap[r]) for r in set(sparse) if r < rmap.size and rmap[r] >= 0}
    if D:
        for r in g.odd_emb:
            j = pos.get(r)
            if j is not None:
                vec[j] = 0.0
    child = ["[]"] * n
    for r, ch in g.children.items():
        j = pos.get(r)
        if j is not None:
            child[j] = json.dumps(ch)
    par = cols.pop("parent")
    parent_id = [""] * n
    pj = np.nonzero(par >= 0)[0]
    if pj.size:
        ids = g.ids
        for j, pr in zip(pj.tolist(), par[pj].tolist()):
            parent_id[j] = ids[pr]
    sh = cols.pop("shard")
    names = np.asarray(list(g.shard_names) + ["default"], dtype=object)
    shard_key = names[np.where(sh >= 0, sh, len(g.shard_names))].tolist()
    return {
        "count": n,
        "id": list(map(g.ids.__getitem__, rl)),
        "content": list(map(g.content.__getitem__, rl)),
        "vector": vec if torch.is_tensor(vec) else np.ascontiguousarray(vec, dtype=np.float32),
        "type": list(map(g.types.__getitem__, rl)),
        "timestamp": cols["timestamp"].astype(np.float64),
        "access_count": cols["access_count"].astype(np.int32),
        "last_accessed": cols["last_accessed"].astype(np.float64),
        "salience": cols["salience"].astype(np.float32),
        "is_super_node": cols["is_super_node"].astype(np.uint8),
        "child_ids": child,
        "parent_id": parent_id,
        "shard_key": shard_key,
        "metadata": ["{}"] * n,
        "decay_clock": np.full(n, g.decay_log, dtype=np.float64),
        "fresh": cols["stored"] == 0,
    }


def export_edge_columns(g: TenantGraph, idx: np.ndarray) -> Dict:
    idx = np.asarray(idx, dtype=np.int64)
    n = idx.size
    if n == 0:
        return {"count": 0, "id": []}
    with g.on_stream():
        it = torch.as_tensor(idx).to(g.device)
        s, d = g.e["src"][it].cpu().numpy(), g.e["dst"][it].cpu().numpy()
        w, co = g.e["w"][it].cpu().numpy(), g.e["co"][it].cpu().numpy()
        lu, meta = g.e["lu"][it].cpu().numpy(), g.e["meta"][it].cpu().numpy()
    ids = g.ids
    src = [ids[a] for a in s.tolist()]
    dst = [ids[b] for b in d.tolist()]
    return {
        "count": n,
        "id": [f"{a}_{b}" for a, b in zip(src, dst)],
        "source_id": src, "target_id": dst,
        "weight": w.astype(np.float32),
        "edge_type": [g.etype_names[(m >> 24) & TYPE_MASK] for m in meta.tolist()],
        "co_occurrence": co.astype(np.int32),
        "last_updated": lu.astype(np.float64),
        "metadata": ["{}"] * n,
        "decay_clock": np.full(n, g.decay_log, dtype=np.float64),
    }


def _rows_to_columns(rows: List[Dict]) -> Dict:
    """Reference-shaped node dicts (``Store.get_nodes``) -> columns."""
    if not rows:
        return {"id": []}
    vec = [r.get("vector", r.get("embedding")) for r in rows]
    dims = {len(v) for v in vec if v is not None and len(v)}
    D = dims.pop() if len(dims) == 1 else 0
    V = np.zeros((len(rows), D), dtype=np.float32)
    odd = {}
    for i, v in enumerate(vec):
        if v is not None and len(v):
            if len(v) == D:
                V[i] = np.asarray(v, dtype=np.float32)
            else:
                odd[i] = list(v)

    def js(v):
        if isinstance(v, str):
            return v
        return json.dumps(v if v is not None else [])
    return {
        "id": [r["id"] for r in rows], "content": [r.get("content", "") for r in rows], "vector": V,
        "_odd": odd, "_has": [v is not None and len(v) > 0 for v in vec],
        "type": [r.get("type", "semantic") for r in rows],
        "timestamp": np.asarray([float(r.get("timestamp", 0.0)) for r in rows]),
        "access_count": np.asarray([int(r.get("access_count", 0)) for r in rows], dtype=np.int32),
        "last_accessed": np.asarray([float(r.get("last_accessed", 0.0)) for r in rows]),
        "salience": np.asarray([float(r.get("salience", 0.5)) for r in rows], dtype=np.float32),
        "is_super_node": np.asarray([bool(r.get("is_super_node", False)) for r in rows], dtype=np.uint8),
        "child_ids": [js(r.get("child_ids", [])) for r in rows],
        "parent_id": [r.get("parent_id") or "" for r in rows],
        "shard_key": [r.get("shard_key", "default") for r in rows],
    }


def _edge_rows_to_columns(rows: List[Dict]) -> Dict:
    if not rows:
        return {"id": []}
    return {
        "id": [r.get("id", "") for r in rows],
        "source_id": [r.get("source_id", r.get("source")) for r in rows],
        "target_id": [r.get("target_id", r.get("target")) for r in rows],
        "weight": np.asarray([float(r.get("weight", 1.0)) for r in rows], dtype=np.float32),
        "edge_type": [r.get("edge_type") or r.get("type") or "relates_to" for r in rows],
        "co_occurrence": np.asarray([int(r.get("co_occurrence", 1)) for r in rows], dtype=np.int32),
        "last_updated": np.asarray([float(r.get("last_updated", 0.0)) for r in rows]),
    }


def bulk_load(g: TenantGraph, nc: Dict, ec: Optional[Dict], clock: float) -> None:
    """Columns -> an empty tenant graph (reference _load_from_persistence
    :1304-1410 semantics): super rows go to ``super_nodes``; an edge goes to
    its source node's shard and is dropped when its source is not a node;
    repeated (source, target) rows strengthen like ``MemoryShard.add_edge``.
    Rows written at an older decay clock get the decay applied since."""
    import pandas as pd

    ids = list(nc["id"])
    N = len(ids)
    if N == 0:
        return
    is_sup = np.asarray(nc["is_super_node"]).astype(bool)
    shard_keys = list(nc["shard_key"])
    # reference shard creation order: first non-super occurrence (factorize
    # keeps first-appearance order), then any key only super rows use
    keys = pd.Series(shard_keys, dtype=object)
    for k in pd.unique(keys[~is_sup]):
        if k not in g.shard_code:
            g.shard_id(k)
    kcode, kuniq = pd.factorize(keys, sort=False)
    ucode = np.asarray([g.shard_code[k] if k in g.shard_code else g.shard_id(k, live=False) for k in kuniq],
                       dtype=np.int32)
    codes = ucode[kcode]
    dc = np.asarray(nc.get("decay_clock", np.zeros(N)), dtype=np.float64)
    fac = np.exp(np.minimum(0.0, clock - dc))
    sal = np.asarray(nc["salience"], dtype=np.float64)
    decayed = fac < 1.0
    sal = np.where(decayed & ~is_sup, np.where(sal > SALIENCE_FLOOR, SALIENCE_FLOOR + (sal - SALIENCE_FLOOR) * fac,
                                               SALIENCE_FLOOR), sal)
    V = nc["vector"]
    has = nc.get("_has")
    emb = None
    if isinstance(V, list):  # pieces of the mapped store fragments, in row order
        D = next((int(x.shape[1]) for x in V if x.shape[1]), 0)
        if D:
            if g.on_gpu:
                emb = _h2d_pieces(V, N, D, g.device)
            else:
                emb = torch.from_numpy(np.concatenate([np.asarray(x, dtype=np.float32) for x in V])
                                       if len(V) > 1 else np.array(V[0], dtype=np.float32))
    elif torch.is_tensor(V):  # already a tensor (a migrated tenant's device rows)
        emb = V.to(g.device, torch.float32) if V.shape[1] else None
    elif V.shape[1]:
        emb = _h2d(np.ascontiguousarray(V, dtype=np.float32), g.device) if g.on_gpu else torch.from_numpy(
            np.ascontiguousarray(V, dtype=np.float32))
    children = {}
    for j in np.nonzero(is_sup)[0].tolist():
        try:
            children[j] = json.loads(nc["child_ids"][j]) if isinstance(nc["child_ids"][j], str) \
                else list(nc["child_ids"][j])
        except json.JSONDecodeError:
            children[j] = []
    parents = list(nc["parent_id"])
    rows = g.add_nodes(ids, list(nc["content"]), emb, shard=codes, types=list(nc["type"]), sal=sal.astype(np.float32),
                       acc=np.asarray(nc["access_count"]), last=np.asarray(nc["last_accessed"]),
                       ts=np.asarray(nc["timestamp"]), sup=is_sup.astype(np.uint8),
                       parents=parents if any(parents) else None, children=children, stored=True)
    if has is not None and not all(has):
        miss = torch.as_tensor([not h for h in has]).to(g.device)
        with g.on_stream():
            g.has_emb[rows[miss]] = 0
        g._bump(store=True)
    for j, v in nc.get("_odd", {}).items():
        g.odd_emb[int(rows[j])] = v
    if ec is not None and len(ec.get("id", [])):
        idx = pd.Index(g.ids.tolist() if hasattr(g.ids, "tolist") else g.ids)
        src = idx.get_indexer(pd.Index(list(ec["source_id"])))
        node_src = src >= 0
        if node_src.any():
            kind = g.mirror("kind")
            node_src &= kind[np.maximum(src, 0)] == NODE
        keep = np.nonzero(node_src)[0]
        if keep.size:
            tgt_ids = [ec["target_id"][i] for i in keep.tolist()]
            dst = np.asarray([g._ensure_row(t) for t in tgt_ids], dtype=np.int64)
            s = src[keep].astype(np.int64)
            sh = g.mirror("shard")[s]
            w = np.asarray(ec["weight"], dtype=np.float64)[keep]
            edc = np.asarray(ec.get("decay_clock", np.zeros(len(ec["id"]))), dtype=np.float64)[keep]
            w = w * np.exp(np.minimum(0.0, clock - edc))
            et = [g.etype(ec["edge_type"][i] or "relates_to") for i in keep.tolist()]
            g.upsert_edges(torch.as_tensor(s), torch.as_tensor(dst), torch.as_tensor(w, dtype=torch.float32),
                           torch.as_tensor(sh, dtype=torch.int32), torch.as_tensor(et, dtype=torch.int32),
                           co=torch.as_tensor(np.asarray(ec["co_occurrence"])[keep], dtype=torch.int32),
                           lu=torch.as_tensor(np.asarray(ec["last_updated"])[keep], dtype=torch.float64))
    g.decay_log = clock
    g.clear_tracking()


def _jsonable_cols(cols: Dict) -> Dict:
    return {k: (v.tolist() if isinstance(v, np.ndarray) else v) for k, v in cols.items()}


def _max_node_num(ids) -> int:
    """Largest n of the ``node_<n>`` ids (reference id scheme), 0 if none
    (a C loop over the list when the runtime is built)."""
    if len(ids) > 4096:
        try:
            from ..store.colstore import _rt
            return int(_rt().max_node_num(ids))
        except (ImportError, AttributeError):
            pass
    mx = 0
    for nid in ids:
        m = _NODE_ID.match(nid)
        if m:
            mx = max(mx, int(m.group(1)))
    return mx


def _h2d_pieces(pieces, n: int, d: int, dev, chunk_bytes: int = 256 << 20) -> torch.Tensor:
    """[n, d] fp32 device tensor from row-ordered host pieces (views of the
    store's mapped fragments): each 256 MB chunk is copied by the runtime's
    multi-threaded memcpy (GIL released) into one of two pinned staging
    buffers while the previous one's async copy to the device runs."""
    from ..store.colstore import _rt
    out = torch.empty((n, d), dtype=torch.float32, device=dev)
    per_rows = max(1, chunk_bytes // (4 * d))
    bufs = [torch.empty((per_rows, d), dtype=torch.float32).pin_memory() for _ in range(2)]
    evs = [None, None]
    st = torch.cuda.current_stream(dev)
    rt = _rt()
    r0, j = 0, 0
    for p in pieces:
        p = np.ascontiguousarray(p, dtype=np.float32)
        m = p.shape[0]
        for a in range(0, m, per_rows):
            b = min(m, a + per_rows)
            k = j & 1
            if evs[k] is not None:
                evs[k].synchronize()
            rt.par_copy(bufs[k].data_ptr(), p[a:b].ctypes.data, (b - a) * d * 4)
            out[r0 + a: r0 + b].copy_(bufs[k][: b - a], non_blocking=True)
            evs[k] = torch.cuda.Event()
            evs[k].record(st)
            j += 1
        r0 += m
    if r0 != n:
        raise RuntimeError(f"vector pieces hold {r0} rows, expected {n}")
    st.synchronize()
    return out


def _h2d(a: np.ndarray, dev, chunk_bytes: int = 64 << 20) -> torch.Tensor:
    """Host array -> device tensor through two pinned staging buffers (the
    memcpy into one overlaps the async copy out of the other): no pinning of
    the whole array, no pageable-memory DMA."""
    out = torch.empty(a.shape, dtype=torch.from_numpy(a[:0]).dtype, device=dev)
    flat_src = a.reshape(-1)
    flat_dst = out.view(-1)
    per = max(1, chunk_bytes // a.itemsize)
    bufs = [torch.empty(per, dtype=out.dtype).pin_memory() for _ in range(2)]
    evs = [None, None]
    st = torch.cuda.current_stream(dev)
    for j, c0 in enumerate(range(0, flat_src.size, per)):
        c1 = min(flat_src.size, c0 + per)
        b = j & 1
        if evs[b] is not None:
            evs[b].synchronize()
        bufs[b][: c1 - c0].copy_(torch.from_numpy(flat_src[c0:c1]))  # multi-threaded host copy
        flat_dst[c0:c1].copy_(bufs[b][: c1 - c0], non_blocking=True)
        evs[b] = torch.cuda.Event()
        evs[b].record(st)
    st.synchronize()
    return out


def _default_local_embedder() -> EmbeddingProvider:
    """Offline default: on-device encoder when weights are configured
    (``LZK_ENCODER_WEIGHTS``), else the lexical hash embedder."""
    w = os.environ.get("LZK_ENCODER_WEIGHTS")
    if w:
        from .embedders import OnDeviceEmbedder
        return OnDeviceEmbedder(os.environ.get("LZK_ENCODER_MODEL", "minilm-l6"), weights=w)
    return HashEmbedder()
