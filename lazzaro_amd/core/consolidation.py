"""Consolidation pipeline of :class:`MemorySystem` (mixin).

Reference: ``core/memory_system.py:535-1120`` (buffer-limit eviction,
end-of-conversation fact extraction, dedupe, associative linking, super-node
hierarchy, deep consolidation, profile extraction, merge-similar).

Same observable behaviour and constants; the engine work is
batched instead of pairwise:

* dedupe (reference :719-733) = ONE batched top-1 store search for all new
  facts -- equivalent because the store does not change inside the loop;
* linking (:797-889) = one ``[new x existing]`` cosine top-3 per pass
  (``similarity.topk_cosine``: float64 host GEMM or the MFMA kernel on GPU);
* eviction scores (:535-578) are one vectorised importance + stable argsort;
* component edge averages (:970-985) are one pass over the edges.

Fixes, all behind documented defaults:
* embeddings are aligned per kept fact (reference :706/:720 misalignment);
* zero-vector facts (failed embedding) are not stored;
* background consolidation and the caller's end_conversation are serialised
  by ``self._graph_lock`` (the reference mutates shared state from 2 threads);
* ``merge_mode="pairwise"`` enables the intended all-pairs merge; the default
  ``"reference"`` keeps the reference's effective no-op (:1073-1077).
"""
from __future__ import annotations

import json
import time
from collections import defaultdict
from typing import Dict, List, Set, Tuple

import numpy as np

from ..models.graph import Edge, Node
from .similarity import topk_cosine
from ..utils.faults import EmbeddingError, ProviderError, degenerate_embedding
from ..utils.tracing import tracer

EXTRACTION_PROMPT = """Extract distinct, atomic facts from this conversation.
Categorization Guidelines:
1. semantic: Stable facts, preferences, or knowledge (e.g., "User likes Python", "User lives in London").
2. episodic: Specific events, occurrences, or recent activities (e.g., "User started a new job today", "User fixed a bug in the API").
3. procedural: Processes, workflows, or instructions (e.g., "User follows the git-flow model", "User prefers TDD for testing").

Format Rules:
- Formulate facts in the THIRD PERSON.
- Abstract from conversational filler.
- If no new facts, return empty list.

Return JSON: {"memories": [{"content": "...", "type": "semantic|episodic|procedural", "salience": 0.0-1.0, "topic": "work|personal|learning|health|other"}]}
"""

PROFILE_PROMPT = """Analyze these related memories and generate brief, factual personality insights (1-2 sentences each).
Identify all applicable domains: preferences, personality_traits, knowledge_domains, interaction_style, or key_experiences.
Return a JSON object where keys are the domain names and values are the specific insights.
Example: {"preferences": "User prefers Python for data science.", "knowledge_domains": "Exhibits deep expertise in memory systems."}"""

DEDUPE_THRESHOLD = 0.95
LINK_THRESHOLD = 0.5
LINK_TOPK = 3
LINK_WEIGHT_SCALE = 0.8
CHAIN_WEIGHT = 0.5
MIN_FACT_LEN = 5


def _parse_json(response: str):
    if response is None:
        raise json.JSONDecodeError("empty", "", 0)
    if "```json" in response:
        response = response.split("```json")[1].split("```")[0].strip()
    return json.loads(response)


class ConsolidationMixin:
    # ------------------------------------------------------------ eviction
    def _enforce_buffer_limit(self):
        total, _ = self.buffer.size()
        if total <= self.max_buffer_size:
            return
        excess = total - self.max_buffer_size
        now = time.time()
        cand: List[Tuple[str, str]] = []
        sal, acc, last = [], [], []
        for sh in self.shards.values():
            for nid, n in sh.nodes.items():
                if n.is_super_node:
                    continue
                cand.append((nid, n.shard_key))
                sal.append(n.salience)
                acc.append(n.access_count)
                last.append(n.last_accessed)
        if not cand:
            return
        sal = np.asarray(sal, dtype=np.float64)
        acc = np.asarray(acc, dtype=np.float64)
        days = (now - np.asarray(last, dtype=np.float64)) / 86400.0
        importance = 0.5 * sal + 0.3 * np.minimum(1.0, acc / 10.0) + 0.2 / (1.0 + days)
        order = np.argsort(importance, kind="stable")[:excess]
        victims = [cand[i] for i in order]
        removed = 0
        for nid, skey in victims:
            sh = self.shards.get(skey)
            if sh is not None and sh.remove_node(nid):
                removed += 1
        if removed:
            ids = [nid for nid, _ in victims]
            self._emb_cache.forget(ids)
            self.vector_store.delete_nodes(ids, user_id=self.user_id)
            self._say(f"⚠ Buffer limit reached! Archived {removed} old nodes (limit: {self.max_buffer_size})")

    # ------------------------------------------------------------ end of conversation
    def end_conversation(self) -> str:
        if not self.conversation_active:
            return "⚠ No active conversation to end."
        self.conversation_active = False
        if not self.short_term_memory:
            return "✓ Conversation ended. No memories to consolidate."
        results = []
        if self.enable_async and self.background_executor:
            self._say(f"🔄 Queueing consolidation for {len(self.short_term_memory)} exchanges...")
            with self._queue_lock:
                self.consolidation_queue.append({"memories": list(self.short_term_memory),
                                                 "timestamp": time.time()})
            self._pending.append(self.background_executor.submit(self._async_consolidate))
            results.append("✓ Conversation ended (consolidation queued)")
        else:
            self._say(f"🔄 Consolidating {len(self.short_term_memory)} exchanges...")
            results.append(self._consolidate_to_buffer())

        with self._graph_lock:
            self.buffer.apply_temporal_decay(decay_rate=0.01)
            results.append("✓ Applied temporal decay")
            if self.auto_prune:
                pruned = self.buffer.prune_weak_edges(threshold=self.prune_threshold)
                if pruned > 0:
                    results.append(f"✓ Auto-pruned {pruned} weak edges")
            self._enforce_buffer_limit()
            self.conversation_count += 1
            if self.auto_consolidate and self.conversation_count % self.consolidate_every == 0:
                self._say(f"🔄 Auto-consolidation triggered (every {self.consolidate_every} conversations)...")
                results.append(self.run_consolidation())
            self.short_term_memory = []
            self.conversation_history = []
            self._save_to_persistence()
        return "\n".join(results)

    def _consolidate_to_buffer(self) -> str:
        with self._queue_lock:
            self.consolidation_queue.append({"memories": list(self.short_term_memory),
                                             "timestamp": time.time()})
        self._async_consolidate()
        n, e = self.buffer.size()
        return f"✓ Consolidation complete. Memory: {n} nodes, {e} edges"

    def _side_stream(self):
        """Background consolidation runs on its own HIP stream so its kernels
        overlap the caller's retrieval kernels (SURVEY.md §2.6 async row)."""
        import contextlib

        import torch

        dev = self._device
        if dev is None or getattr(dev, "type", "cpu") != "cuda" or not torch.cuda.is_available():
            return contextlib.nullcontext()
        if getattr(self, "_cstream", None) is None:
            self._cstream = torch.cuda.Stream(device=dev)
        return torch.cuda.stream(self._cstream)

    def flush(self, timeout: float = None) -> None:
        """Block until queued background consolidations have finished."""
        pend, self._pending = self._pending, []
        for f in pend:
            f.result(timeout=timeout)

    # ------------------------------------------------------------ fact extraction
    def _async_consolidate(self):
        """Fact extraction -> embed -> ingest (reference memory_system.py:651-785).

        Failure policy: the reference drains the queue first and
        loses the memories when the LLM call, the JSON parse or the embedding
        fails. Here a failed batch is put back at the FRONT of the queue with an
        attempt count and retried by the next consolidation; after
        ``max_consolidation_retries`` attempts it is dropped and counted.
        ``strict_errors`` re-raises instead."""
        with self._queue_lock:
            if not self.consolidation_queue:
                return
            batches, self.consolidation_queue = self.consolidation_queue, []
        t0 = time.time()
        try:
            self._consolidate_batches(batches)
        except Exception as e:
            self.metrics["consolidation_failures"] = self.metrics.get("consolidation_failures", 0) + 1
            retry = []
            for b in batches:
                b = dict(b)
                b["attempts"] = b.get("attempts", 0) + 1
                if b["attempts"] < self.max_consolidation_retries:
                    retry.append(b)
                else:
                    self.metrics["dropped_batches"] = self.metrics.get("dropped_batches", 0) + 1
            with self._queue_lock:
                self.consolidation_queue[:0] = retry
            self._say(f"⚠ Consolidation failed ({type(e).__name__}: {e}); "
                      f"{len(retry)} batch(es) re-queued")
            if self.strict_errors:
                raise
            return
        elapsed = time.time() - t0
        self.metrics["consolidation_times"].append(elapsed)
        self._say(f"✓ Background consolidation complete ({elapsed:.2f}s)")
        with self._graph_lock:
            self._save_to_persistence()

    def _consolidate_batches(self, batches: List[Dict]) -> None:
        memories = [m for b in batches for m in b["memories"]]
        self._say(f"🔄 Processing {len(memories)} memories in background...")
        with tracer.stage("extract_llm", "cpu"):
            response = self._call_llm(
                [{"role": "system", "content": EXTRACTION_PROMPT},
                 {"role": "user", "content": json.dumps(memories)}],
                response_format={"type": "json_object"})
        try:
            data = _parse_json(response)
        except (json.JSONDecodeError, TypeError) as e:
            self._say(f"⚠ Parse error: {e}")
            raise ProviderError(f"unparseable extraction response: {e}") from e
        if isinstance(data, dict):
            facts = data.get("memories", [])
        elif isinstance(data, list):
            facts = data
        else:
            self._say(f"⚠ Unexpected data type: {type(data)}")
            return
        facts = [m for m in facts if isinstance(m, dict)] if isinstance(facts, list) else []
        self._say(f"✓ Extracted {len(facts)} memory candidates")
        kept = [m for m in facts if m.get("content") and len(m.get("content", "")) >= MIN_FACT_LEN]
        with self._side_stream():
            with tracer.stage("embed_facts", self._device):
                embs = self._batch_embed([m["content"] for m in kept]) if kept else []
            if kept and all(degenerate_embedding(e) for e in embs):
                # a provider outage (zero vectors for everything): retry later
                raise EmbeddingError("embedding provider returned only degenerate vectors")
            with self._graph_lock, tracer.stage("ingest", self._device):
                self._ingest_facts(kept, embs)

    def _ingest_facts(self, facts: List[Dict], embs: List[List[float]]) -> List[Tuple[str, str]]:
        # K5: one batched top-1 search for every fact (the store is unchanged
        # during this loop in the reference too, so this is equivalent).
        valid = [i for i, e in enumerate(embs) if e is not None and len(e) and not degenerate_embedding(e)]
        rejected = len(facts) - len(valid)
        if rejected:
            self.metrics["rejected_embeddings"] = self.metrics.get("rejected_embeddings", 0) + rejected
        hits = {}
        if valid:
            res = self._search_batch([embs[i] for i in valid], 1)
            hits = {i: (r[0] if r else None) for i, r in zip(valid, res)}
        new_nodes: List[Tuple[str, str]] = []
        rows = []
        undo = []  # (node, salience, last_accessed, access_count) of merged duplicates
        for i, mem in enumerate(facts):
            content = mem["content"]
            emb = embs[i] if i < len(embs) else []
            if i not in hits:
                self._say("   (skipped fact with empty/zero embedding)")
                continue
            shard_key = mem.get("topic", self._infer_shard_key(content))
            shard = self._get_or_create_shard(shard_key)
            best_id = hits.get(i)
            if best_id is not None:
                best = self.buffer.get_node(best_id)
                if best is not None and self._cosine_similarity(emb, best.embedding) > DEDUPE_THRESHOLD:
                    undo.append((best, best.salience, best.last_accessed, best.access_count))
                    best.salience = max(best.salience, mem.get("salience", 0.5))
                    best.last_accessed = time.time()
                    best.access_count += 1
                    self._say(f"   (Merged semantic duplicate into {best.id})")
                    continue
            nid = self._generate_node_id()
            node = Node(id=nid, content=content, embedding=list(emb), type=mem.get("type", "semantic"),
                        salience=mem.get("salience", 0.5), shard_key=shard_key)
            shard.add_node(node)
            new_nodes.append((nid, shard_key))
            rows.append({"id": nid, "content": content, "embedding": node.embedding, "type": node.type,
                         "salience": node.salience, "shard_key": node.shard_key,
                         "timestamp": node.timestamp})
        if rows:
            try:
                self.vector_store.add_nodes(rows, user_id=self.user_id)
            except Exception:
                # roll the graph back so the re-queued batch applies exactly once
                for nid, skey in new_nodes:
                    self.shards[skey].remove_node(nid)
                for node, sal, la, ac in undo:
                    node.salience, node.last_accessed, node.access_count = sal, la, ac
                raise
            if self.query_cache:
                self.query_cache.invalidate_results()
        self._link_within_shards(new_nodes)
        self._link_to_existing_memories(new_nodes)
        self._enforce_buffer_limit()
        if self.enable_hierarchy:
            for skey in dict.fromkeys(sk for _, sk in new_nodes):
                sh = self.shards.get(skey)
                if sh is not None and len(sh.nodes) > self.super_node_threshold:
                    self._create_super_nodes_for_shard(skey)
        return new_nodes

    # ------------------------------------------------------------ linking (K6)
    def _link_within_shards(self, new_nodes: List[Tuple[str, str]]):
        groups: Dict[str, List[str]] = defaultdict(list)
        for nid, sk in new_nodes:
            groups[sk].append(nid)
        for sk, ids in groups.items():
            if len(ids) < 2:
                continue
            shard = self.shards[sk]
            for a, b in zip(ids, ids[1:]):
                shard.add_edge(Edge(source=a, target=b, weight=CHAIN_WEIGHT, edge_type="relates_to"))
            new_set = set(ids)
            cand_ids = [x for x in shard.nodes if x not in new_set]
            if not cand_ids:
                continue
            Q = self._emb_cache.matrix([shard.nodes[x] for x in ids])
            C = self._emb_cache.matrix([shard.nodes[x] for x in cand_ids], dim=Q.shape[1])
            sims, idx = topk_cosine(Q, C, LINK_TOPK, device=self._device)
            for qi, nid in enumerate(ids):
                for s, j in zip(sims[qi], idx[qi]):
                    if j >= 0 and s > LINK_THRESHOLD:
                        shard.add_edge(Edge(source=nid, target=cand_ids[j], weight=float(s) * LINK_WEIGHT_SCALE,
                                            edge_type="relates_to"))

    def _edge_exists_any(self, a: str, b: str) -> bool:
        for sh in self.shards.values():
            if (a, b) in sh.edges or (b, a) in sh.edges:
                return True
        return False

    def _link_to_existing_memories(self, new_nodes: List[Tuple[str, str]]):
        if not new_nodes:
            return
        new_ids = {nid for nid, _ in new_nodes}
        existing: Dict[str, Node] = {}
        for sh in self.shards.values():
            for nid, n in sh.nodes.items():
                if nid not in new_ids and not n.is_super_node:
                    existing[nid] = n
        if not existing:
            return
        ex_ids = list(existing.keys())
        live = [(nid, sk, self.buffer.get_node(nid)) for nid, sk in new_nodes]
        live = [(nid, sk, n) for nid, sk, n in live if n is not None]
        if not live:
            return
        Q = self._emb_cache.matrix([n for _, _, n in live])
        C = self._emb_cache.matrix([existing[x] for x in ex_ids], dim=Q.shape[1])
        sims, idx = topk_cosine(Q, C, LINK_TOPK, device=self._device)
        made = 0
        for qi, (nid, sk, _) in enumerate(live):
            for s, j in zip(sims[qi], idx[qi]):
                if j < 0 or not s > LINK_THRESHOLD:
                    continue
                tgt = ex_ids[j]
                if self._edge_exists_any(nid, tgt):
                    continue
                sh = self.shards.get(sk)
                if sh is not None:
                    sh.add_edge(Edge(source=nid, target=tgt, weight=float(s) * LINK_WEIGHT_SCALE,
                                     edge_type="relates_to"))
                    made += 1
        if made:
            self._say(f"✓ Created {made} cross-conversation links")

    # ------------------------------------------------------------ hierarchy (K8/K16)
    def _create_super_nodes_for_shard(self, shard_key: str):
        shard = self.shards[shard_key]
        if len(shard.nodes) < self.super_node_threshold:
            return
        if any(n.shard_key == shard_key for n in self.super_nodes.values()):
            return
        self._say(f"  Creating super-node for shard '{shard_key}' ({len(shard.nodes)} nodes)")
        nodes = list(shard.nodes.values())
        sid = f"super_{shard_key}_{int(time.time())}"
        summary = f"Topic: {shard_key}. Contains memories about: " + "; ".join(n.content for n in nodes[:3])
        embs = [n.embedding for n in nodes if n.embedding]
        mean = np.mean(np.asarray(embs, dtype=np.float64), axis=0).tolist() if embs else []
        sup = Node(id=sid, content=summary, embedding=mean, type="semantic", is_super_node=True,
                   child_ids=[n.id for n in nodes], shard_key=shard_key)
        for n in nodes:
            n.parent_id = sid
        self.super_nodes[sid] = sup
        self._say(f"  ✓ Created super-node {sid} with {len(nodes)} children")

    # ------------------------------------------------------------ deep consolidation
    def run_consolidation(self, weight_threshold: float = 0.6, merge_similar: bool = True) -> str:
        results = []
        self._say("🔄 Running consolidation...")
        with self._graph_lock:
            if merge_similar:
                merged = self._merge_similar_nodes(similarity_threshold=DEDUPE_THRESHOLD)
                if merged > 0:
                    results.append(f"✓ Merged {merged} similar nodes")
            comps = self.buffer.get_connected_components()
            comp_of = {}
            for ci, comp in enumerate(comps):
                for nid in comp:
                    comp_of[nid] = ci
            wsum = defaultdict(float)
            wcnt = defaultdict(int)
            for sh in self.shards.values():
                for (s, t), e in sh.edges.items():
                    cs = comp_of.get(s)
                    if cs is not None and cs == comp_of.get(t):
                        wsum[cs] += e.weight
                        wcnt[cs] += 1
        updates = 0
        for ci, comp in enumerate(comps):
            if len(comp) < 3 or not wcnt.get(ci):
                continue
            if wsum[ci] / wcnt[ci] > 0.3:
                r = self._extract_profile_from_component(comp)
                if "Updated" in r:
                    updates += 1
                    results.append(r)
        with self._graph_lock:
            pruned = self.buffer.prune_weak_edges(threshold=self.prune_threshold)
        if pruned > 0:
            results.append(f"✓ Pruned {pruned} weak edges")
        if updates > 0:
            results.append(f"✓ Updated {updates} profile domains")
        else:
            contents = [n.content for n in self.buffer.nodes.values() if not n.is_super_node]
            if len(contents) >= 3:
                r = self._extract_profile_from_contents(contents)
                if "Updated" in r:
                    results.append(r)
        if not results:
            results.append("✓ No consolidation actions needed")
        return "\n".join(results)

    def _extract_profile_from_component(self, component: Set[str]) -> str:
        contents = []
        for nid in component:
            n = self.buffer.get_node(nid)
            if n is not None and not n.is_super_node:
                contents.append(n.content)
        if not contents:
            return "No content to extract"
        return self._extract_profile_from_contents(contents)

    def _extract_profile_from_contents(self, contents: List[str]) -> str:
        if not contents:
            return "No content to extract"
        prompt = "Related memories:\n" + "\n".join(f"- {c}" for c in contents[:10])
        response = self._call_llm([{"role": "system", "content": PROFILE_PROMPT},
                                   {"role": "user", "content": prompt}],
                                  response_format={"type": "json_object"})
        try:
            data = _parse_json(response)
            if not isinstance(data, dict):
                return "Failed to extract profile"
            updated = False
            for domain, insight in data.items():
                if domain not in self.profile.data or not insight:
                    continue
                insight = insight if isinstance(insight, str) else str(insight)
                cur = self.profile.data.get(domain, "")
                new = f"{cur}. {insight}".strip() if (cur and insight not in cur) else insight
                self.profile.update_domain(domain, new)
                self._say(f"  ✓ Profile updated: {domain} = {insight[:50]}...")
                updated = True
            if updated:
                return "✓ Updated profile domains"
        except (json.JSONDecodeError, TypeError) as e:
            self._say(f"  ⚠ JSON parse error: {e}")
        return "Failed to extract profile"

    # ------------------------------------------------------------ merge (K7)
    def _merge_similar_nodes(self, similarity_threshold: float = DEDUPE_THRESHOLD) -> int:
        nodes = self.buffer.nodes
        if len(nodes) < 2:
            return 0
        if self.merge_mode != "pairwise":
            # reference behaviour: the inner loop is dedented out of the outer
            # one (memory_system.py:1073-1077) so nothing is ever compared
            return 0
        items = [(nid, n) for nid, n in nodes.items() if not n.is_super_node]
        if len(items) < 2:
            return 0
        M = self._emb_cache.matrix([n for _, n in items])
        S = M @ M.T
        processed: Set[str] = set()
        merged = 0
        for i, (id1, n1) in enumerate(items):
            if id1 in processed:
                continue
            for j in range(i + 1, len(items)):
                id2, n2 = items[j]
                if id2 in processed or not S[i, j] > similarity_threshold:
                    continue
                n1.content = f"{n1.content} | {n2.content}"
                n1.salience = max(n1.salience, n2.salience)
                n1.access_count += n2.access_count
                for sh in self.shards.values():
                    if id2 not in sh.nodes:
                        continue
                    for key in list(sh.edges.incident(id2)):
                        e = sh.edges.pop(key)
                        s, t = key
                        e.source, e.target = (id1 if s == id2 else s), (id1 if t == id2 else t)
                        if (e.source, e.target) in sh.edges:
                            sh.add_edge(e)
                        else:
                            sh.edges[(e.source, e.target)] = e
                    del sh.nodes[id2]
                    break
                processed.add(id2)
                merged += 1
                self._emb_cache.forget([id2])
                self.vector_store.delete_nodes([id2, id1], user_id=self.user_id)
                self.vector_store.add_nodes([{
                    "id": id1, "content": n1.content, "embedding": n1.embedding, "type": n1.type,
                    "salience": n1.salience, "shard_key": n1.shard_key, "timestamp": n1.timestamp}],
                    user_id=self.user_id)
        return merged
