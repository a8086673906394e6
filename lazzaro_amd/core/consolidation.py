"""Consolidation pipeline of :class:`MemorySystem` (mixin), on the device graph.

Reference: ``core/memory_system.py:535-1120`` (buffer-limit eviction,
end-of-conversation fact extraction, dedupe, associative linking, super-node
hierarchy, deep consolidation, profile extraction, merge-similar).

Same observable behaviour and constants; every graph step
runs on the tenant's :class:`~lazzaro_amd.engine.TenantGraph` (HBM columns +
HIP kernels on a GPU, the same tensor code on the CPU):

* dedupe, within-shard links and cross-memory links of a batch of M facts come
  from ONE fused scan (``flat_topk_dual``: a global and a shard-filtered list)
  with exact float64 re-ranking -- the reference does M store searches plus
  2*M*N Python cosines (:719-733, :797-889);
* decay + auto-prune is one kernel pass over the edge and node columns
  (``tg_decay_kernel``), eviction is ``tg_importance_kernel`` + a stable select
  + ``tg_flag_remove`` compaction, neighbour boost ``tg_boost_kernel``;
* connected components are the hook/compress kernels; per-component edge
  weight averages one segmented reduction;
* the pairwise merge (opt-in) takes candidate pairs from the MFMA
  ``pairs_kernel`` and confirms them in float64.

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
from typing import Dict, List, Sequence, Set, Tuple

import numpy as np
import torch

from ..engine.tenant_graph import NODE, SHARD_MASK, TYPE_MASK, TenantGraph
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
DECAY_RATE = 0.01
PROFILE_CONTENTS = 10  # contents per profile prompt (reference memory_system.py:1032)
SALIENCE_FLOOR_ = 0.2  # node salience decays towards it (reference memory_shard.py:64-77)


def batch_dedupe(Qn: torch.Tensor, ct: torch.Tensor, gb_s: torch.Tensor, gb_node: torch.Tensor):
    """In-batch dedupe of a fact batch (reference :719-741 applied to B
    conversations in order): fact j is a duplicate when its best match -- the
    store top-1 over the pre-batch graph (``gb_s``, cosine; ``gb_node``: it is
    a live node) or a KEPT fact of an earlier conversation -- exceeds
    DEDUPE_THRESHOLD. Kept-ness depends on earlier facts' decisions, so the
    masks are iterated to their fixed point. Qn: unit fp64 [M, D]; ct: the
    conversation of each fact [M]. Returns (S = Qn Qn^T, earlier[j, i],
    dup, batch_best, bb_i, ins)."""
    NEG = float("-inf")
    M = Qn.shape[0]
    S = Qn @ Qn.T
    earlier = ct[None, :] < ct[:, None]  # [j, i]: fact i is from an earlier conversation than j
    ins = torch.ones(M, dtype=torch.bool, device=Qn.device)
    for _ in range(M + 1):
        A = torch.where(earlier & ins[None, :], S, torch.full_like(S, NEG))
        bb_s = A.max(1).values
        bb_i = torch.argmax((A == bb_s[:, None]).to(torch.int8), 1)
        batch_best = bb_s > gb_s
        best_s = torch.where(batch_best, bb_s, gb_s)
        dup = (best_s > DEDUPE_THRESHOLD) & (batch_best | gb_node)
        if torch.equal(~dup, ins):
            break
        ins = ~dup
    return S, earlier, dup, batch_best, bb_i, ins


def salience_decayed(s: torch.Tensor, n: torch.Tensor, keep: float) -> torch.Tensor:
    """Node salience after ``n`` decays (floor SALIENCE_FLOOR_, memory_shard.py:64-77)."""
    kn = torch.pow(torch.full_like(s, keep), n.double())
    return torch.where(s > SALIENCE_FLOOR_, SALIENCE_FLOOR_ + (s - SALIENCE_FLOOR_) * kn,
                       torch.full_like(s, SALIENCE_FLOOR_))


def batch_link_plan(kidx, new_row, code_all, ct, S, earlier, shard_hits, global_hits, keep: float, B: int, thr,
                    stats: Dict[str, int]):
    """Edges created by the kept facts of a batch (reference :797-891), in
    the reference's order (per conversation: chain, within-shard, cross-memory)
    and pre-decayed by the end_conversation calls from their conversation on.

    ``kidx``: kept fact positions; ``new_row[M]``: the node key each fact
    became (-1 not kept) -- graph rows here, global node numbers for a
    row-sharded tenant; ``code_all[M]``: shard codes; ``shard_hits`` /
    ``global_hits``: (sims [M, 3], keys [M, 3]) from the pre-batch graph in the
    same key space. Updates stats (linked, cross_links, pruned). Returns
    (src, dst, w fp64, shard) keys or None, and the cross-link count."""
    dev = S.device
    M = S.shape[0]
    NEG = float("-inf")
    K = kidx.numel()
    kc = ct[kidx]
    kcode = code_all[kidx].long()
    # shards with >= 2 new nodes in the same conversation (reference :814-815)
    key = kc * (1 << 24) + kcode
    uniq, inv, cnt = torch.unique(key, return_inverse=True, return_counts=True)
    multi = cnt[inv] >= 2
    ins_b = torch.zeros(M, dtype=torch.bool, device=dev)
    ins_b[kidx] = True
    code_all = code_all.long()
    es, ed, ew, eh, order = [], [], [], [], []
    # chain edges between consecutive new nodes of a (conversation, shard)
    o = torch.argsort(key * K + torch.arange(K, device=dev))
    ks = key[o]
    adj = torch.nonzero(ks[1:] == ks[:-1]).flatten()
    if adj.numel():
        a, b = o[adj], o[adj + 1]
        es.append(new_row[kidx[a]])
        ed.append(new_row[kidx[b]])
        ew.append(torch.full((a.numel(),), CHAIN_WEIGHT, dtype=torch.float64, device=dev))
        eh.append(kcode[a])
        order.append(kc[a] * 4)
    Sk = S[kidx]  # [K, M]
    ek = earlier[kidx] & ins_b[None, :]

    def merged_top(graph_s, graph_r, batch_mask):
        bs = torch.where(batch_mask, Sk, torch.full_like(Sk, NEG))
        t = min(LINK_TOPK, M)
        tb_s, tb_i = torch.topk(bs, t, dim=1)
        tb_r = torch.where(torch.isneginf(tb_s), torch.full_like(tb_i, -1), new_row[tb_i])
        cs = torch.cat([graph_s[kidx], tb_s], 1)
        cr = torch.cat([graph_r[kidx], tb_r], 1)
        keyr = torch.where(cr >= 0, cr, torch.full_like(cr, 1 << 62))
        o2 = torch.argsort(keyr, dim=1, stable=True)
        cs, cr = torch.gather(cs, 1, o2), torch.gather(cr, 1, o2)
        o3 = torch.sort(cs, dim=1, descending=True, stable=True).indices[:, :LINK_TOPK]
        return torch.gather(cs, 1, o3), torch.gather(cr, 1, o3)

    # within-shard similarity links: same shard, from the graph or earlier conversations
    sw_, sr_ = merged_top(shard_hits[0], shard_hits[1], ek & (code_all[None, :] == kcode[:, None]))
    src = new_row[kidx][:, None].expand(-1, LINK_TOPK)
    mw = (sr_ >= 0) & (sw_ > LINK_THRESHOLD) & multi[:, None]
    es.append(src[mw])
    ed.append(sr_[mw])
    ew.append(sw_[mw] * LINK_WEIGHT_SCALE)
    eh.append(kcode[:, None].expand_as(sr_)[mw])
    order.append(kc[:, None].expand_as(sr_)[mw] * 4 + 1)
    # cross-memory links: any non-super node, skipping pairs linked within the shard
    gw_, gr_ = merged_top(global_hits[0], global_hits[1], ek)
    mg = (gr_ >= 0) & (gw_ > LINK_THRESHOLD)
    mg &= ~((gr_[:, :, None] == sr_[:, None, :]) & mw[:, None, :]).any(dim=2)
    es.append(src[mg])
    ed.append(gr_[mg])
    ew.append(gw_[mg] * LINK_WEIGHT_SCALE)
    eh.append(kcode[:, None].expand_as(gr_)[mg])
    order.append(kc[:, None].expand_as(gr_)[mg] * 4 + 2)
    n_cross = int(mg.sum())
    Sr, Dr = torch.cat(es), torch.cat(ed)
    if Sr.numel() == 0:
        return None, n_cross
    W = torch.cat(ew)
    Ord = torch.cat(order)
    # decays of the end_conversation calls from the edge's conversation on
    W = W * torch.pow(torch.full_like(W, keep), (B - torch.div(Ord, 4, rounding_mode="floor")).double())
    stats["linked"] += int(Sr.numel())
    stats["cross_links"] += n_cross
    H = torch.cat(eh)
    o = torch.argsort(Ord, stable=True)
    Sr, Dr, W, H = Sr[o], Dr[o], W[o], H[o]
    if thr is not None:
        alive = W >= thr
        stats["pruned"] += int((~alive).sum())
        Sr, Dr, W, H = Sr[alive], Dr[alive], W[alive], H[alive]
    if Sr.numel() == 0:
        return None, n_cross
    return (Sr, Dr, W, H), n_cross


def _parse_json(response: str):
    if response is None:
        raise json.JSONDecodeError("empty", "", 0)
    if "```json" in response:
        response = response.split("```json")[1].split("```")[0].strip()
    return json.loads(response)


class ConsolidationMixin:
    graph: TenantGraph

    # ------------------------------------------------------------ eviction
    def _enforce_buffer_limit(self):
        g = self.graph
        if g.num_nodes() <= self.max_buffer_size:
            return
        with tracer.stage("evict", self._device):
            victims = g.evict(self.max_buffer_size)
        if victims:
            ids = [g.ids[r] for r in victims]
            self._store_delete(ids)
            self._say(f"⚠ Buffer limit reached! Archived {len(victims)} old nodes (limit: {self.max_buffer_size})")

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
            # decay (memory_shard.py:64-77) and auto-prune (:79-84) in one pass
            with tracer.stage("decay_prune", self._device):
                pruned = self.graph.decay(DECAY_RATE, self.prune_threshold if self.auto_prune else None)
            results.append("✓ Applied temporal decay")
            if self.auto_prune and pruned > 0:
                results.append(f"✓ Auto-pruned {pruned} weak edges")
            self._enforce_buffer_limit()
            self.conversation_count += 1
            if self.auto_consolidate and self.conversation_count % self.consolidate_every == 0:
                self._say(f"🔄 Auto-consolidation triggered (every {self.consolidate_every} conversations)...")
                results.append(self.run_consolidation())
            self._maybe_cluster(self.conversation_count - 1)
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

    def flush(self, timeout: float = None) -> None:
        """Block until queued background consolidations have finished."""
        pend, self._pending = self._pending, []
        for f in pend:
            f.result(timeout=timeout)
        self.flush_persistence()

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
        with tracer.stage("embed_facts", self._device):
            embs = self._batch_embed_any([m["content"] for m in kept]) if kept else None
        if kept and self._all_degenerate(embs):
            # a provider outage (zero vectors for everything): retry later
            raise EmbeddingError("embedding provider returned only degenerate vectors")
        with self._graph_lock, tracer.stage("ingest", self._device):
            self._ingest_facts(kept, embs)

    @staticmethod
    def _all_degenerate(embs) -> bool:
        if embs is None:
            return True
        if torch.is_tensor(embs):
            if embs.numel() == 0:
                return True
            ok = torch.isfinite(embs).all(1) & (embs.abs().sum(1) > 0)
            return not bool(ok.any())
        return all(degenerate_embedding(e) for e in embs)

    # ------------------------------------------------------------ ingest (K5 + K6)
    def _ingest_facts(self, facts: List[Dict], embs) -> List[Tuple[str, str]]:
        """Dedupe, insert and link one batch of extracted facts (reference
        :706-785) on the device graph. ``embs``: [M, D] tensor or list of
        vectors aligned with ``facts``. Returns [(new node id, shard key)]."""
        g = self.graph
        M = len(facts)
        if M == 0:
            return []
        now = time.time()
        E, valid = self._fact_matrix(embs, M)
        rejected = M - int(valid.sum())
        if rejected:
            self.metrics["rejected_embeddings"] = self.metrics.get("rejected_embeddings", 0) + rejected
            self._say("   (skipped fact(s) with empty/zero embedding)")
        vidx = np.nonzero(valid)[0]
        if vidx.size == 0:
            return []
        # shards are created in fact order, duplicates included (reference :716-718)
        shard_keys = [facts[i].get("topic", self._infer_shard_key(facts[i]["content"])) for i in vidx]
        codes = np.asarray([g.shard_id(k) for k in shard_keys], dtype=np.int32)
        Q = E[torch.as_tensor(vidx, dtype=torch.long).to(E.device)]
        sal_in = torch.as_tensor([float(facts[i].get("salience", 0.5)) for i in vidx], dtype=torch.float32)

        with g.on_stream():
            (br, bs, bnode), (ls, lr), (ws, wr) = self._scan_batch(Q, torch.as_tensor(codes))
            dup_rows = torch.where(bnode & (br >= 0) & (bs > DEDUPE_THRESHOLD), br, -1)
        # --- dedupe: best store row is a node and cosine > 0.95 (reference :719-742)
        dup = dup_rows >= 0
        undo = None
        if bool(dup.any()):
            rows = dup_rows[dup]
            with g.on_stream():
                undo = (rows.clone(), g.sal[rows].clone(), g.last[rows].clone(), g.acc[rows].clone())
                g.sal.scatter_reduce_(0, rows, sal_in.to(g.device)[dup.to(sal_in.device)], "amax", include_self=True)
                g.last[rows] = now
                g.acc.index_add_(0, rows, torch.ones_like(rows, dtype=torch.int32))
                g.dirty[rows] = 1
            g._bump()
            for _ in range(int(dup.sum())):
                self._say("   (Merged semantic duplicate)")
        keep = (~dup).cpu().numpy()
        kidx = np.nonzero(keep)[0]
        if kidx.size == 0:
            return []
        kfacts = [facts[vidx[i]] for i in kidx]
        ids = [self._generate_node_id() for _ in kidx]
        kcodes = codes[kidx]
        kt = torch.as_tensor(kidx, dtype=torch.long).to(g.device)
        stored = self._store_binds_graph()
        rows = g.add_nodes(ids, [f["content"] for f in kfacts], Q[kt.to(Q.device)], shard=kcodes,
                           types=[f.get("type", "semantic") for f in kfacts], sal=sal_in[torch.as_tensor(kidx)],
                           now=now, stored=stored)
        new_nodes = [(i, shard_keys[j]) for i, j in zip(ids, kidx)]
        if not stored:
            try:
                self.vector_store.add_nodes([
                    {"id": i, "content": f["content"], "embedding": g.embedding(int(r)), "type": f.get("type", "semantic"),
                     "salience": float(f.get("salience", 0.5)), "shard_key": sk, "timestamp": now}
                    for i, f, r, (_, sk) in zip(ids, kfacts, rows.tolist(), new_nodes)], user_id=self.user_id)
            except Exception:
                # roll the graph back so the re-queued batch applies exactly once
                g.remove_nodes(rows, drop_edges=True)
                self.node_counter -= len(ids)
                if undo is not None:
                    with g.on_stream():
                        r_, s_, l_, a_ = undo
                        g.sal[r_], g.last[r_], g.acc[r_] = s_, l_, a_
                    g._bump()
                raise
        if self.query_cache:
            self.query_cache.invalidate_results()
        with tracer.stage("link", self._device):
            made = self._link_batch(rows, kcodes, (ws[kt], wr[kt]), (ls[kt], lr[kt]), now)
        if made:
            self._say(f"✓ Created {made} cross-conversation links")
        self._enforce_buffer_limit()
        if self.enable_hierarchy and getattr(self, "hierarchy_mode", "reference") == "reference":
            for skey in dict.fromkeys(sk for _, sk in new_nodes):
                c = g.shard_code.get(skey)
                if c is not None and g.shard_count[c] > self.super_node_threshold:
                    self._create_super_nodes_for_shard(skey)
        return new_nodes

    def _fact_matrix(self, embs, M: int):
        """[M, D] fp32 device tensor + valid mask (right dim, finite, non-zero)."""
        g = self.graph
        if torch.is_tensor(embs):
            E = embs.to(g.device, torch.float32)
            if g.dim is None:
                g._set_dim(E.shape[1])
            if E.shape[1] != g.dim:
                return E, np.zeros(M, dtype=bool)
            ok = torch.isfinite(E).all(1) & (E.abs().sum(1) > 0)
            return E, ok.cpu().numpy()
        rows = list(embs) if embs is not None else []
        if g.dim is None:
            for e in rows:
                if e is not None and len(e):
                    g._set_dim(len(e))
                    break
        D = g.dim or 0
        A = np.zeros((M, D), dtype=np.float32)
        ok = np.zeros(M, dtype=bool)
        for i in range(M):
            e = rows[i] if i < len(rows) else None
            if e is None or len(e) != D or degenerate_embedding(e):
                continue
            A[i] = np.asarray(e, dtype=np.float32)
            ok[i] = np.isfinite(A[i]).all()
        return torch.from_numpy(A).to(g.device), ok

    def _store_binds_graph(self) -> bool:
        return getattr(self.vector_store, "bound_graph", lambda u: None)(self.user_id) is self.graph

    def _scan_batch(self, Q: torch.Tensor, codes: torch.Tensor):
        """Dedupe best rows + link candidate lists for a fact batch.

        Returns (store top-1 row [M] (-1 none), its cosine, whether it is a
        live node), (global top-3 sims, rows) over existing non-super nodes,
        (same-shard top-3 sims, rows).
        Fast path (GPU, unit rows, store == graph nodes): one dual scan; the
        dedupe top-1 over store rows is the better of the global list's head
        and the (few) super-node rows. Otherwise the store search runs as the
        reference does it (L2 top-1 over the store's rows) and the links use
        the exact float64 scan."""
        g = self.graph
        n = g.n
        M = Q.shape[0]
        dev = g.device
        link_mask = (g.kind[:n] == NODE) & (g.sup[:n] == 0)
        fast = g._use_kernel(M) and self._store_binds_graph() and self.vector_store.metric == "l2" and \
            not bool(((g.stored[:n] == 1) & (g.kind[:n] != NODE)).any()) and \
            not bool(((g.kind[:n] == NODE) & (g.stored[:n] == 0)).any())
        kq = max(LINK_TOPK, 1)
        # decisions read only entries above LINK_THRESHOLD (links: cos > 0.5;
        # dedupe: top-1 > 0.95), so the scan may skip everything below it
        (gs, gr), (ws, wr) = g.cos_topk(Q, kq, link_mask, dual_label=codes, min_score=LINK_THRESHOLD)
        Qd = Q.to(dev, torch.float64)
        qn = Qd.norm(dim=1, keepdim=True)
        Qn = Qd / torch.where(qn > 0, qn, torch.ones_like(qn))
        if fast:
            best_s, best_r = gs[:, 0].clone(), gr[:, 0].clone()
            if g.n_super:
                srows = torch.as_tensor(g.node_rows_where(super_=True), dtype=torch.long).to(dev)
                ss, sr = g._exact_cos(Qn, torch.zeros(n, dtype=torch.bool, device=dev).index_fill_(0, srows, True), 1)
                better = (ss[:, 0] > best_s) | ((ss[:, 0] == best_s) & (sr[:, 0] < best_r))
                best_s = torch.where(better, ss[:, 0], best_s)
                best_r = torch.where(better, sr[:, 0], best_r)
            isnode = best_r >= 0
        else:
            _, top = self._store_top1(Q)
            best_r = top.to(dev).reshape(M, -1)[:, 0]
            ok = best_r >= 0
            rr = best_r.clamp_min(0)
            isnode = (g.kind[rr] == NODE) & ok
            X = g.emb32[rr].double()
            nrm = g.sqn[rr].double().sqrt()
            best_s = (Qn * X).sum(1) / torch.where(nrm > 0, nrm, torch.ones_like(nrm))
            best_s = torch.where(ok, best_s, torch.full_like(best_s, float("-inf")))
        return (best_r, best_s, isnode), (gs, gr), (ws, wr)

    def _store_top1(self, Q: torch.Tensor):
        """Top-1 of the store's vector search for each fact -> graph rows."""
        g = self.graph
        if self._store_binds_graph():
            return g.store_search(Q, 1, self.vector_store.metric)
        ids = self._search_batch(Q.cpu().tolist(), 1)
        rows = torch.as_tensor([g.row_of.get(r[0], -1) if r else -1 for r in ids], dtype=torch.long)
        return None, rows

    def _link_batch(self, rows: torch.Tensor, codes: np.ndarray, shard_hits, global_hits, now: float) -> int:
        """Chain + within-shard + cross-memory edges for the new rows
        (reference _link_within_shards :797-836, _link_to_existing :838-891).
        Returns the number of cross-conversation links (the reference's count)."""
        g = self.graph
        dev = g.device
        k = int(rows.numel())
        rows = rows.to(dev)
        ct = torch.as_tensor(codes, dtype=torch.int32).to(dev)
        es, ed, ew, eh = [], [], [], []
        # chain edges between consecutive new nodes of the same shard, in order
        order = np.argsort(codes, kind="stable")
        oc = codes[order]
        same = np.nonzero(oc[1:] == oc[:-1])[0]
        # the reference only links within shards that received >= 2 new nodes
        if same.size:
            a = torch.as_tensor(order[same], dtype=torch.long).to(dev)
            b = torch.as_tensor(order[same + 1], dtype=torch.long).to(dev)
            es.append(rows[a])
            ed.append(rows[b])
            ew.append(torch.full((a.numel(),), CHAIN_WEIGHT, device=dev))
            eh.append(ct[a])
        sw, sr = shard_hits
        src = rows[:, None].expand(-1, sr.shape[1])
        # within-shard similarity links only for shards with >= 2 new nodes (reference :814-815)
        multi = np.zeros(k, dtype=bool)
        uc, cnt = np.unique(codes, return_counts=True)
        multi_codes = set(uc[cnt >= 2].tolist())
        for i, c in enumerate(codes.tolist()):
            multi[i] = c in multi_codes
        mt = torch.as_tensor(multi).to(dev)
        mw = (sr >= 0) & (sw > LINK_THRESHOLD) & mt[:, None]
        es.append(src[mw])
        ed.append(sr[mw])
        ew.append((sw[mw] * LINK_WEIGHT_SCALE).float())
        eh.append(ct[:, None].expand_as(sr)[mw])
        gw, gr = global_hits
        mg = (gr >= 0) & (gw > LINK_THRESHOLD)
        # skip a cross-memory pair already linked within the shard (either direction)
        in_shard = ((gr[:, :, None] == sr[:, None, :]) & mw[:, None, :]).any(dim=2)
        mg = mg & ~in_shard
        srcg = rows[:, None].expand(-1, gr.shape[1])
        es.append(srcg[mg])
        ed.append(gr[mg])
        ew.append((gw[mg] * LINK_WEIGHT_SCALE).float())
        eh.append(ct[:, None].expand_as(gr)[mg])
        made = int(mg.sum())
        S, Dd = torch.cat(es), torch.cat(ed)
        if S.numel():
            # keep the reference's edge order: per new node, chain first, then
            # within-shard links, then cross-memory links
            g.append_edges(S, Dd, torch.cat(ew), torch.cat(eh), g.etype("relates_to"), now=now)
        return made

    # ------------------------------------------------------------ batched end_conversation
    def consolidate_batch(self, conversations: Sequence[Sequence[Dict]], embeddings=None,
                          now: float = None) -> Dict[str, int]:
        """``end_conversation`` for B finished conversations at once, given
        their extracted facts (``conversations[c]`` = fact dicts with
        ``content`` / ``type`` / ``salience`` / ``topic``, the extraction
        LLM's output, reference :684-716). ``embeddings``: optional [F, D]
        vectors aligned with the flattened facts (else the embedder runs once
        for the whole batch).

        Result = B sequential ``end_conversation`` calls (reference :580-649,
        :706-891) -- conversation c's facts dedupe against, and link to, the
        graph plus the facts kept from conversations < c; then decay
        (0.01 per conversation) and auto-prune -- computed in one device pass:

        * ONE fused scan of all facts against the pre-batch graph (dedupe
          top-1 + within-shard and cross-memory top-3), plus an F x F float64
          block for the facts of earlier conversations in the batch; in-batch
          duplicate chains are resolved by a fixed point;
        * decay is applied in closed form: the pre-batch graph by
          (1-r)^B in one ``tg_decay_kernel`` pass, a new node / edge of
          conversation c by (1-r)^(B-c) at insert (the decays of the
          end_conversation calls that follow it); a duplicate merge onto a
          node keeps max(decayed salience, decayed fact salience) -- exactly
          the sequential result, as decay is monotone;
        * eviction to ``max_buffer_size``, super-node creation, the
          ``run_consolidation`` trigger (once if any of the B counts crosses a
          multiple of ``consolidate_every``) and the persistence commit run
          once per batch instead of once per conversation.

        Returns counts: conversations, facts, dup, inserted, linked (edges
        created), cross_links (the reference's "cross-conversation links"),
        pruned (edges removed by decay, incl. new ones below the threshold),
        evicted."""
        flat, conv, idx = [], [], []
        j = 0
        for c, fs in enumerate(conversations):
            for f in fs:
                if isinstance(f, dict) and f.get("content") and len(f["content"]) >= MIN_FACT_LEN:
                    flat.append(f)
                    conv.append(c)
                    idx.append(j)
                j += 1
        B = len(conversations)
        now = time.time() if now is None else now
        stats = {"conversations": B, "facts": len(flat), "dup": 0, "inserted": 0, "linked": 0, "cross_links": 0,
                 "pruned": 0, "evicted": 0}
        if B == 0:
            return stats
        if embeddings is not None and len(flat):
            E = embeddings if torch.is_tensor(embeddings) else torch.as_tensor(np.asarray(embeddings, np.float32))
            embs = E[torch.as_tensor(idx, dtype=torch.long).to(E.device)] if len(idx) != len(E) else E
        elif flat:
            with tracer.stage("embed_facts", self._device):
                embs = self._batch_embed_any([f["content"] for f in flat])
        else:
            embs = None
        with self._graph_lock, tracer.stage("consolidate_batch", self._device):
            self._consolidate_batch(flat, np.asarray(conv, dtype=np.int64), B, embs, now, stats)
            self._enforce_buffer_limit_counted(stats)
            c0 = self.conversation_count
            self.conversation_count += B
            if self.auto_consolidate and (self.conversation_count // self.consolidate_every
                                          > c0 // self.consolidate_every):
                with tracer.stage("run_consolidation", self._device):
                    self.run_consolidation()
            self._maybe_cluster(c0)
            self._save_to_persistence()
        return stats

    def _maybe_cluster(self, c0: int) -> None:
        """hierarchy_mode="kmeans": re-cluster when the conversation count
        crosses a multiple of hierarchy_params["every"]."""
        if not self.enable_hierarchy or getattr(self, "hierarchy_mode", "reference") != "kmeans":
            return
        hp = self.hierarchy_params
        if self.conversation_count // hp["every"] > c0 // hp["every"] or getattr(self.graph, "hier", None) is None:
            with tracer.stage("cluster", self._device):
                self.graph.cluster_pass(hp["fine"], hp["top"], hp["iters"])

    def _enforce_buffer_limit_counted(self, stats: Dict[str, int]) -> None:
        g = self.graph
        if g.num_nodes() <= self.max_buffer_size:
            return
        with tracer.stage("evict", self._device):
            victims = g.evict(self.max_buffer_size)
        if victims:
            with tracer.stage("evict_store", "cpu"):
                self._store_delete([g.ids[r] for r in victims])
            stats["evicted"] += len(victims)

    def _consolidate_batch(self, facts: List[Dict], conv: np.ndarray, B: int, embs, now: float,
                           stats: Dict[str, int]) -> None:
        g = self.graph
        keep = 1.0 - DECAY_RATE
        thr = self.prune_threshold if self.auto_prune else None
        M = len(facts)
        if M:
            E, valid = self._fact_matrix(embs, M)
            rejected = M - int(valid.sum())
            if rejected:
                self.metrics["rejected_embeddings"] = self.metrics.get("rejected_embeddings", 0) + rejected
            vidx = np.nonzero(valid)[0]
            facts = [facts[i] for i in vidx]
            conv = conv[vidx]
            E = E[torch.as_tensor(vidx, dtype=torch.long).to(E.device)]
            M = len(facts)
        if M == 0:
            stats["pruned"] += g.decay(1.0 - keep ** B, thr)
            return
        dev = g.device
        # shards are created in fact order, duplicates included (reference :716-718)
        shard_keys = [f.get("topic", self._infer_shard_key(f["content"])) for f in facts]
        codes = np.asarray([g.shard_id(k) for k in shard_keys], dtype=np.int32)
        sal_in = torch.as_tensor([float(f.get("salience", 0.5)) for f in facts], dtype=torch.float64).to(dev)
        ct = torch.as_tensor(conv).to(dev)
        Q = E.to(dev, torch.float32)
        Qd = Q.double()
        qn = Qd.norm(dim=1, keepdim=True)
        Qn = Qd / torch.where(qn > 0, qn, torch.ones_like(qn))
        NEG = float("-inf")

        # ---- 1. one scan of the batch against the pre-batch graph
        if g.n:
            with g.on_stream(), tracer.stage("cb_scan", self._device):
                (gb_r, gb_s, gb_node), (gs, gr), (ws, wr) = self._scan_batch(Q, torch.as_tensor(codes))
        else:
            gb_r = torch.full((M,), -1, dtype=torch.long, device=dev)
            gb_s = torch.full((M,), NEG, dtype=torch.float64, device=dev)
            gb_node = torch.zeros(M, dtype=torch.bool, device=dev)
            gs = ws = torch.full((M, LINK_TOPK), NEG, dtype=torch.float64, device=dev)
            gr = wr = torch.full((M, LINK_TOPK), -1, dtype=torch.long, device=dev)

        # ---- 2. in-batch dedupe: the store top-1 over graph rows + the facts
        # kept from earlier conversations, to a fixed point
        with tracer.stage("cb_dedupe", self._device):
            S, earlier, dup, batch_best, bb_i, ins = batch_dedupe(Qn, ct, gb_s, gb_node)
        dup_graph = dup & ~batch_best
        dup_batch = dup & batch_best

        left = (B - ct).double()  # decays still to come for a fact of conversation c
        sal_dec = salience_decayed(sal_in, left, keep)

        # ---- 3. decay + prune the pre-batch graph by B conversations at once
        with tracer.stage("cb_decay", self._device):
            stats["pruned"] += g.decay(1.0 - keep ** B, thr)

        # ---- 4. duplicate merges (reference :736-740)
        ndup = int(dup.sum())
        stats["dup"] += ndup
        if bool(dup_graph.any()):
            rows = gb_r[dup_graph]
            with g.on_stream():
                g.sal.scatter_reduce_(0, rows, sal_dec[dup_graph].float(), "amax", include_self=True)
                g.last[rows] = now
                g.acc.index_add_(0, rows, torch.ones_like(rows, dtype=torch.int32))
                g.dirty[rows] = 1
            g._bump()
        sal_new = sal_dec.clone()
        acc_new = torch.zeros(M, dtype=torch.int32, device=dev)
        if bool(dup_batch.any()):
            tgt = bb_i[dup_batch]
            sal_new.scatter_reduce_(0, tgt, sal_dec[dup_batch], "amax", include_self=True)
            acc_new.index_add_(0, tgt, torch.ones_like(tgt, dtype=torch.int32))
        for _ in range(ndup):
            self._say("   (Merged semantic duplicate)")

        # ---- 5. insert the kept facts (conversation order) with pre-decayed salience
        kidx = torch.nonzero(ins).flatten()
        kh = kidx.cpu().numpy()
        if kh.size == 0:
            return
        kfacts = [facts[i] for i in kh]
        ids = [self._generate_node_id() for _ in kh]
        with tracer.stage("cb_insert", self._device):
            rows = g.add_nodes(ids, [f["content"] for f in kfacts], Q[kidx], shard=codes[kh],
                               types=[f.get("type", "semantic") for f in kfacts], sal=sal_new[kidx].float(),
                               acc=acc_new[kidx], now=now, stored=self._store_binds_graph())
        stats["inserted"] += int(kh.size)
        if not self._store_binds_graph():
            self.vector_store.add_nodes([
                {"id": i, "content": f["content"], "embedding": g.embedding(int(r)), "type": f.get("type", "semantic"),
                 "salience": float(f.get("salience", 0.5)), "shard_key": shard_keys[j], "timestamp": now}
                for i, f, r, j in zip(ids, kfacts, rows.tolist(), kh.tolist())], user_id=self.user_id)
        if self.query_cache:
            self.query_cache.invalidate_results()
        new_row = torch.full((M,), -1, dtype=torch.long, device=dev)
        new_row[kidx] = rows.to(dev)

        # ---- 6. links of the kept facts (reference :797-891), pre-decayed
        with tracer.stage("cb_link", self._device):
            self._link_batch_multi(kidx, new_row, codes, ct, S, earlier, (ws, wr), (gs, gr), keep, B, thr, now,
                                   stats)
        if self.enable_hierarchy and getattr(self, "hierarchy_mode", "reference") == "reference":
            for skey in dict.fromkeys(shard_keys[j] for j in kh.tolist()):
                c = g.shard_code.get(skey)
                if c is not None and g.shard_count[c] > self.super_node_threshold:
                    self._create_super_nodes_for_shard(skey)

    def _link_batch_multi(self, kidx, new_row, codes, ct, S, earlier, shard_hits, global_hits, keep, B, thr, now,
                          stats) -> None:
        g = self.graph
        plan, n_cross = batch_link_plan(kidx, new_row, torch.as_tensor(codes).to(g.device), ct, S, earlier,
                                        shard_hits, global_hits, keep, B, thr, stats)
        if n_cross:
            self._say(f"✓ Created {n_cross} cross-conversation links")
        if plan is not None:
            Sr, Dr, W, H = plan
            g.append_edges(Sr, Dr, W.float(), H.to(torch.int32), g.etype("relates_to"), now=now)

    # ------------------------------------------------------------ hierarchy (K8/K16)
    def _create_super_nodes_for_shard(self, shard_key: str):
        g = self.graph
        c = g.shard_code.get(shard_key)
        if c is None or g.shard_count[c] < self.super_node_threshold:
            return
        srows = g.node_rows_where(super_=True)
        if srows.size and (g.mirror("shard")[srows] == c).any():
            return
        rows = g.node_rows_where(c, super_=False)
        self._say(f"  Creating super-node for shard '{shard_key}' ({rows.size} nodes)")
        sid = f"super_{shard_key}_{int(time.time())}"
        summary = f"Topic: {shard_key}. Contains memories about: " + "; ".join(g.content[r] for r in rows[:3])
        rt = torch.as_tensor(rows, dtype=torch.long).to(g.device)
        mean = g.mean_embedding(rt)
        child_ids = [g.ids[r] for r in rows]
        srow = g.add_nodes([sid], [summary], (mean[None, :].float() if mean is not None else None),
                           shard=[c], sup=[1], children={0: child_ids}, stored=False)
        with g.on_stream():
            g.parent[rt] = srow.to(torch.int32)[0]
            g.dirty[rt] = 1
        g._bump()
        self._say(f"  ✓ Created super-node {sid} with {rows.size} children")

    # ------------------------------------------------------------ deep consolidation
    def run_consolidation(self, weight_threshold: float = 0.6, merge_similar: bool = True) -> str:
        results = []
        self._say("🔄 Running consolidation...")
        g = self.graph
        with self._graph_lock:
            if merge_similar:
                merged = self._merge_similar_nodes(similarity_threshold=DEDUPE_THRESHOLD)
                if merged > 0:
                    results.append(f"✓ Merged {merged} similar nodes")
            with tracer.stage("components", self._device):
                # components with >= 3 members and mean edge weight > 0.3
                # (reference :967-990), as their first 10 shard-node rows
                digest = g.component_digest(3, 0.3, PROFILE_CONTENTS)
            contents = [[g.content[r] for r in rows.tolist()] for rows in digest]
        updates = 0
        for cs in contents:
            r = self._extract_profile_from_contents(cs)
            if "Updated" in r:
                updates += 1
                results.append(r)
        with self._graph_lock:
            pruned = g.prune(self.prune_threshold)
        if pruned > 0:
            results.append(f"✓ Pruned {pruned} weak edges")
        if updates > 0:
            results.append(f"✓ Updated {updates} profile domains")
        else:
            with self._graph_lock:
                rows = g.first_node_rows_dev(PROFILE_CONTENTS, super_=False)
                contents = [g.content[r] for r in rows.tolist()]
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
        prompt = "Related memories:\n" + "\n".join(f"- {c}" for c in contents[:PROFILE_CONTENTS])
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
    def _similar_pairs(self, rows: np.ndarray, tau: float) -> List[Tuple[int, int]]:
        """Pairs (i < j, positions into ``rows``) with cosine > tau, sorted.
        GPU + unit rows: candidates from the MFMA all-pairs kernel at a
        lowered threshold (bf16 error margin), confirmed in float64."""
        g = self.graph
        m = rows.size
        if m < 2:
            return []
        rt = torch.as_tensor(rows, dtype=torch.long).to(g.device)
        with g.on_stream():
            X = g.emb32[rt].double()
            nrm = g.sqn[rt].double().sqrt()
            U = X / torch.where(nrm > 0, nrm, torch.ones_like(nrm))[:, None]
            if g._use_kernel(m) and m * m >= (1 << 20):
                from ..ops.graph_ops import pairs_above
                U16 = torch.zeros((m, g.Dp), dtype=torch.bfloat16, device=g.device)
                U16[:, : g.dim] = U.to(torch.bfloat16)
                cand = pairs_above(U16, tau - 0.02).long()
                if cand.numel() == 0:
                    return []
                cs = (U[cand[:, 0]] * U[cand[:, 1]]).sum(1)
                p = cand[cs > tau]
            else:
                S = U @ U.T
                iu = torch.triu_indices(m, m, 1, device=g.device)
                keep = S[iu[0], iu[1]] > tau
                p = torch.stack([iu[0][keep], iu[1][keep]], 1)
            if p.numel() == 0:
                return []
            o = torch.argsort(p[:, 0] * m + p[:, 1])
            return [tuple(x) for x in p[o].cpu().tolist()]

    def _merge_similar_nodes(self, similarity_threshold: float = DEDUPE_THRESHOLD) -> int:
        g = self.graph
        if g.num_nodes() < 2:
            return 0
        if self.merge_mode != "pairwise":
            # reference behaviour: the inner loop is dedented out of the outer
            # one (memory_system.py:1073-1077) so nothing is ever compared
            return 0
        # the intended semantics: for i < j in node order, merge j into i
        rows = g.ordered_node_rows()
        rows = rows[g.mirror("sup")[rows] == 0]
        pairs = self._similar_pairs(rows, similarity_threshold)
        if not pairs:
            return 0
        processed: Set[int] = set()
        merged = 0
        touched_store = []
        sal, acc = g.mirror("sal").copy(), g.mirror("acc").copy()
        for i, j in pairs:
            if i in processed or j in processed:
                continue
            r1, r2 = int(rows[i]), int(rows[j])
            g.content[r1] = f"{g.content[r1]} | {g.content[r2]}"
            sal[r1] = max(sal[r1], sal[r2])
            acc[r1] = acc[r1] + acc[r2]
            g.set_scalar(r1, "sal", float(sal[r1]))
            g.set_scalar(r1, "acc", int(acc[r1]))
            self._rewire(r2, r1)
            g.remove_nodes([r2], drop_edges=False, unstore=True)
            processed.add(j)
            merged += 1
            touched_store.append((g.ids[r2], g.ids[r1]))
        for id2, id1 in touched_store:
            self._store_delete([id2, id1])
            n1 = self.buffer.get_node(id1)
            if n1 is not None:
                self._store_add_rows([g.row_of[id1]], [{
                    "id": id1, "content": n1.content, "embedding": n1.embedding, "type": n1.type,
                    "salience": n1.salience, "shard_key": n1.shard_key, "timestamp": n1.timestamp}])
        return merged

    def _rewire(self, r_from: int, r_to: int) -> None:
        """Move the edges of ``r_from``'s shard that touch it onto ``r_to``; a
        moved edge whose new key already exists strengthens that edge
        (reference memory_system.py:1087-1104)."""
        g = self.graph
        sc = int(g.mirror("shard")[r_from])
        idx = g.edges_incident(r_from, sc)
        if idx.numel() == 0:
            return
        with g.on_stream():
            e = g.e
            s, d = e["src"][idx].clone(), e["dst"][idx].clone()
            w, co, lu, meta = e["w"][idx].clone(), e["co"][idx].clone(), e["lu"][idx].clone(), e["meta"][idx].clone()
        g.remove_edges(idx)
        s = torch.where(s == r_from, torch.full_like(s, r_to), s)
        d = torch.where(d == r_from, torch.full_like(d, r_to), d)
        g.upsert_edges(s, d, w, meta & SHARD_MASK, (meta >> 24) & TYPE_MASK, co=co, lu=lu)
