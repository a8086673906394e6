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
import math
import os
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


def decay_steps_f32(x: torch.Tensor, n: torch.Tensor, keep: float, salience: bool) -> torch.Tensor:
    """``x`` after ``n[i]`` end_conversation decays, each rounded to fp32 the
    way ``tg_decay_kernel`` rounds it (salience: floor + (s - floor) * keep
    op by op; edge weight: w * keep) -- B rounded steps, not one multiply by
    keep^B, so a value at the prune threshold lands exactly where B
    sequential calls put it."""
    x = x.float().clone()
    kf = torch.tensor(keep, dtype=torch.float32, device=x.device)
    fl = torch.tensor(SALIENCE_FLOOR_, dtype=torch.float32, device=x.device)
    n = n.to(x.device)
    for t in range(int(n.max()) if n.numel() else 0):
        d = torch.where(x > fl, fl + (x - fl) * kf, fl) if salience else x * kf
        x = torch.where(n > t, d, x)
    return x


def salience_decayed(s: torch.Tensor, n: torch.Tensor, keep: float) -> torch.Tensor:
    """Node salience (fp32) after ``n`` decays (floor SALIENCE_FLOOR_,
    memory_shard.py:64-77), rounded per step like the sequential calls."""
    return decay_steps_f32(s, n, keep, True)


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
    # decays of the end_conversation calls from the edge's conversation on,
    # rounded per step in fp32 like the sequential calls
    W = decay_steps_f32(W, B - torch.div(Ord, 4, rounding_mode="floor"), keep, False)
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


def _lowest_keys(imp: torch.Tensor, okey: torch.Tensor, P: int) -> torch.Tensor:
    """Rows of the P smallest (importance, shard, row) keys -- the eviction
    order: every row with a smaller importance than the P-th, then the tied
    rows by (shard, row)."""
    t = torch.topk(imp, P, largest=False, sorted=False).values.max()
    lt = torch.nonzero(imp < t).flatten()
    m = P - int(lt.numel())
    big = torch.iinfo(torch.int64).max
    tv, ti = torch.topk(torch.where(imp == t, okey, torch.full_like(okey, big)), m, largest=False, sorted=False)
    return torch.cat([lt, ti[tv != big]])


def _host_pinned(owner, attr: str, t: torch.Tensor) -> np.ndarray:
    """``t.cpu().numpy()`` through a pinned buffer cached on ``owner``
    (grown, never shrunk): the planner's F x F float64 block is 8 MB per
    1024-fact batch, which a pageable copy moved at a few GB/s. The array is
    valid until the next call with the same ``attr``."""
    if not t.is_cuda:
        return t.cpu().numpy()
    n = t.numel()
    buf = getattr(owner, attr, None)
    if buf is None or buf.numel() < n or buf.dtype != t.dtype:
        buf = torch.empty(max(n, 1), dtype=t.dtype, pin_memory=True)
        setattr(owner, attr, buf)
    h = buf[:n].view(t.shape)
    h.copy_(t)  # (synchronous: the caller reads it right away)
    return h.numpy()


def shard_keys_of(g: TenantGraph, code: int) -> str:
    """The shard name of a shard code."""
    for k, c in g.shard_code.items():
        if c == code:
            return k
    raise KeyError(code)


def _parse_json(response: str):
    if response is None:
        raise json.JSONDecodeError("empty", "", 0)
    if "```json" in response:
        response = response.split("```json")[1].split("```")[0].strip()
    return json.loads(response)


_PF_STREAMS: Dict = {}


def _prefetch_stream(dev):
    """One side stream per device for prefetched candidate scans, at high
    priority: HIP maps streams of one priority round-robin onto a few
    hardware queues, and a prefetched scan that shared the graph stream's
    queue would run in line with the apply it is meant to overlap."""
    st = _PF_STREAMS.get(dev)
    if st is None:
        st = _PF_STREAMS[dev] = torch.cuda.Stream(dev, priority=-1)
    return st


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

    def _fact_shard_key(self, f: Dict) -> str:
        """A fact's shard: its extracted topic, else the keyword inference
        (reference :716-718) -- evaluated only when there is no topic."""
        t = f.get("topic")
        return t if t is not None or "topic" in f else self._infer_shard_key(f["content"])

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
        shard_keys = [self._fact_shard_key(facts[i]) for i in vidx]
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
                # the store's top-1 is by L2: score 2|q||x|cos - |x|^2. The
                # global list's head is the L2-best unit row; super-nodes (means
                # of unit rows) are not unit, so every one is scored
                srows = torch.as_tensor(g.node_rows_where(super_=True), dtype=torch.long).to(dev)
                X = g.emb32[srows].double()
                n2 = g.sqn[srows].double()
                l2s = 2.0 * (Qd @ X.T) - n2[None, :]
                j = torch.argmax(l2s, dim=1)  # first maximum: the lowest super row on a tie
                sl2 = l2s.gather(1, j[:, None])[:, 0]
                sr = srows[j]
                hn2 = g.sqn[best_r.clamp_min(0)].double()
                hl2 = torch.where(best_r >= 0, 2.0 * qn[:, 0] * best_s * hn2.sqrt() - hn2,
                                  torch.full_like(best_s, float("-inf")))
                better = (sl2 > hl2) | ((sl2 == hl2) & (sr < best_r))
                nx = n2.sqrt()[j]
                scos = (Qn * X[j]).sum(1) / torch.where(nx > 0, nx, torch.ones_like(nx))
                best_s = torch.where(better, scos, best_s)
                best_r = torch.where(better, sr, best_r)
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
    # candidate list length per fact in the batch scan: 3 links + headroom for
    # rows the batch evicts before the fact's conversation (else: fallback)
    BATCH_LIST_K = 8

    def consolidate_batch(self, conversations: Sequence[Sequence[Dict]], embeddings=None,
                          now: float = None, cadence: str = "conversation", commit: str = "batch") -> Dict[str, int]:
        """``end_conversation`` for B finished conversations at once, given
        their extracted facts (``conversations[c]`` = fact dicts with
        ``content`` / ``type`` / ``salience`` / ``topic``, the extraction
        LLM's output, reference :684-716). ``embeddings``: optional [F, D]
        vectors aligned with the flattened facts (else the embedder runs once
        for the whole batch). ``now``: the clock of the whole batch.

        The result is B sequential ``end_conversation`` calls at the
        reference's cadence (reference :580-649, :651-933): per conversation
        dedupe against and links to the graph of that moment, insert,
        buffer-limit eviction, super-node creation, decay + auto-prune,
        eviction again; ``run_consolidation`` at every multiple of
        ``consolidate_every``. :mod:`.batch_plan` simulates the B
        conversations on the host from ONE fused scan of all facts against
        the pre-batch graph (eviction: an exact pool argument), and the plan
        is applied to the device graph in segments that end at the
        ``run_consolidation`` points, where run_consolidation runs on the
        real graph. ``commit="batch"`` (default): one persistence commit per
        batch (the store then holds the same rows / edges / profile as after
        the last call; a crash mid-batch loses the batch, not just the
        current conversation); ``commit="conversation"``: the plan closes a
        segment after every conversation and each is committed as it is
        applied -- the reference's save per ``end_conversation`` (reference
        :648, :785), at the cost of one commit per conversation.

        ``cadence="batch"``: the coarser batch semantics of the row-sharded
        buffer (``ShardedMemorySystem``): every conversation's facts are
        matched against the pre-batch graph plus earlier conversations'
        facts with closed-form decays, and eviction, super-node creation,
        ``run_consolidation`` (once, if a multiple of ``consolidate_every``
        was crossed) happen once at the end of the batch.

        Returns counts: conversations, facts, dup, inserted, linked (edges
        created), cross_links (the reference's "cross-conversation links"),
        pruned (edges removed by decay), evicted, consolidations (the
        run_consolidation calls), fallbacks (candidate lists recomputed)."""
        if cadence not in ("conversation", "batch"):
            raise ValueError("cadence must be 'conversation' or 'batch'")
        if commit not in ("conversation", "batch"):
            raise ValueError("commit must be 'conversation' or 'batch'")
        self._commit_each = commit == "conversation" and cadence == "conversation"
        self._batch_src = embeddings  # a prefetched scan is keyed by its batch's embeddings object
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
                 "pruned": 0, "evicted": 0, "consolidations": 0, "fallbacks": 0}
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
            conv = np.asarray(conv, dtype=np.int64)
            if cadence == "batch":
                self._consolidate_batch_coarse(flat, conv, B, embs, now, stats)
                self._enforce_buffer_limit_counted(stats)
                c0 = self.conversation_count
                self.conversation_count += B
                if self.auto_consolidate and (self.conversation_count // self.consolidate_every
                                              > c0 // self.consolidate_every):
                    stats["consolidations"] += 1
                    with tracer.stage("run_consolidation", self._device):
                        self.run_consolidation()
                self._maybe_cluster(c0)
            elif self._plannable():
                self._consolidate_planned(flat, conv, B, embs, now, stats)
            else:
                self._consolidate_stepwise(flat, conv, B, embs, now, stats)
            if self.query_cache:
                self.query_cache.invalidate_results()
            self._save_to_persistence()
        return stats

    def consolidate_stream(self, batches, cadence: str = "conversation", commit: str = "batch",
                           lookahead: int = 2):
        """:meth:`consolidate_batch` over a stream of batches, yielding each
        batch's counts. ``batches`` yields ``(conversations, embeddings)`` or
        ``(conversations, embeddings, now)``. The result is the sequential
        calls' exactly; what differs is when the work runs: batch i+1's
        candidate scan (the batch's one pass over the whole tenant) is
        launched on a side stream as soon as batch i is planned, and runs
        while batch i's plan is applied on the host and the graph stream;
        batch i+1 then completes it against the graph as batch i left it
        (TenantGraph.cos_topk_finish: rows that left re-scanned, rows that
        arrived re-ranked in). Items are drawn from ``batches`` ``lookahead``
        batches ahead (>= 1; the default 2 draws batch i+2 before batch i is
        applied): a generator that embeds its facts on the device then has
        batch i+1's embed queued a whole batch before the prefetch reads its
        validity, instead of waiting for it there."""
        from collections import deque
        it = iter(batches)
        ahead = deque()

        def fill():
            while len(ahead) < max(1, int(lookahead)):
                b = next(it, None)
                if b is None:
                    break
                ahead.append(b)
        fill()
        try:
            while ahead:
                cur = ahead.popleft()
                fill()
                self._prefetch_next = ahead[0] if ahead else None
                convs, embs = cur[0], cur[1]
                now = cur[2] if len(cur) > 2 else None
                yield self.consolidate_batch(convs, embeddings=embs, now=now, cadence=cadence, commit=commit)
        finally:
            self._prefetch_next = None
            self._prefetched = None

    _prefetch_next = None
    _prefetched = None
    # False: no prefetch past a batch that runs a k-means pass (A/B only,
    # bench/bench_consolidate.py --no-prefetch-under-cluster)
    PREFETCH_UNDER_CLUSTER = True

    def _launch_prefetch(self, new_rows: int, cluster: bool) -> None:
        """Batch i+1's dual candidate scan (see :meth:`consolidate_stream`),
        launched on a side stream once batch i's own candidate lists are
        known (before its plan when batch i's scan was itself prefetched, so
        the scan runs under batch i's planner, verification and apply).
        ``new_rows``: a bound of the rows batch i inserts (reserved now: no
        column moves under the scan). Skipped when the scan is not the kernel
        path. A k-means pass inside batch i (``cluster``) does not stop it:
        the pass only rewrites ``TenantGraph.hier``, which neither the scan
        nor :meth:`TenantGraph.cos_topk_finish` reads (rows, kinds and
        super-node flags are untouched), so batch i+1's scan runs under the
        pass too instead of after it."""
        nxt, self._prefetch_next = self._prefetch_next, None
        self._prefetched = None
        g = self.graph
        if nxt is None or not g.on_gpu or nxt[1] is None or (cluster and not self.PREFETCH_UNDER_CLUSTER):
            return
        convs, embs = nxt[0], nxt[1]
        flat, idx, j = [], [], 0
        for fs in convs:
            for f in fs:
                if isinstance(f, dict) and f.get("content") and len(f["content"]) >= MIN_FACT_LEN:
                    flat.append(f)
                    idx.append(j)
                j += 1
        M = len(flat)
        if M == 0 or not g.dual_prefetch_ok(M, self.BATCH_LIST_K):
            return
        E = embs if torch.is_tensor(embs) else torch.as_tensor(np.asarray(embs, np.float32))
        E = E[torch.as_tensor(idx, dtype=torch.long).to(E.device)] if len(idx) != len(E) else E
        E, valid = self._fact_matrix(E, M)
        vidx = np.nonzero(valid)[0]
        flat = [flat[i] for i in vidx]
        E = E[torch.as_tensor(vidx, dtype=torch.long).to(E.device)]
        # the shards of batch i+1 are registered now, in its fact order: the
        # codes batch i+1 will assign (batch i registers none while applied)
        codes = np.asarray([g.shard_id(self._fact_shard_key(f)) for f in flat],
                           dtype=np.int64)
        g.reserve(g.n + int(new_rows) + 16)  # no column moves under the scan
        n = g.n
        with g.on_stream():
            Q = E.to(g.device, torch.float32)
            mask = (g.kind[:n] == NODE) & (g.sup[:n] == 0)
            h = g.cos_topk_prefetch(Q, mask, torch.as_tensor(codes), LINK_THRESHOLD, _prefetch_stream(g.device))
        self._prefetched = {"src": embs, "codes": codes, "M": len(flat), "h": h}

    # the planned batch's k-means passes run in the background
    # (TenantGraph.cluster_pass(background=True)): the rest of the batch and
    # the next one are applied under them. False: in line (A/B,
    # bench/bench_consolidate.py --cluster-inline)
    CLUSTER_BACKGROUND = True

    def _maybe_cluster(self, c0: int, background: bool = False) -> None:
        """hierarchy_mode="kmeans": re-cluster when the conversation count
        crosses a multiple of hierarchy_params["every"]."""
        if not self.enable_hierarchy or getattr(self, "hierarchy_mode", "reference") != "kmeans":
            return
        hp = self.hierarchy_params
        if self.conversation_count // hp["every"] > c0 // hp["every"] or not self.graph.has_hier():
            with tracer.stage("cluster", self._device):
                self.graph.cluster_pass(hp["fine"], hp["top"], hp["iters"],
                                        background=background and self.CLUSTER_BACKGROUND)

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

    def _plannable(self) -> bool:
        """The host plan needs the graph-bound store (its search = the
        graph's stored node rows, L2) and a run_consolidation that leaves the
        graph as it is (the reference's no-op merge)."""
        return (self._store_binds_graph() and getattr(self.vector_store, "metric", "l2") == "l2"
                and self.merge_mode == "reference")

    def _consolidate_stepwise(self, facts, conv, B, embs, now, stats) -> None:
        """B end_conversation bodies one after another (third-party stores,
        merge_mode="pairwise"): the same code path as the sequential calls."""
        E = None
        if facts:
            E, valid = self._fact_matrix(embs, len(facts))
        for c in range(B):
            jj = [j for j in np.nonzero(conv == c)[0].tolist() if E is not None and valid[j]]
            n0 = self.graph.num_nodes()
            if jj:
                made = self._ingest_facts([facts[j] for j in jj], E[torch.as_tensor(jj, device=E.device)])
                stats["inserted"] += len(made)
                stats["dup"] += len(jj) - len(made)
            pruned = self.graph.decay(DECAY_RATE, self.prune_threshold if self.auto_prune else None)
            stats["pruned"] += pruned
            self._enforce_buffer_limit_counted(stats)
            self.conversation_count += 1
            if self.auto_consolidate and self.conversation_count % self.consolidate_every == 0:
                stats["consolidations"] += 1
                self.run_consolidation()
            self._maybe_cluster(self.conversation_count - 1)
            if self._commit_each:
                self._save_to_persistence()

    # False: the Python reference planner instead of the native one
    NATIVE_PLANNER = True

    def _consolidate_planned(self, facts, conv, B, embs, now, stats) -> None:
        # one switch to the graph's stream for the whole batch: the hundreds of
        # graph operations inside then run without a stream hop each
        with self.graph.on_stream():
            self._consolidate_planned_body(facts, conv, B, embs, now, stats)

    def _consolidate_planned_body(self, facts, conv, B, embs, now, stats) -> None:
        from .batch_plan import PoolTooSmall, plan
        g = self.graph
        M = len(facts)
        E = None
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
        # shards are created in fact order, duplicates included (reference :716-718)
        shard_keys = [self._fact_shard_key(f) for f in facts]
        codes = np.asarray([g.shard_id(k) for k in shard_keys], dtype=np.int64)
        sal_in = np.asarray([float(f.get("salience", 0.5)) for f in facts], dtype=np.float32)
        thr = self.prune_threshold if self.auto_prune else None
        hp = self.hierarchy_params if getattr(self, "hierarchy_mode", "") == "kmeans" else None
        cl_every = hp["every"] if (hp and self.enable_hierarchy) else 0
        # this batch's candidate scan, if it was prefetched (under the previous batch)
        pf, self._prefetched = self._prefetched, None
        if not (pf is not None and pf["src"] is getattr(self, "_batch_src", None) and pf["M"] == M
                and np.array_equal(pf["codes"], codes)):
            pf = None
        # a k-means pass inside this batch (the planner's cluster points), or
        # the first one at its end
        c0 = self.conversation_count
        cluster = bool(cl_every) and ((c0 + B) // cl_every > c0 // cl_every or not g.has_hier())
        # rows this batch can insert: its facts and at most one super-node per
        # shard it touches (a super-node is never evicted, so a shard gets one)
        new_rows = M + len(set(codes.tolist()))
        early = pf is not None and self._prefetch_next is not None
        if early:
            # batch i+1's scan starts now, on the side stream: it reads the
            # graph as it is before this batch's apply, as a launch after the
            # plan did (the plan does not change the graph) -- and runs under
            # the planner instead of only under the apply
            with tracer.stage("cb_prefetch", self._device):
                self._launch_prefetch(new_rows, cluster)
        with tracer.stage("cb_scan", self._device):
            inputs = self._plan_inputs(E, codes, B, M, pf)
        P = inputs.pop("P0")
        while True:
            pool, pool_mask = self._eviction_pool(B, P, now)
            kw = dict(ct=conv, code=codes, sal_in=sal_in, n0=g.n, node_count=g.num_nodes(),
                      shard_count=list(g.shard_count), super_codes=self._super_codes(),
                      pre_members=lambda c: np.asarray(g.node_rows_where(c, super_=False), np.int64),
                      max_buffer=self.max_buffer_size, super_threshold=self.super_node_threshold,
                      ref_hierarchy=bool(self.enable_hierarchy and getattr(self, "hierarchy_mode",
                                                                           "reference") == "reference"),
                      prune_thr=thr, keep=1.0 - DECAY_RATE, now=now, pool=pool, **self._plan_rows(inputs, pool),
                      **inputs)
            with tracer.stage("cb_plan", "cpu"):
                pl = plan(kw, B, self.conversation_count, self.auto_consolidate, self.consolidate_every, cl_every,
                          native=self.NATIVE_PLANNER, seg_each=self._commit_each)
            with tracer.stage("cb_verify", self._device):
                ok = pool_mask is None or self._verify_pool(pool_mask, pl["events"], now)
            if ok:
                break
            if P >= g.n:
                raise PoolTooSmall("eviction plan failed verification with every row in the pool")
            stats["pool_retries"] = stats.get("pool_retries", 0) + 1
            P = min(g.n, 4 * P)
        ps = pl["stats"]
        for k in ("dup", "inserted", "linked", "cross_links", "evicted", "fallbacks"):
            stats[k] += int(ps[k])
        stats["pruned"] += int(ps["pruned_new"])
        if self._prefetch_next is not None and not early:
            with tracer.stage("cb_prefetch", self._device):
                self._launch_prefetch(int(pl["stats"]["inserted"]) + len(pl["supers"]),
                                      any(seg["cluster"] for seg in pl["segments"]))
        fact_key = np.asarray(pl["fact_key"], np.int64)
        fact_of = {int(k): int(j) for j, k in enumerate(fact_key.tolist()) if k >= 0}
        id_of = {}
        count0 = self.conversation_count
        # run_consolidation's profile prompts wait for the end of the batch
        # (graph reads captured at each point, no host wait in the loop) unless
        # every conversation is committed on its own, or a super-node of the
        # batch could re-use a row id (its row's content would change)
        defer = not self._commit_each and self._supers_fresh(pl, now)
        pending = []
        # the components of every run_consolidation point of the batch from
        # one base labelling (TenantGraph.cc_begin): the plan names every
        # victim of the batch up front
        cc = False
        if any(seg["consolidate"] for seg in pl["segments"]):
            vic = [np.asarray(seg["victims"], np.int64).reshape(-1) for seg in pl["segments"]]
            with tracer.stage("cc_begin", self._device):
                cc = g.cc_begin(np.concatenate(vic) if vic else np.zeros(0, np.int64), self.prune_threshold,
                                1.0 - DECAY_RATE, B)
        try:
            self._apply_planned_segments(pl, fact_key, fact_of, facts, codes, E, id_of, thr, now, stats, count0,
                                         defer, pending, cc=cc)
        finally:
            if cc:
                g.cc_end()
        if pending:
            with tracer.stage("rc_deferred", "cpu"):
                for cap in pending:
                    self._rc_host(cap)
        if getattr(self, "hierarchy_mode", "") == "kmeans" and not g.has_hier():
            self._maybe_cluster(self.conversation_count - 1, background=True)

    # the segments of a plan through the native applier (csrc/kernels/apply.hip
    # via engine/native_apply.py) where eligible; False: the per-segment path
    NATIVE_APPLY = True

    def _native_apply_ok(self, pl: Dict, defer: bool, cc: bool, thr, E) -> bool:
        """The native applier covers the steady state of the reference
        cadence on the GPU: captures deferred (no per-point host read), no
        per-conversation commit, the decay's prune on (auto_prune), no
        incremental components (graphs whose edges fit the one-block digest,
        digest.hip dg_small_kernel, for the whole batch), an int8 or no
        low-precision copy, and every insert a fresh row in plan order."""
        from ..engine import native_apply as NA
        from ..engine import tenant_graph as TG
        g = self.graph
        if not (self.NATIVE_APPLY and g.on_gpu and defer and not self._commit_each and thr is not None
                and TG.SEG_END_KERNEL and TG.SET_ROWS_KERNEL and not g._digest_sorted and NA.available()):
            return False
        if g.emb8 is not None and g.emb8.dtype != torch.int8:
            return False
        if g.dim is None or g.dim > 1024 or (E is not None and not E.is_cuda) or PROFILE_CONTENTS > 64:
            return False
        from ..ops import tenant_ops as T
        app = sum(len(seg["edge_src"]) for seg in pl["segments"])
        n_end = g.n + sum(len(seg["ins_kind"]) for seg in pl["segments"])
        if cc:
            # the partitioned batch: every point takes the incremental digest
            # (TenantGraph.component_digest) -- the stable prefix alone keeps
            # the graph off the O(edges) local digest at every point
            c = g._cc
            ns = c.get("ns") if c is not None else None
            if ns is None or ns <= T.dg_small_max_edges() or 16 * ns <= n_end:
                return False
        elif g.num_edges + app > T.dg_small_max_edges():
            return False
        # every insert is the next fresh row, in plan order (the add_nodes bulk path)
        fact_key = np.asarray(pl["fact_key"], np.int64)
        n = g.n
        nid = self.node_counter
        for seg in pl["segments"]:
            kinds = np.asarray(seg["ins_kind"]).tolist()
            idx = np.asarray(seg["ins_idx"]).tolist()
            for k, j in zip(kinds, idx):
                key = int(fact_key[j]) if k == 0 else int(pl["supers"][j]["key"])
                if key != n:
                    return False
                n += 1
                if k == 0:
                    nid += 1
                    if f"node_{nid}" in g.row_of:
                        return False
        return True

    def _apply_planned_native(self, pl, fact_key, fact_of, facts, codes, E, id_of, thr, now, stats, count0,
                              pending) -> None:
        """:meth:`_apply_planned_segments` through ONE native call per run of
        segments (a run ends at a segment that runs a cluster pass): the
        device work of every segment is issued by csrc/kernels/apply.hip
        from one uploaded block, and the host bookkeeping is replayed here in
        segment order from its records (engine/native_apply.py)."""
        segs = pl["segments"]
        i = 0
        while i < len(segs):
            j = i
            while j < len(segs) - 1 and not segs[j]["cluster"]:
                j += 1
            self._native_run(segs[i:j + 1], pl["supers"], fact_key, fact_of, facts, codes, E, id_of, thr, now,
                             stats, count0, pending)
            i = j + 1

    def _native_run(self, segs, supers, fact_key, fact_of, facts, codes, E, id_of, thr, now, stats, count0,
                    pending) -> None:
        from ..engine.native_apply import SegmentProgram
        g = self.graph
        stored = self._store_binds_graph()
        # (the edge type is registered only by a segment that links, as append_edges_host does)
        etype = g.etype("relates_to") if any(len(seg["edge_src"]) for seg in segs) else 0
        # a prune threshold <= 0 prunes nothing: no keep flags (TenantGraph.segment_begin)
        prog = SegmentProgram(g, now, thr if thr is not None and thr > 0.0 else float("-inf"), 1.0 - DECAY_RATE,
                              etype, PROFILE_CONTENTS)
        n0 = g.n
        g.reserve(n0 + sum(len(seg["ins_kind"]) for seg in segs))  # no column moves under the native loop
        n = n0
        prog.n(n)
        host = []  # per segment: the inserts' host columns and the store deletes, replayed after the run
        with tracer.stage("ap_build", "cpu"):
            for seg in segs:
                ik = np.asarray(seg["ins_kind"])
                for key in sorted(fact_key[np.asarray(seg["ins_idx"], np.int64)[ik == 0]].tolist()):
                    id_of[key] = self._generate_node_id()
                prog.decay(int(seg["c1"]) - int(seg["c0"]) + 1)
                tr = np.asarray(seg["tch_rows"], np.int64)
                if tr.size:
                    prog.touch_rows(tr, seg["tch_sal"], seg["tch_acc"], seg["tch_last"])
                kinds = ik.tolist()
                idx = np.asarray(seg["ins_idx"]).tolist()
                isal = np.asarray(seg["ins_sal"], np.float32)
                iacc = np.asarray(seg["ins_acc"], np.int32)
                ilast = np.asarray(seg["ins_last"], np.float64)
                ins = []
                k = 0
                while k < len(kinds):
                    if kinds[k] == 0:
                        k2 = k
                        while k2 < len(kinds) and kinds[k2] == 0:
                            k2 += 1
                        js = idx[k:k2]
                        m = len(js)
                        sh = codes[js].astype(np.int32)
                        prog.insert_rows(n, m, {"sal": isal[k:k2], "acc": iacc[k:k2], "last": ilast[k:k2],
                                                "shard": sh}, stored)
                        prog.embeddings(js, n)
                        cnt = np.bincount(sh[sh >= 0], minlength=1)
                        for c in np.nonzero(cnt)[0].tolist():
                            prog.shard_delta(c, int(cnt[c]))
                        ins.append(("facts", [id_of[int(fact_key[j])] for j in js],
                                    [facts[j]["content"] for j in js],
                                    [facts[j].get("type", "semantic") for j in js], sh))
                        n += m
                        prog.n(n)
                        k = k2
                    else:
                        sp = supers[idx[k]]
                        children = np.asarray(sp["children"], np.int64).tolist()
                        skey = shard_keys_of(g, int(sp["code"]))
                        ch_ids = [id_of[r] if r in fact_of else g.ids[r] for r in children]
                        content = [facts[fact_of[r]]["content"] if r in fact_of else g.content[r]
                                   for r in children[:3]]
                        summary = f"Topic: {skey}. Contains memories about: " + "; ".join(content)
                        emb = self._plan_super_emb[tuple(children)]
                        prog.insert_rows(n, 1, {"sal": float(isal[k]), "acc": int(iacc[k]), "last": float(ilast[k]),
                                                "shard": int(sp["code"]), "sup": 1}, False)
                        prog.embeddings([prog.extra_embedding(emb)], n)
                        prog.set_parent(children, n)
                        ins.append(("super", f"super_{skey}_{int(now)}", summary, ch_ids, n))
                        n += 1
                        prog.n(n)
                        k += 1
                es = np.asarray(seg["edge_src"], np.int64)
                if es.size:
                    prog.append_edges(es, seg["edge_dst"], seg["edge_w"], seg["edge_code"])
                vic = np.asarray(seg["victims"], np.int64).tolist()
                prog.segment_end(sorted({r for r in vic if 0 <= r < n}))
                if seg["consolidate"]:
                    prog.point()
                host.append((ins, [g.ids[r] if r < n0 else None for r in vic], vic))
        with tracer.stage("ap_native", g.device):
            res = prog.run(g.shard_count, E, g._cc)
        # ---- host replay, segment by segment (TenantGraph.add_nodes / segment_end, _rc_device)
        p = 0
        gone = []  # the victims' ids, deleted from the store in one call (one commit covers the batch)
        for s, (seg, (ins, vid0, vic)) in enumerate(zip(segs, host)):
            steps = int(seg["c1"]) - int(seg["c0"]) + 1
            g.decay_log += steps * math.log1p(-DECAY_RATE)
            if g._cc is not None:
                g._cc["steps"] += steps
            g._bump(edges=True)
            for it in ins:
                if it[0] == "facts":
                    _, ids, contents, types, sh = it
                    m = len(ids)
                    r0 = g.n
                    g.ids.extend(ids)
                    g.content.extend(contents)
                    g.types.extend(types)
                    g.row_of.update(zip(ids, range(r0, r0 + m)))
                    g.n = r0 + m
                    g.n_sumsq += m
                    cnt = np.bincount(sh[sh >= 0], minlength=len(g.shard_count))
                    for c in np.nonzero(cnt)[0]:
                        g.shard_count[int(c)] += int(cnt[c])
                    if g.deleted_ids:
                        for x in ids:
                            g.deleted_ids.pop(x, None)
                    g.last_add_rows = range(r0, r0 + m)
                else:
                    _, sid, summary, ch_ids, r = it
                    g.ids.append(sid)
                    g.content.append(summary)
                    g.types.append("semantic")
                    g.row_of[sid] = r
                    g.n = r + 1
                    g.n_sumsq += 1
                    g.n_super += 1
                    g.children[r] = list(ch_ids)
                    if g.deleted_ids:
                        g.deleted_ids.pop(sid, None)
                    g.last_add_rows = [r]
                if not g._dv_acc_pending:
                    g._norm_dev_pending.append(g._dv_acc[0])
                    g._dv_acc_pending = True
                g._bump(store=True)
            stats["pruned"] += prog.finish_segment(res, s)
            gone += [x if x is not None else g.ids[r] for x, r in zip(vid0, vic)]
            self.conversation_count = count0 + int(seg["c1"]) + 1
            if seg["consolidate"]:
                stats["consolidations"] += 1
                self._say("🔄 Running consolidation...")
                dig, first = prog.captures(res, p)
                p += 1
                pending.append({"results": [], "digest": dig, "pruned": 0, "first": first})
            if seg["cluster"]:
                if gone:
                    self._store_delete(gone, graph_unstored=True)
                    gone = []
                self._maybe_cluster(self.conversation_count - 1, background=True)
        if gone:
            with tracer.stage("ap_store_delete", "cpu"):
                self._store_delete(gone, graph_unstored=True)
        if list(res["shard_count"][:len(g.shard_count)]) != list(g.shard_count):
            raise RuntimeError("native segment apply diverged from the host shard counts")

    def _apply_planned_segments(self, pl, fact_key, fact_of, facts, codes, E, id_of, thr, now, stats, count0,
                                defer, pending, cc=False) -> None:
        if self._native_apply_ok(pl, defer, cc, thr, E):
            return self._apply_planned_native(pl, fact_key, fact_of, facts, codes, E, id_of, thr, now, stats, count0,
                                              pending)
        for seg in pl["segments"]:
            # node ids as the segment's facts are inserted (keys grow segment by
            # segment): a per-segment commit persists the sequential counter
            ik = np.asarray(seg["ins_kind"])
            for key in sorted(fact_key[np.asarray(seg["ins_idx"], np.int64)[ik == 0]].tolist()):
                id_of[key] = self._generate_node_id()
            with tracer.stage("cb_apply", self._device):
                stats["pruned"] += self._apply_segment(seg, pl["supers"], fact_key, fact_of, facts, codes, E,
                                                       id_of, thr, now)
            self.conversation_count = count0 + int(seg["c1"]) + 1
            if seg["consolidate"]:
                stats["consolidations"] += 1
                with tracer.stage("run_consolidation", self._device):
                    if defer:
                        pending.append(self._rc_device(prune=not self.auto_prune))
                    else:
                        self.run_consolidation(prune=not self.auto_prune)
            if seg["cluster"]:
                self._maybe_cluster(self.conversation_count - 1, background=not self._commit_each)
            if self._commit_each:
                with tracer.stage("commit", "cpu"):
                    self._save_to_persistence()

    def _supers_fresh(self, pl: Dict, now: float) -> bool:
        """No super-node of the plan re-uses an id (the id is
        ``super_<shard>_<int(now)>``): a re-used id rewrites its row's content,
        which a deferred profile prompt of an earlier point would read."""
        g = self.graph
        seen = set()
        for sp in pl["supers"]:
            sid = f"super_{shard_keys_of(g, int(sp['code']))}_{int(now)}"
            if sid in seen or sid in g.row_of:
                return False
            seen.add(sid)
        return True

    def _super_codes(self) -> List[int]:
        g = self.graph
        srows = g.node_rows_where(super_=True)
        return sorted(set(g.mirror("shard")[srows].tolist())) if srows.size else []

    def _plan_inputs(self, E, codes: np.ndarray, B: int, M: int, pf: Dict = None) -> Dict:
        """One scan of the batch against the pre-batch graph + the F x F
        block: candidate lists, super-node cosines, the fallback and
        super-embedding callbacks of the planner."""
        g = self.graph
        n = g.n
        dev = g.device
        K = self.BATCH_LIST_K
        NEGF = float("-inf")
        if M:
            Q = E.to(dev, torch.float32)
            Qd = Q.double()
            qn = Qd.norm(dim=1, keepdim=True)
            Qn = Qd / torch.where(qn > 0, qn, torch.ones_like(qn))
        else:
            Q = Qn = torch.zeros((0, g.dim or 1), dtype=torch.float64, device=dev)
        link_mask = (g.kind[:n] == NODE) & (g.sup[:n] == 0) if n else None
        if n and M and pf is not None:  # batch i+1's scan ran under batch i's apply
            with g.on_stream(), tracer.stage("cb_prefetch_finish", dev):
                (gs, gr), (ws, wr) = g.cos_topk_finish(pf["h"], K, link_mask)
        elif n and M:
            with g.on_stream():
                (gs, gr), (ws, wr) = g.cos_topk(Q, K, link_mask, dual_label=torch.as_tensor(codes),
                                                min_score=LINK_THRESHOLD)
        else:
            gs = ws = torch.full((M, K), NEGF, dtype=torch.float64)
            gr = wr = torch.full((M, K), -1, dtype=torch.long)
        # stored super-nodes: the store top-1 compares them by L2 (they are not unit rows)
        srows = g.node_rows_where(super_=True) if n else np.zeros(0, np.int64)
        if srows.size and M:
            with g.on_stream():
                st = torch.as_tensor(srows, dtype=torch.long).to(dev)
                X = g.emb32[st].double()
                nrm = g.sqn[st].double().sqrt()
                sup_cos = ((Qn @ X.T) / torch.where(nrm > 0, nrm, torch.ones_like(nrm))[None, :]).cpu().numpy()
                sup_n2 = g.sqn[st].double().cpu().numpy()
        else:
            sup_cos, sup_n2 = np.zeros((M, 0)), np.zeros(0)
        # fact x fact cosine with the scan's formula (rows stored as fp32, |x|^2 rounded to fp32)
        if M:
            X = Q.double()
            nrm = (X * X).sum(1).float().double().sqrt()
            S = _host_pinned(self, "_pin_S", (Qn @ X.T) / torch.where(nrm > 0, nrm, torch.ones_like(nrm))[None, :])
            qnorm = qn.flatten().cpu().numpy()
            fact_n2 = (X * X).sum(1).float().double().cpu().numpy()
        else:
            S, qnorm, fact_n2 = np.zeros((0, 0)), np.zeros(0), np.zeros(0)

        def fallback(j, evicted, same_shard):
            m = link_mask.clone()
            if evicted.size:
                m[torch.as_tensor(evicted, dtype=torch.long).to(dev)] = False
            with g.on_stream():
                if same_shard:
                    s_, r_ = g._exact_cos(Qn[j:j + 1], m, K, row_label=g.shard[:n],
                                          q_label=torch.as_tensor(codes[j:j + 1]).to(dev))
                else:
                    s_, r_ = g._exact_cos(Qn[j:j + 1], m, K)
            return s_[0].cpu().numpy(), r_[0].cpu().numpy()

        n0 = n

        def super_cos(children, new_facts):
            """Cosine of every fact against the mean embedding of ``children``
            (pre-batch rows, then batch rows = facts ``new_facts``: the row
            order the graph's mean_embedding reads), as the dedupe scan of a
            stored super-node. Returns (cos [M], |e|^2 of the fp32 row)."""
            ch = np.asarray(children, dtype=np.int64)
            nf = np.asarray(new_facts, dtype=np.int64)
            parts = []
            pre = ch[ch < n0]
            if pre.size:
                parts.append(g.emb32[torch.as_tensor(pre, dtype=torch.long).to(dev)])
            if nf.size:
                parts.append(Q[torch.as_tensor(nf, dtype=torch.long, device=dev)])
            if not parts:
                return np.full(M, NEGF), 1.0
            e = torch.cat(parts).double().mean(0).float()
            self._plan_super_emb[tuple(ch.tolist())] = e
            ed = e.double()
            n2 = float((ed * ed).sum().float())
            en = n2 ** 0.5
            return (((Qn @ ed) / (en if en > 0 else 1.0)).cpu().numpy() if M else np.zeros(0)), n2

        self._plan_super_emb = {}
        excess0 = max(0, g.num_nodes() - self.max_buffer_size)
        return {"glob": (gs.cpu().numpy(), gr.cpu().numpy()), "shard": (ws.cpu().numpy(), wr.cpu().numpy()),
                "sup_rows": srows, "sup_cos": sup_cos, "sup_n2": sup_n2, "qnorm": qnorm, "fact_n2": fact_n2, "S": S,
                "super_cos": super_cos, "fallback": fallback, "P0": min(n, 4 * (M + excess0) + 1024)}

    # the eviction pool's sampled thresholds (GPU, large tenants): row sample
    # stride and the pool size they aim for, in multiples of P (0: the exact
    # P lowest rows by four top-k selections)
    POOL_SAMPLE_STRIDE = 64
    POOL_OVERSAMPLE = 2.0
    POOL_MAX_OVER = 8

    def _eviction_pool(self, B: int, P: int, now: float):
        """The eviction pool of a batch plan: the P lowest-importance
        evictable rows now and after all B decays (ties in any order: the
        plan is verified against every other row afterwards,
        :meth:`_verify_pool`) -- on a large GPU tenant a sampled superset of
        them (POOL_SAMPLE_STRIDE). Returns (rows, device mask) -- mask None
        when the pool is every evictable row (nothing to verify)."""
        from ..ops import tenant_ops as T
        g = self.graph
        n = g.n
        if n == 0:
            return np.zeros(0, np.int64), None
        with g.on_stream():
            imp0 = T.importance(g.sal[:n], g.acc[:n], g.last[:n], g.kind[:n], g.sup[:n], now)
            nev = int(torch.isfinite(imp0).sum())
            if P >= nev:
                return torch.nonzero(torch.isfinite(imp0)).flatten().cpu().numpy(), None
            sal = g.sal[:n].clone()
            empty = {"src": torch.zeros(0, dtype=torch.int32, device=g.device),
                     "dst": torch.zeros(0, dtype=torch.int32, device=g.device),
                     "w": torch.zeros(0, dtype=torch.float32, device=g.device)}
            T.decay_prune(empty, sal, g.kind[:n], g.sup[:n], DECAY_RATE, None, steps=B)
            impB = T.importance(sal, g.acc[:n], g.last[:n], g.kind[:n], g.sup[:n], now)
            S = self.POOL_SAMPLE_STRIDE
            if g.on_gpu and S and n >= 64 * S and 4 * P < nev:
                # a superset of the P lowest rows of each importance: every
                # row at or under a threshold set from a 1/S row sample for
                # ~POOL_OVERSAMPLE x P rows (one pass, two host reads instead
                # of four top-k selections over the tenant); _verify_pool
                # checks the plan against every row outside it either way
                k = int(self.POOL_OVERSAMPLE * P / S) + 16
                fin = torch.isfinite(imp0)  # (evictable rows; the same rows are finite in impB)
                okey = g.shard[:n].long() * (1 << 32) + torch.arange(n, device=g.device)
                big = torch.iinfo(torch.int64).max
                sel, ok = [], True
                for imp in (imp0, impB):
                    sm, so = imp[::S], okey[::S]
                    kk = min(k, int(sm.numel()))
                    # the sample's kk-th smallest (importance, shard, row) key: the
                    # importance t by a top-k (not kthvalue: ATen's kthvalue sorts --
                    # 1.4 ms per call here), then the tied sample rows' keys -- a
                    # threshold inside a long run of equal importances (every row
                    # of a freshly loaded tenant) splits the run by key instead of
                    # pooling all of it
                    t = torch.topk(sm, kk, largest=False, sorted=False)[0].max()
                    j = (kk - (sm < t).sum()).clamp_min(1)
                    tied = torch.sort(torch.where(sm == t, so, torch.full_like(so, big))).values
                    to = tied[(j - 1).clamp_max(tied.numel() - 1)]
                    sel.append((imp < t) | ((imp == t) & (okey <= to)))
                cnt = torch.stack([(sel[0] & fin).sum(), (sel[1] & fin).sum()]).cpu().tolist()
                # (a threshold inside a large run of equal importances would
                # pool the whole run: the exact selection then)
                if min(cnt) >= P and max(cnt) <= self.POOL_MAX_OVER * P:
                    mask = ((sel[0] | sel[1]) & fin).to(torch.uint8)
                    return torch.nonzero(mask).flatten().cpu().numpy(), mask
            okey = g.shard[:n].long() * (1 << 32) + torch.arange(n, device=g.device)
            mask = torch.zeros(n, dtype=torch.uint8, device=g.device)
            for imp in (imp0, impB):
                mask[_lowest_keys(imp, okey, P)] = 1
            return torch.nonzero(mask).flatten().cpu().numpy(), mask

    def _verify_pool(self, pool_mask: torch.Tensor, events, now: float) -> bool:
        from ..ops import tenant_ops as T
        g = self.graph
        n = g.n
        with g.on_stream():
            return T.evict_verify(g.sal[:n], g.acc[:n], g.last[:n], g.kind[:n], g.sup[:n], g.shard[:n], pool_mask,
                                  now, 1.0 - DECAY_RATE, events)

    def _plan_rows(self, inputs: Dict, pool: np.ndarray) -> Dict:
        """Host state (sal, acc, last, shard, super) of every pre-batch row the
        batch can touch: the pool, the candidate-list rows, the super-nodes."""
        g = self.graph
        gr, wr = inputs["glob"][1], inputs["shard"][1]
        rows = np.unique(np.concatenate([pool.astype(np.int64), gr[gr >= 0].astype(np.int64),
                                         wr[wr >= 0].astype(np.int64),
                                         np.asarray(inputs["sup_rows"], np.int64)]))
        if rows.size:
            with g.on_stream():
                rt = torch.as_tensor(rows, dtype=torch.long).to(g.device)
                # one float64 block, one device read (every column is exact in float64)
                a = torch.stack([g.sal[rt].double(), g.acc[rt].double(), g.last[rt], g.shard[rt].double(),
                                 (g.sup[rt] != 0).double(), g.sqn[rt].double()]).cpu().numpy()
                cols = (a[0].astype(np.float32), a[1].astype(np.int64), a[2].copy(), a[3].astype(np.int64),
                        a[4] != 0, a[5].copy())
        else:
            cols = (np.zeros(0, np.float32), np.zeros(0, np.int64), np.zeros(0), np.zeros(0, np.int64),
                    np.zeros(0, bool), np.zeros(0))
        return {"rows": rows, "cols": cols}

    def _apply_segment(self, seg: Dict, supers: List[Dict], fact_key: np.ndarray, fact_of: Dict[int, int],
                       facts, codes: np.ndarray, E, id_of, thr, now) -> int:
        """Apply conversations [c0, c1] of a plan to the device graph: B-step
        decay + prune of what existed before, the touched rows' state, the
        inserts (facts and super-nodes, in row order), the new edges, the
        victims. Returns the edges pruned by the decay."""
        from ..ops import tenant_ops as T
        g = self.graph
        dev = g.device
        steps = int(seg["c1"]) - int(seg["c0"]) + 1
        with tracer.stage("ap_decay", dev):
            tok = g.segment_begin(DECAY_RATE, thr, steps)  # the prune lands in segment_end, with the victims
        tr = np.asarray(seg["tch_rows"], np.int64)
        if tr.size:
            with g.on_stream():
                if g.on_gpu:  # one pinned block, one launch (tenant.hip tg_set_rows_kernel)
                    m = int(tr.size)
                    blk = torch.empty(7 + 4 * m, dtype=torch.float64).pin_memory()
                    bn = blk.numpy()
                    bn[:7] = 0.0
                    for j, c in enumerate((tr, seg["tch_sal"], seg["tch_acc"], seg["tch_last"])):
                        bn[7 + j * m: 7 + (j + 1) * m] = np.asarray(c, dtype=np.float64).reshape(-1)
                    # per-row sal / acc / last; ts, shard, sup, parent, kind, stored untouched
                    T.set_rows(g, None, blk.to(dev, non_blocking=True), 0b111 | (0b1111000 << 8), -1, -1, m=m)
                else:
                    r64, s64, a64, l64 = T.to_dev_packed([tr, seg["tch_sal"], seg["tch_acc"], seg["tch_last"]], dev)
                    rt = r64.long()
                    g.sal[rt] = s64.float()
                    g.acc[rt] = a64.int()
                    g.last[rt] = l64
                    g.dirty[rt] = 1
            g._bump()
        stored = self._store_binds_graph()
        kinds = np.asarray(seg["ins_kind"]).tolist()
        idx = np.asarray(seg["ins_idx"]).tolist()
        isal = np.asarray(seg["ins_sal"], np.float32)
        iacc = np.asarray(seg["ins_acc"], np.int32)
        ilast = np.asarray(seg["ins_last"], np.float64)
        i = 0
        with tracer.stage("ap_insert", dev):
            while i < len(kinds):
                if kinds[i] == 0:
                    k = i
                    while k < len(kinds) and kinds[k] == 0:
                        k += 1
                    js = idx[i:k]
                    keys = fact_key[js].tolist()
                    g.add_nodes([id_of[key] for key in keys], [facts[j]["content"] for j in js],
                                       E[torch.as_tensor(js, dtype=torch.long).to(E.device)],
                                       shard=codes[js].astype(np.int32),
                                       types=[facts[j].get("type", "semantic") for j in js],
                                       sal=torch.from_numpy(isal[i:k]), acc=torch.from_numpy(iacc[i:k]),
                                       last=torch.from_numpy(ilast[i:k]), now=now, stored=stored, want_rows=False)
                    if list(g.last_add_rows) != keys:  # host rows: no device round trip
                        raise RuntimeError("batch plan row assignment diverged from the graph")
                    i = k
                else:
                    sp = supers[idx[i]]
                    children = np.asarray(sp["children"], np.int64).tolist()
                    skey = shard_keys_of(g, int(sp["code"]))
                    ch_ids = [id_of[r] if r in fact_of else g.ids[r] for r in children]
                    content = [facts[fact_of[r]]["content"] if r in fact_of else g.content[r] for r in children[:3]]
                    summary = f"Topic: {skey}. Contains memories about: " + "; ".join(content)
                    emb = self._plan_super_emb[tuple(children)]
                    srow = g.add_nodes([f"super_{skey}_{int(now)}"], [summary], emb[None, :], shard=[int(sp["code"])],
                                       sup=[1], children={0: ch_ids}, stored=False, sal=float(isal[i]),
                                       acc=int(iacc[i]), last=float(ilast[i]), now=now)
                    if int(g.last_add_rows[0]) != int(sp["key"]):
                        raise RuntimeError("batch plan super-node row diverged from the graph")
                    with g.on_stream():
                        rt = torch.as_tensor(children, dtype=torch.long).to(dev)
                        g.parent[rt] = srow.to(torch.int32)[0]
                        g.dirty[rt] = 1
                    g._bump()
                    i += 1
        es = np.asarray(seg["edge_src"], np.int64)
        if es.size:
            with tracer.stage("ap_edges", dev):
                g.append_edges_host(es, seg["edge_dst"], seg["edge_w"], seg["edge_code"], g.etype("relates_to"),
                                    now=now)
        vic = np.asarray(seg["victims"], np.int64).tolist()
        ids = [g.ids[r] for r in vic]
        with tracer.stage("ap_remove", dev):
            pruned = g.segment_end(tok, vic, unstore=True)
        if ids:
            with tracer.stage("ap_store_delete", "cpu"):
                self._store_delete(ids, graph_unstored=True)
        return pruned

    def _consolidate_batch_coarse(self, facts: List[Dict], conv: np.ndarray, B: int, embs, now: float,
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
            stats["pruned"] += g.decay(DECAY_RATE, thr, steps=B)
            return
        dev = g.device
        # shards are created in fact order, duplicates included (reference :716-718)
        shard_keys = [self._fact_shard_key(f) for f in facts]
        codes = np.asarray([g.shard_id(k) for k in shard_keys], dtype=np.int32)
        sal_in = torch.as_tensor([float(f.get("salience", 0.5)) for f in facts], dtype=torch.float32).to(dev)
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
            stats["pruned"] += g.decay(DECAY_RATE, thr, steps=B)

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

    @staticmethod
    def _fact_of_key(pl, key: int) -> int:
        return int(np.nonzero(pl.fact_key == key)[0][0])

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
    def run_consolidation(self, weight_threshold: float = 0.6, merge_similar: bool = True,
                          prune: bool = True) -> str:
        """Reference memory_system.py:951-1010. ``prune=False``: the caller
        guarantees no edge is below the prune threshold -- consolidate_batch,
        whose segment just pruned every decayed old edge (segment_end) and
        whose planner drops new links at each decay (batch_plan end_decay);
        weights only fall by decay, so the reference's prune here finds
        nothing. The graph work (:meth:`_rc_device`) and the profile prompts
        it feeds (:meth:`_rc_host`) are split so that consolidate_batch can
        read the graph at every consolidation point without waiting for the
        device and run the prompts, in order, at the end of the batch."""
        return self._rc_host(self._rc_device(merge_similar, prune))

    def _rc_device(self, merge_similar: bool = True, prune: bool = True) -> Dict:
        """The graph side of run_consolidation at this moment: merge (a no-op
        in the reference's merge mode), the component digest, the prune and
        the first shard rows -- the latter two as captures (the rows are read
        on the host in :meth:`_rc_host`). The first rows do not depend on the
        edges, so reading them after the prune matches the reference, which
        reads them after its profile prompts and prune (:1003-1008)."""
        results = []
        self._say("🔄 Running consolidation...")
        g = self.graph
        with self._graph_lock:
            if merge_similar:
                with tracer.stage("rc_merge", self._device):
                    merged = self._merge_similar_nodes(similarity_threshold=DEDUPE_THRESHOLD)
                if merged > 0:
                    results.append(f"✓ Merged {merged} similar nodes")
            with tracer.stage("components", self._device):
                # components with >= 3 members and mean edge weight > 0.3
                # (reference :967-990), as their first 10 shard-node rows
                digest = g.digest_capture(3, 0.3, PROFILE_CONTENTS)
            pruned = 0
            if prune:
                with tracer.stage("rc_prune", self._device):
                    pruned = g.prune(self.prune_threshold)
            with tracer.stage("rc_first_rows", self._device):
                first = g.first_rows_capture(PROFILE_CONTENTS)
        return {"results": results, "digest": digest, "pruned": pruned, "first": first}

    def _rc_host(self, cap: Dict) -> str:
        """The profile prompts of one :meth:`_rc_device` capture."""
        results = cap["results"]
        g = self.graph
        updates = 0
        with tracer.stage("rc_profile", "cpu"):
            for rows in cap["digest"].get():
                r = self._extract_profile_from_contents([g.content[x] for x in rows.tolist()])
                if "Updated" in r:
                    updates += 1
                    results.append(r)
        if cap["pruned"] > 0:
            results.append(f"✓ Pruned {cap['pruned']} weak edges")
        if updates > 0:
            results.append(f"✓ Updated {updates} profile domains")
        else:
            contents = [g.content[r] for r in cap["first"].get().tolist()]
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
