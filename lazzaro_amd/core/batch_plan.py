"""Exact plan of B sequential ``end_conversation`` calls (reference
memory_system.py:580-649 with :651-933) for ``MemorySystem.consolidate_batch``.

The batch keeps the reference's per-conversation cadence exactly: facts of
conversation c dedupe against / link to the graph as it stands after
conversation c-1 (evicted nodes gone, earlier facts present), every
conversation ends with its own decay + prune and buffer-limit eviction,
super-nodes appear at the conversation whose insert pushes a shard past the
threshold, and ``run_consolidation`` runs at every multiple of
``consolidate_every`` on the graph of that moment.

How, without B passes over a 10M-row tenant:

* ONE fused scan of all facts against the pre-batch graph gives each fact a
  short candidate list (top ``K`` global and same-shard rows, exact float64
  cosine). The graph only loses pre-batch rows during a batch, so the best
  rows still present are the first list entries not evicted yet; a list that
  runs short while its last entry is still above the link threshold is
  recomputed exactly (``fallback``, counted in the stats).
* Facts of earlier conversations are candidates through an F x F cosine block
  computed with the scan's formula (the same float64 values).
* Eviction removes the lowest-importance nodes (importance, then shard and
  row). The planner scores only a pool -- the ``P`` lowest pre-batch rows by
  importance before the batch and after all B decays -- plus the batch's own
  nodes, as ``tg_importance_kernel`` does (the same IEEE float64 operations,
  no contraction). Every eviction records its last victim's key; afterwards
  ``tg_evict_verify_kernel`` walks every row outside the pool through the
  same decays and checks none would have ranked before those victims (a row
  a merge touched only gains importance). If one would, the pool was too
  small and the caller plans again with a larger one.
* Salience and edge weights follow the decay kernel's fp32 operations:
  ``floor + (s - floor) * keep`` op by op, ``w *= keep``, once per
  conversation.

The plan is applied to the device graph in segments that end at the
``run_consolidation`` points and the k-means cluster points, so
``run_consolidation`` runs unmodified on the real graph of that moment.
"""
from __future__ import annotations

import json
import os
from dataclasses import dataclass, field
from typing import Callable, Dict, List, Optional, Sequence, Tuple

import numpy as np

F32 = np.float32
SAL_FLOOR = F32(0.2)
_plan_calls = 0
NEG = float("-inf")


def decay_sal_np(s: np.ndarray, keep) -> np.ndarray:
    """One tg_decay_kernel salience round (``decay_sal``, no contraction)."""
    s = np.asarray(s, dtype=F32)
    return np.where(s > SAL_FLOOR, SAL_FLOOR + (s - SAL_FLOOR) * F32(keep), SAL_FLOOR).astype(F32)


def importance_np(sal: np.ndarray, acc: np.ndarray, last: np.ndarray, now: float) -> np.ndarray:
    """``tg_importance_kernel`` in numpy float64 (the same operations, in
    order; reference memory_system.py:541-549)."""
    days = (np.float64(now) - last.astype(np.float64)) / 86400.0
    return (sal.astype(np.float64) * 0.5 + np.minimum(1.0, acc.astype(np.float64) / 10.0) * 0.3
            + (1.0 / (1.0 + days)) * 0.2)


class PoolTooSmall(Exception):
    """A row outside the eviction pool would have been a victim: plan again
    with a larger pool."""


@dataclass
class Super:
    code: int
    key: int               # the graph row it gets
    children: List[int]    # child rows, shard order
    conv: int
    cos: np.ndarray        # cosine of every fact against its embedding
    n2: float              # |embedding|^2 of the stored fp32 row


@dataclass
class Segment:
    """Conversations [c0, c1], applied to the device graph in one go."""
    c0: int
    c1: int
    inserts: List[Tuple[str, int]] = field(default_factory=list)    # ("fact", j) / ("super", s), row order
    edges: List[int] = field(default_factory=list)                   # batch edge ids created here, alive at c1
    victims: List[int] = field(default_factory=list)                 # rows evicted in [c0, c1]
    touched: Dict[int, Tuple[float, int, float]] = field(default_factory=dict)  # earlier row -> (sal, acc, last)
    new_state: Dict[int, Tuple[float, int, float]] = field(default_factory=dict)  # row inserted here -> state
    edge_w: np.ndarray = None                                        # their weights at c1
    consolidate: bool = False
    cluster: bool = False


class BatchPlanner:
    """Host simulation of B end_conversation calls (numpy inputs).

    Facts (valid, in conversation order): ``ct`` conversation, ``code`` shard
    code, ``sal_in`` fp32 salience. Pre-batch graph: ``n0`` rows,
    ``node_count`` (super-nodes included), ``shard_count`` per code,
    ``super_codes`` (shards that have a super-node), ``pre_members(code)`` its
    live shard rows in row order. Lists: ``glob`` / ``shard`` = (cos, row)
    [M, K] over live non-super node rows, sorted (cos desc, row asc);
    ``sup_rows`` / ``sup_cos`` [M, S] the stored super-nodes. ``S`` fact x
    fact cosine [M, M]. ``rows`` / ``cols``: (sal fp32, acc, last, code, super)
    of every pre-batch row the batch can touch; ``pool`` the eviction pool
    rows (checked afterwards against every other row, see :attr:`events`)."""

    def __init__(self, *, ct, code, sal_in, n0, node_count, shard_count, super_codes, pre_members, max_buffer,
                 super_threshold, ref_hierarchy, prune_thr, keep, now, glob, shard, sup_rows, sup_cos, sup_n2, S,
                 qnorm, fact_n2, rows, cols, pool, super_cos: Callable, fallback: Callable, dedupe_thr=0.95,
                 link_thr=0.5, link_k=3, link_scale=0.8, chain_w=0.5):
        self.ct = np.asarray(ct, np.int64)
        self.code = np.asarray(code, np.int64)
        self.sal_in = np.asarray(sal_in, F32)
        self.M = len(self.ct)
        self.n0 = int(n0)
        self.node_count = int(node_count)
        self.shard_count = [int(x) for x in shard_count]
        self.super_codes = set(int(x) for x in super_codes)
        self.pre_members = pre_members
        self.max_buffer, self.sthr, self.ref_h = int(max_buffer), super_threshold, ref_hierarchy
        self.thr = None if prune_thr is None else F32(prune_thr)
        self.keep, self.now = F32(keep), float(now)
        self.gs, self.gr = glob
        self.ss, self.sr = shard
        self.K = self.gs.shape[1]
        self.sup_rows, self.sup_cos = list(int(r) for r in sup_rows), sup_cos
        self.sup_n2 = np.asarray(sup_n2, np.float64)
        self.S = S
        self.qnorm = np.asarray(qnorm, np.float64)
        self.fact_n2 = np.asarray(fact_n2, np.float64)
        self.super_cos, self.fallback = super_cos, fallback
        self.dedupe_thr, self.link_thr, self.link_k = dedupe_thr, link_thr, link_k
        self.link_scale, self.chain_w = link_scale, F32(chain_w)
        # (decays so far, importance, shard, row) of each eviction's last victim
        self.events: List[Tuple[int, float, int, int]] = []
        self._decays = 0
        # node state table: pre-batch rows the batch can touch, then batch rows
        rows = np.asarray(rows, np.int64)
        n = rows.size
        cap = n + self.M + 64
        self.row = np.zeros(cap, np.int64)
        self.sal = np.zeros(cap, F32)
        self.acc = np.zeros(cap, np.int64)
        self.last = np.zeros(cap, np.float64)
        self.ncode = np.zeros(cap, np.int64)
        self.sup = np.zeros(cap, bool)
        self.alive = np.zeros(cap, bool)
        self.cand = np.zeros(cap, bool)     # eviction candidate (pool / batch node)
        self.n2 = np.zeros(cap, np.float64)   # |x|^2 of the stored fp32 row (the store's L2)
        self.nl = n
        self.row[:n] = rows
        self.sal[:n], self.acc[:n], self.last[:n] = cols[0], cols[1], cols[2]
        self.ncode[:n], self.sup[:n], self.n2[:n] = cols[3], cols[4], cols[5]
        self.alive[:n] = True
        self.loc = {int(r): i for i, r in enumerate(rows.tolist())}
        pool_l = [self.loc[int(r)] for r in pool]
        self.cand[pool_l] = True
        self.cand[:n] &= ~self.sup[:n]
        # batch edges
        self.e_src: List[int] = []
        self.e_dst: List[int] = []
        self.e_code: List[int] = []
        self.e_conv: List[int] = []
        self.e_w = np.zeros(0, F32)
        self.e_alive = np.zeros(0, bool)
        self.inc: Dict[int, List[int]] = {}
        # outputs
        self.fact_key = np.full(self.M, -1, np.int64)
        self.key_fact: Dict[int, int] = {}
        self.fact_live = np.zeros(self.M, bool)   # kept and not evicted
        self.dup_of = np.full(self.M, -1, np.int64)
        self.supers: List[Super] = []
        self.evicted: Dict[int, int] = {}
        self.stats = {"dup": 0, "inserted": 0, "linked": 0, "cross_links": 0, "pruned_new": 0, "evicted": 0,
                      "fallbacks": 0}

    # ------------------------------------------------------------------ state
    def _l(self, r: int) -> int:
        return self.loc[r]

    def _present(self, r: int) -> bool:
        return r not in self.evicted

    def _add_state(self, r: int, sal, code: int, sup: bool, n2: float = 1.0) -> int:
        i = self.nl
        self.nl += 1
        if i >= self.row.size:  # (supers beyond the reserve)
            for name in ("row", "sal", "acc", "last", "ncode", "sup", "alive", "cand", "n2"):
                a = getattr(self, name)
                setattr(self, name, np.concatenate([a, np.zeros_like(a[:64])]))
        self.row[i], self.sal[i], self.acc[i], self.last[i] = r, F32(sal), 0, self.now
        self.ncode[i], self.sup[i], self.alive[i], self.cand[i] = code, sup, True, not sup
        self.n2[i] = n2
        self.loc[r] = i
        return i

    # ------------------------------------------------------------------ candidates
    def _cands(self, j: int, same_shard: bool, kept_mask: np.ndarray) -> List[Tuple[float, int]]:
        """(cos, row) of fact j's best present rows above the link threshold:
        pre-batch rows from its list (or the exact fallback) and kept facts
        of earlier conversations; sorted (cos desc, row asc)."""
        s, r = (self.ss[j], self.sr[j]) if same_shard else (self.gs[j], self.gr[j])
        out = [(float(a), int(b)) for a, b in zip(s, r) if b >= 0 and a > self.link_thr and self._present(int(b))]
        full = r[-1] >= 0 and s[-1] > self.link_thr  # entries may exist past the list
        if full and len(out) < self.link_k + 1:
            s2, r2 = self.fallback(j, np.fromiter((x for x in self.evicted if x < self.n0), np.int64), same_shard)
            self.stats["fallbacks"] += 1
            out = [(float(a), int(b)) for a, b in zip(s2, r2) if b >= 0 and a > self.link_thr
                   and self._present(int(b))]
        m = kept_mask & (self.code == self.code[j]) if same_shard else kept_mask
        idx = np.nonzero(m)[0]
        if idx.size:
            v = self.S[j, idx]
            ok = v > self.link_thr
            out += [(float(a), int(b)) for a, b in zip(v[ok], self.fact_key[idx[ok]])]
        out.sort(key=lambda t: (-t[0], t[1]))
        return out

    # ------------------------------------------------------------------ one conversation
    def _dedupe(self, jj: Sequence[int], kept_mask: np.ndarray) -> List[int]:
        kept = []
        for j in jj:
            # the store's top-1 is by L2 (reference vector_store.py:132-140):
            # score 2|q||x|cos - |x|^2; the candidate list holds the unit rows
            # by cosine, which is their L2 order; super-nodes are not unit rows
            qn = self.qnorm[j]
            best = (NEG, -1, NEG)   # (l2 score, row, cos)

            def offer(cos, r, n2):
                nonlocal best
                l2 = 2.0 * qn * cos * np.sqrt(n2) - n2
                if l2 > best[0] or (l2 == best[0] and r < best[1]):
                    best = (l2, r, cos)
            c = self._cands(j, False, kept_mask)
            if c:
                v, r = c[0]
                offer(v, r, self.n2[self._l(r)])
            for si, sr in enumerate(self.sup_rows):
                offer(float(self.sup_cos[j, si]), sr, self.sup_n2[si])
            for sp in self.supers:
                if sp.conv < self.ct[j]:
                    offer(float(sp.cos[j]), sp.key, sp.n2)
            best_s, best_r = best[2], best[1]
            if best_r >= 0 and best_s > self.dedupe_thr:
                dups = self._pending_dups.setdefault(best_r, [])
                dups.append(j)
                self.dup_of[j] = best_r
                self.stats["dup"] += 1
            else:
                kept.append(j)
        # merges land after the whole conversation was matched (one scatter per
        # conversation in the sequential path): max salience, +1 access each
        for r, js in self._pending_dups.items():
            i = self._l(r)
            self.sal[i] = F32(max(self.sal[i], self.sal_in[js].max()))
            self.acc[i] += len(js)
            self.last[i] = self.now
            self._seg_touch.add(r)
        self._pending_dups = {}
        return kept

    def _insert(self, kept: List[int]) -> None:
        for j in kept:
            key = self._next_row
            self._next_row += 1
            self.fact_key[j] = key
            self.key_fact[key] = j
            self.fact_live[j] = True
            self._add_state(key, self.sal_in[j], int(self.code[j]), False, float(self.fact_n2[j]))
            self.shard_count[int(self.code[j])] += 1
            self.node_count += 1
            self._seg.inserts.append(("fact", j))
            self.stats["inserted"] += 1

    def _edge(self, s: int, d: int, w, h: int, c: int) -> None:
        e = len(self.e_src)
        self.e_src.append(s)
        self.e_dst.append(d)
        self.e_code.append(h)
        self.e_conv.append(c)
        self._new_w.append(F32(w))
        self.inc.setdefault(s, []).append(e)
        self.inc.setdefault(d, []).append(e)
        self._seg.edges.append(e)

    def _link(self, kept: List[int], c: int, kept_mask: np.ndarray) -> None:
        """Chain, within-shard and cross-memory edges of the conversation's
        new nodes, in the sequential path's order (MemorySystem._link_batch)."""
        if not kept:
            return
        self._new_w = []
        codes = self.code[kept]
        order = np.argsort(codes, kind="stable")
        oc = codes[order]
        for p in np.nonzero(oc[1:] == oc[:-1])[0].tolist():
            a, b = kept[order[p]], kept[order[p + 1]]
            self._edge(int(self.fact_key[a]), int(self.fact_key[b]), self.chain_w, int(self.code[a]), c)
        uc, cnt = np.unique(codes, return_counts=True)
        multi = set(uc[cnt >= 2].tolist())
        within: Dict[int, set] = {}
        for j in kept:
            if int(self.code[j]) not in multi:
                continue
            within[j] = set()
            for v, r in self._cands(j, True, kept_mask)[: self.link_k]:
                self._edge(int(self.fact_key[j]), r, F32(v * self.link_scale), int(self.code[j]), c)
                within[j].add(r)
        nc = 0
        for j in kept:
            for v, r in self._cands(j, False, kept_mask)[: self.link_k]:
                if r in within.get(j, ()):
                    continue
                self._edge(int(self.fact_key[j]), r, F32(v * self.link_scale), int(self.code[j]), c)
                nc += 1
        self.stats["linked"] += len(self._new_w)
        self.stats["cross_links"] += nc
        self.e_w = np.concatenate([self.e_w, np.asarray(self._new_w, F32)])
        self.e_alive = np.concatenate([self.e_alive, np.ones(len(self._new_w), bool)])

    def _evict(self, c: int) -> None:
        excess = self.node_count - self.max_buffer
        if excess <= 0:
            return
        li = np.nonzero(self.cand[: self.nl] & self.alive[: self.nl])[0]
        if li.size == 0:
            return
        imp = importance_np(self.sal[li], self.acc[li], self.last[li], self.now)
        if excess < li.size:
            t = np.partition(imp, excess - 1)[excess - 1]
            sel = np.nonzero(imp <= t)[0]
        else:
            sel = np.arange(li.size)
        rows = self.row[li[sel]]
        o = sel[np.lexsort((rows, self.ncode[li[sel]], imp[sel]))][:excess]
        last = o[-1]
        self.events.append((self._decays, float(imp[last]), int(self.ncode[li[last]]), int(self.row[li[last]])))
        for k in o.tolist():
            i = int(li[k])
            r = int(self.row[i])
            self.alive[i] = False
            self.evicted[r] = c
            if r >= self.n0 and r in self.key_fact:
                self.fact_live[self.key_fact[r]] = False
            self.node_count -= 1
            self.shard_count[int(self.ncode[i])] -= 1
            self._seg.victims.append(r)
            self._seg_touch.add(r)
            self.stats["evicted"] += 1
            for e in self.inc.get(r, ()):  # the victim's shard's batch edges go with it
                if self.e_alive[e] and self.e_code[e] == self.ncode[i]:
                    self.e_alive[e] = False

    def _make_supers(self, kept: List[int], c: int) -> None:
        if not self.ref_h:
            return
        for code in dict.fromkeys(int(self.code[j]) for j in kept):
            if self.shard_count[code] <= self.sthr or self.shard_count[code] < self.sthr or \
                    code in self.super_codes:
                continue
            key = self._next_row
            self._next_row += 1
            pre = [int(r) for r in self.pre_members(code) if self._present(int(r))]
            new = [int(self.fact_key[j]) for j in np.nonzero((self.fact_key >= 0) & (self.code == code))[0]]
            children = pre + [k for k in new if self._present(k)]
            cos, n2 = self.super_cos(np.asarray(children, np.int64),
                                     np.asarray([self.key_fact[k] for k in children if k >= self.n0], np.int64))
            sp = Super(code, key, children, c, cos, n2)
            self.supers.append(sp)
            self.super_codes.add(code)
            self.node_count += 1
            self._add_state(key, 0.5, code, True, sp.n2)
            self._seg.inserts.append(("super", len(self.supers) - 1))

    def _end_decay(self) -> None:
        self._decays += 1
        m = self.alive[: self.nl] & ~self.sup[: self.nl]
        self.sal[: self.nl][m] = decay_sal_np(self.sal[: self.nl][m], self.keep)
        if self.e_w.size:
            live = self.e_alive
            self.e_w[live] = (self.e_w[live] * self.keep).astype(F32)
            if self.thr is not None:
                dead = live & (self.e_w < self.thr)
                self.stats["pruned_new"] += int(dead.sum())
                self.e_alive &= ~dead

    # ------------------------------------------------------------------ driver
    def run(self, B: int, count0: int, auto: bool, every: int, cluster_every: int,
            seg_each: bool = False) -> List[Segment]:
        """Conversations 0..B-1; segments end where ``run_consolidation``
        (count % every == 0) or a k-means cluster pass is due, and at B-1
        (``seg_each``: after every conversation)."""
        self._next_row = self.n0
        self._pending_dups = {}
        segs: List[Segment] = []
        self._seg = Segment(0, 0)
        self._seg_touch = set()
        for c in range(B):
            self._seg.c1 = c
            jj = np.nonzero(self.ct == c)[0].tolist()
            kept_mask = self.fact_live & (self.ct < c)
            kept = self._dedupe(jj, kept_mask)
            self._insert(kept)
            self._link(kept, c, kept_mask)
            self._evict(c)                 # inside the consolidation (reference :773)
            self._make_supers(kept, c)     # :775-780
            self._end_decay()              # end_conversation decay + auto-prune (:624-630)
            self._evict(c)                 # :632
            count = count0 + c + 1
            point = bool(auto) and count % every == 0
            clus = bool(cluster_every) and count // cluster_every > (count - 1) // cluster_every
            if point or clus or seg_each or c == B - 1:
                self._seg.consolidate, self._seg.cluster = point, clus
                segs.append(self._close())
                if c < B - 1:
                    self._seg = Segment(c + 1, c + 1)
                    self._seg_touch = set()
        return segs

    def _close(self) -> Segment:
        s = self._seg
        new_keys = set()
        for kind, i in s.inserts:
            key = int(self.fact_key[i]) if kind == "fact" else self.supers[i].key
            new_keys.add(key)
            li = self._l(key)
            s.new_state[key] = (float(self.sal[li]), int(self.acc[li]), float(self.last[li]))
        for r in self._seg_touch:
            if r in new_keys:
                continue
            li = self._l(r)
            s.touched[r] = (float(self.sal[li]), int(self.acc[li]), float(self.last[li]))
        s.edges = [e for e in s.edges if self.e_alive[e]]
        s.edge_w = self.e_w[s.edges].copy() if s.edges else np.zeros(0, F32)  # weights at c1
        return s


def segments_as_dicts(pl: "BatchPlanner", segs: List[Segment]) -> List[Dict]:
    """The Python planner's segments in the native planner's format
    (``_lzrt.plan_batch``): what ``MemorySystem._apply_segment`` reads."""
    out = []
    for sg in segs:
        kinds = np.asarray([0 if k == "fact" else 1 for k, _ in sg.inserts], np.int32)
        idx = np.asarray([i for _, i in sg.inserts], np.int32)
        keys = [int(pl.fact_key[i]) if k == "fact" else pl.supers[i].key for k, i in sg.inserts]
        st = [sg.new_state[k] for k in keys]
        tr = list(sg.touched.keys())
        tv = [sg.touched[r] for r in tr]
        out.append({"c0": sg.c0, "c1": sg.c1, "consolidate": sg.consolidate, "cluster": sg.cluster,
                    "ins_kind": kinds, "ins_idx": idx,
                    "ins_sal": np.asarray([v[0] for v in st], np.float64),
                    "ins_acc": np.asarray([v[1] for v in st], np.int64),
                    "ins_last": np.asarray([v[2] for v in st], np.float64),
                    "edge_src": np.asarray([pl.e_src[e] for e in sg.edges], np.int64),
                    "edge_dst": np.asarray([pl.e_dst[e] for e in sg.edges], np.int64),
                    "edge_code": np.asarray([pl.e_code[e] for e in sg.edges], np.int64),
                    "edge_w": np.asarray(sg.edge_w, np.float32),
                    "victims": np.asarray(sg.victims, np.int64),
                    "tch_rows": np.asarray(tr, np.int64),
                    "tch_sal": np.asarray([v[0] for v in tv], np.float64),
                    "tch_acc": np.asarray([v[1] for v in tv], np.int64),
                    "tch_last": np.asarray([v[2] for v in tv], np.float64)})
    return out


def plan(kw: Dict, B: int, count0: int, auto: bool, every: int, cluster_every: int, native: bool = True,
         seg_each: bool = False) -> Dict:
    """Run the planner (native ``_lzrt.plan_batch`` by default, this module's
    BatchPlanner as the reference) on one input dict; returns segments,
    supers, events, fact_key, dup_of and stats in the native format.
    ``seg_each``: one segment per conversation (per-conversation commits)."""
    if native:
        from ..store.colstore import _rt
        args = dict(kw)
        args.update(B=B, count0=count0, auto=auto, every=every, cluster_every=cluster_every, seg_each=seg_each)
        gs, gr = args.pop("glob")
        ss, sr = args.pop("shard")
        args.update(gs=np.ascontiguousarray(gs, np.float64), gr=np.ascontiguousarray(gr, np.int64),
                    ss=np.ascontiguousarray(ss, np.float64), sr=np.ascontiguousarray(sr, np.int64))
        rows = args.pop("rows")
        cols = args.pop("cols")
        pool = np.asarray(args.pop("pool"), np.int64)
        args.update(rows=rows, sal=cols[0], acc=cols[1], last=cols[2], ncode=cols[3],
                    sup=np.asarray(cols[4], np.uint8), n2=cols[5],
                    pool=np.isin(np.asarray(rows, np.int64), pool).astype(np.uint8))
        args.setdefault("dedupe_thr", 0.95)
        args.setdefault("link_thr", 0.5)
        args.setdefault("link_k", 3)
        args.setdefault("link_scale", 0.8)
        args.setdefault("chain_w", 0.5)
        args["super_codes"] = np.asarray(sorted(args["super_codes"]), np.int64)
        args["shard_count"] = np.asarray(args["shard_count"], np.int64)
        dump = os.environ.get("LZK_DUMP_PLAN")  # "path:N": the N-th call's planner inputs (tools/plan_bench.py)
        global _plan_calls
        _plan_calls += 1
        if dump and _plan_calls == int(dump.rsplit(":", 1)[1]):
            dump = dump.rsplit(":", 1)[0]
            arrs = {k: v for k, v in args.items() if isinstance(v, np.ndarray)}
            scal = {k: v for k, v in args.items() if isinstance(v, (int, float, bool, str)) or v is None}
            np.savez(dump, **arrs, _scalars=np.asarray(json.dumps(scal)))
        return _rt().plan_batch(args)
    pl = BatchPlanner(**kw)
    segs = pl.run(B, count0, auto, every, cluster_every, seg_each)
    return {"segments": segments_as_dicts(pl, segs),
            "supers": [{"code": sp.code, "key": sp.key, "conv": sp.conv, "children": np.asarray(sp.children)}
                       for sp in pl.supers],
            "events": list(pl.events), "fact_key": pl.fact_key, "dup_of": pl.dup_of, "stats": dict(pl.stats)}
