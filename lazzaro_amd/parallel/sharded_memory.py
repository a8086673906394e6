"""One tenant's memory row-sharded over the ranks of a job (BASELINE config 4:
a 100M-node episodic buffer across the GPUs of a node; SURVEY.md §2.6
"Row-sharded index", §2.5 C1/C3/C4/C5).

:class:`ShardedMemorySystem` keeps the tenant's rows split over the ranks --
each rank's part is an ordinary :class:`~lazzaro_amd.core.MemorySystem` graph
(HBM columns, HIP kernels, incremental persistence under the tenant id
``"{user}@{rank}/{world}"``) -- and runs the reference's consolidation over
the WHOLE buffer with the sequential semantics of the single-process engine:
``consolidate_batch`` on N ranks gives the nodes, saliences, edges,
super-nodes and eviction victims that ``MemorySystem.consolidate_batch`` with
the same ``cadence`` gives on one process holding the union of the rows and
all ranks' conversations (rank-major order). The default
``cadence="conversation"`` is the reference's: eviction, super-nodes and
``run_consolidation`` at every conversation (:meth:`_consolidate_exact`, the
replicated batch planner); ``cadence="batch"`` plays them once per batch
(steps 1-8 below). Reference flow: ``memory_system.py:580-649``
(end_conversation), ``:651-891`` (dedupe, links), ``:535-578`` (eviction),
``:935-1010`` (run_consolidation).

Per batch with ``cadence="batch"`` (every call is collective; each rank
brings its own conversations):

1. fact rows (vector, salience, conversation, shard key) are all-gathered
   (C1, F x (4 D + 24) bytes): dedupe and linking compare every fact with
   every row of the tenant, so each rank scans ALL facts against ITS rows --
   one fused MFMA dual scan (global + same-shard top-3, float64 re-rank);
2. the per-rank top-3 lists (score, global node number, shard, owner row)
   are all-gathered and merged (K2) -- ties break on the global node number,
   the single-process row order;
3. the in-batch dedupe fixed point and the link plan
   (:func:`~lazzaro_amd.core.consolidation.batch_link_plan`) run replicated on
   the merged lists (F x F, identical on every rank), so every rank knows
   every decision without a further exchange;
4. each rank applies what it owns: decay + prune of its edges (one
   ``tg_decay_kernel`` pass), duplicate merges onto its rows, inserts of the
   kept facts of its own conversations (node ids ``node_<n>`` numbered
   globally in batch order), and the new edges whose source it holds; an
   edge to a node held elsewhere points at a ghost row carrying the remote
   node's id and shard (the reference's dangling-edge semantics do the rest);
5. eviction to the GLOBAL ``max_buffer_size``: each rank's ``excess`` lowest
   (importance, shard, node number) candidates are all-gathered and the same
   global victims picked everywhere; edges of a victim's shard that point at
   it are dropped on every rank;
6. ``run_consolidation``: connected components over every rank's edges by
   boundary-label exchange (:func:`~.sharded.distributed_components`, C5),
   component sizes / mean weights / first members reduced at the label's
   home rank (all-to-all-v), profile prompts assembled on rank 0;
7. ``hierarchy_params``: the two-level k-means hierarchy over all rows
   (distributed fine level, all-reduced centroid sums, C4);
8. each rank commits its own changed rows / edges (colstore fragment per
   rank) -- no rank ever writes another's rows.

Per-rank work per batch is (all facts) x (own rows): at a fixed buffer the
scan is split N ways (strong scaling of the buffer); the exchanged bytes are
O(facts), never O(rows).

The reference's per-shard mean super-nodes (``hierarchy_mode="reference"``,
the default without ``hierarchy_params``; memory_system.py:775-780,
893-933): a shard's members span ranks, so the planner's member and mean
callbacks are collective -- each rank contributes the global rows of the
shard's members it holds and the float64 sum of their fp32 rows, the sums
are all-gathered and added in rank order (every rank gets the same mean).
The super-node row lives on the rank holding most of its children; a rank
holding other children points their parent at a ghost row of it. Node ids
follow the single process's counter, which super-nodes do not advance:
a node's global number is its row in the union graph, its id that number
less the super-nodes before it (:meth:`_ids_of_nums`).

Not supported for a row-sharded tenant: ``merge_mode="pairwise"``
(reference default is the no-op).
"""
from __future__ import annotations

import math
import time
from typing import Dict, List, Optional, Sequence, Tuple

import numpy as np
import torch

from ..core.consolidation import (DECAY_RATE, LINK_THRESHOLD, LINK_TOPK, MIN_FACT_LEN, PROFILE_CONTENTS,
                                  _host_pinned, batch_dedupe, batch_link_plan, salience_decayed)
from ..engine.tenant_graph import GHOST, NODE, SHARD_MASK, TYPE_MASK, TYPE_SHIFT, _seg_min, _seg_sum_count
from ..ops import tenant_ops as T
from ..utils.tracing import tracer
from .comm import Communicator
from .sharded import _route, distributed_components

NEG_INF = float("-inf")
BIG = 1 << 62
NUM_BITS = 40  # global node numbers < 2^40; (shard + 1) << 40 | number orders nodes as the reference does


def _digest_compact_host(src: torch.Tensor, dst: torch.Tensor, w: torch.Tensor, valid: torch.Tensor,
                         live: torch.Tensor, shard: torch.Tensor, nl: int, min_size: int, min_avg_w: float,
                         take: int) -> torch.Tensor:
    """Host form of the compact digest (:meth:`ShardedMemorySystem.
    _digest_replicated`; the GPU runs digest.hip): ids 0 .. nl-1, ``valid``
    ids are members, ``live`` ones (shard ``shard``) are candidates. int64
    [2, m] = (order key, id) of the first ``take`` live members of every
    qualifying component, sorted by (key, id)."""
    lab = T.components(src, dst, nl).long()
    size = torch.zeros(nl, dtype=torch.long).index_add_(0, lab[valid], torch.ones(int(valid.sum()), dtype=torch.long))
    wsum, wcnt = _seg_sum_count(lab[src], w.double(), nl)
    ids = torch.arange(nl)
    key = torch.where(live, (shard.clamp_min(0) + 1) * nl + ids, torch.full_like(ids, BIG))
    first = _seg_min(lab, key, nl, BIG)
    ok = (size >= min_size) & (wcnt > 0) & (wsum / wcnt.clamp_min(1).double() > min_avg_w) & (first < BIG)
    ci = torch.nonzero(live & ok[lab]).flatten()
    if ci.numel() == 0:
        return torch.zeros((2, 0), dtype=torch.long)
    ci = ci[torch.argsort(lab[ci], stable=True)]  # grouped by component, id order inside
    cl = lab[ci]
    newg = torch.ones_like(cl, dtype=torch.bool)
    newg[1:] = cl[1:] != cl[:-1]
    gstart = torch.nonzero(newg).flatten()[torch.cumsum(newg.long(), 0) - 1]
    sel = ci[(torch.arange(ci.numel()) - gstart) < take]
    k = first[lab[sel]]
    o = torch.argsort(sel, stable=True)
    o = o[torch.argsort(k[o], stable=True)]
    return torch.stack([k[o], sel[o]])


def shard_user_id(user: str, rank: int, world: int) -> str:
    return f"{user}@{rank}/{world}"


class ShardedMemorySystem:
    """A tenant whose rows are split over ``comm``'s ranks (see module doc).

    ``local_kwargs`` go to each rank's :class:`MemorySystem` (providers,
    ``db_dir``, ``store``, ``device``...). ``max_buffer_size`` is the GLOBAL
    node limit. ``hierarchy_params`` ({"fine", "top", "every", "iters"})
    turns on the distributed k-means hierarchy, re-clustered whenever the
    global conversation count crosses a multiple of ``every``.

    ``prune`` (with a hierarchy): exact cross-rank pruning of the
    consolidation scan -- a fact is compared with this rank's rows only if a
    fine cluster held here can contain a row at cos > LINK_THRESHOLD (angular
    radius bound, :meth:`_reach_mask`). ``placement="cluster"``: a new node
    is held by the home rank of its fine cluster (the rank holding most of
    that cluster's rows) instead of the rank whose conversation made it, so
    topics stay together and the pruned scan stays ~(own facts) x (own
    rows) as ranks are added. Neither changes a decision."""

    def __init__(self, comm: Optional[Communicator] = None, user_id: str = "default", *,
                 max_buffer_size: int = 10, consolidate_every: int = 3, auto_consolidate: bool = True,
                 auto_prune: bool = True, prune_threshold: float = 0.5,
                 hierarchy_params: Optional[Dict] = None, prune: bool = True, placement: str = "origin",
                 force_collectives: Optional[bool] = None, enable_hierarchy: bool = True,
                 hierarchy_mode: Optional[str] = None, super_node_threshold: int = 20, **local_kwargs):
        from ..core.memory_system import MemorySystem

        self.comm = comm or Communicator.local()
        if hierarchy_mode is None:
            hierarchy_mode = "kmeans" if hierarchy_params else "reference"
        if hierarchy_mode not in ("reference", "kmeans"):
            raise ValueError("hierarchy_mode must be 'reference' or 'kmeans'")
        # the reference's per-shard mean super-nodes (memory_system.py:893-933)
        self.ref_hierarchy = bool(enable_hierarchy) and hierarchy_mode == "reference"
        self.super_node_threshold = int(super_node_threshold)
        self._sup_v = np.zeros(0, np.int64)  # global rows of the tenant's super-nodes (sorted, every rank)
        self._super_plan: Dict[Tuple[int, ...], Dict] = {}
        self._commit_each = False
        if force_collectives is None:
            import os
            force_collectives = os.environ.get("LZK_FORCE_COLLECTIVES", "0") == "1"
        # every exchange through the communicator (also at world 1 under a
        # 1-rank torch.distributed.run: the N-rank code path on one GPU)
        self._coll = self.comm.world > 1 or (bool(force_collectives) and self.comm.enabled)
        self.user_id = user_id
        self.max_buffer_size = int(max_buffer_size)
        self.consolidate_every = int(consolidate_every)
        self.auto_consolidate = auto_consolidate
        self.auto_prune = auto_prune
        self.prune_threshold = float(prune_threshold)
        self.hierarchy_params = dict(hierarchy_params) if hierarchy_params else None
        local_kwargs.setdefault("enable_async", False)
        local_kwargs.setdefault("load_from_disk", False)
        local_kwargs.setdefault("enable_caching", False)
        self.local = MemorySystem(user_id=shard_user_id(user_id, self.comm.rank, self.comm.world),
                                  max_buffer_size=1 << 62, auto_consolidate=False, enable_hierarchy=False,
                                  auto_prune=auto_prune, prune_threshold=prune_threshold,
                                  super_node_threshold=super_node_threshold, **local_kwargs)
        self.g = self.local.graph
        self.device = self.g.device
        self.num = torch.full((0,), -1, dtype=torch.long, device=self.device)  # global node number per row
        # rank holding each row's node (a ghost row: the remote holder)
        self.holder = torch.full((0,), -1, dtype=torch.long, device=self.device)
        self.next_id = 0  # last global node number handed out (identical on every rank)
        self.conversation_count = 0
        if placement not in ("origin", "cluster"):
            raise ValueError(f"placement must be 'origin' or 'cluster', not {placement!r}")
        self.prune = bool(prune)
        self.placement = placement
        self._reach: Optional[Dict] = None  # per fine cluster: centroid, angular radius over this rank's rows
        self.scan_work = 0  # facts x rows this rank's consolidation scans compared (cumulative)
        self.last_scan_work = 0

    # ------------------------------------------------------------------ plumbing
    @property
    def rank(self) -> int:
        return self.comm.rank

    @property
    def world(self) -> int:
        return self.comm.world

    def _to_comm(self, t: torch.Tensor) -> torch.Tensor:
        return t.to(self.comm.device) if self._coll else t

    def _gather_rows(self, t: torch.Tensor) -> torch.Tensor:
        """Equal-shaped tensors of every rank, concatenated in rank order."""
        if not self._coll:
            return t
        return self.comm.all_gather_rows(self._to_comm(t.contiguous())).to(t.device)

    def _gather_var(self, t: torch.Tensor) -> Tuple[torch.Tensor, List[int]]:
        """Variable-length rows of every rank in rank order (+ per-rank counts)."""
        if not self._coll:
            return t, [int(t.shape[0])]
        cnt = self._host_ints(int(t.shape[0]))[:, 0].tolist()  # counts over gloo: no device read
        mx = max(cnt)
        if mx == 0:  # nothing anywhere (every rank sees the same counts): no empty collective
            return t, cnt
        pad = torch.zeros((mx,) + tuple(t.shape[1:]), dtype=t.dtype, device=t.device)
        pad[: t.shape[0]] = t
        g = self._gather_rows(pad)
        idx = torch.cat([torch.arange(r * mx, r * mx + c) for r, c in enumerate(cnt)]).to(t.device)
        return g[idx], cnt

    def _host_ints(self, *vals) -> np.ndarray:
        """[world, len(vals)] host ints of every rank (gloo; host metadata
        never waits on the GPU stream)."""
        a = np.asarray([int(v) for v in vals], np.int64)
        return self.comm.host_all_gather(a) if self._coll else a[None]

    def _sum(self, *vals) -> List[int]:
        return [int(x) for x in self._host_ints(*vals).sum(0).tolist()]

    def _sync_num(self) -> None:
        n = self.g.n
        if self.num.numel() < n:
            grow = torch.full((max(n, 2 * self.num.numel()) - self.num.numel(),), -1, dtype=torch.long,
                              device=self.device)
            self.num = torch.cat([self.num, grow])
            self.holder = torch.cat([self.holder, grow.clone()])

    # rows appended since the sorted number index was built are searched in a
    # small sorted delta; the base is rebuilt once the delta outgrows this
    NUM_DELTA_MAX = 1 << 16

    def _num_index(self) -> Dict:
        """Sorted index of the number column: a base over rows [0, n0) and a
        delta over the rows appended since, each (sorted numbers, rows). A
        row's number is written once, right after its row is added, so the
        index only ever grows -- the consolidation looks rows up several
        times per segment, and re-sorting a 10M-row column each time was the
        row-sharded step's largest cost."""
        n = self.g.n
        ix = getattr(self, "_num_ix", None)
        dev = self.device

        def build(a, b):
            key = self.num[a:b]
            o = torch.argsort(key, stable=True)
            return key[o], o + a
        if ix is None or ix["n0"] > n or n - ix["n0"] > max(self.NUM_DELTA_MAX, ix["n0"] >> 4):
            ks, o = build(0, n)
            z = torch.zeros(0, dtype=torch.long, device=dev)
            ix = {"n0": n, "n1": n, "ks": ks, "o": o, "dk": z, "do": z}
            self._num_ix = ix
        elif ix["n1"] < n:
            ix["dk"], ix["do"] = build(ix["n0"], n)
            ix["n1"] = n
        return ix

    def _rows_of_nums(self, nums: torch.Tensor, held: bool = False, add: int = 0) -> torch.Tensor:
        """Local row holding each global node number ``nums + add`` (live or
        ghost), -1 if none: binary searches in the cached sorted number index
        (no host map) -- on the GPU one kernel (tenant_ops.num_rows). ``held``:
        only rows this rank holds live."""
        g = self.g
        n = g.n
        if n == 0 or nums.numel() == 0:
            return torch.full_like(nums, -1)
        ix = self._num_index()
        if g.on_gpu:
            return T.num_rows(nums, add, ix["ks"], ix["o"], ix["dk"], ix["do"], self.holder, g.kind,
                              self.rank if held else -1)
        if add:
            nums = nums + add
        out = torch.full_like(nums, -1)
        for ks, o in ((ix["dk"], ix["do"]), (ix["ks"], ix["o"])):  # the base wins a (never expected) tie
            if ks.numel() == 0:
                continue
            pos = torch.searchsorted(ks, nums).clamp_max(ks.numel() - 1)
            out = torch.where(ks[pos] == nums, o[pos], out)
        if held:
            rc = out.clamp_min(0)
            ok = (out >= 0) & (self.holder[rc] == self.rank) & (g.kind[rc] == NODE)
            out = torch.where(ok, out, torch.full_like(out, -1))
        return out

    def _ids_of_nums(self, nums) -> List[str]:
        """Node ids of fact nodes by global number (row + 1). The single
        process names nodes with a counter that super-nodes do not advance
        (reference memory_system.py:_generate_node_id), so a node's id is its
        number less the super-nodes created before it."""
        a = np.asarray(nums, np.int64).reshape(-1)
        if self._sup_v.size:
            a = a - np.searchsorted(self._sup_v, a - 1, side="left")
        return [f"node_{int(x)}" for x in a.tolist()]

    @property
    def _fact_count(self) -> int:
        """The single process's node counter: fact nodes numbered so far."""
        return int(self.next_id) - int(self._sup_v.size)

    def _register_shards(self, keys: Sequence[str]) -> np.ndarray:
        return np.asarray([self.g.shard_id(k) for k in keys], dtype=np.int32)

    # ------------------------------------------------------------------ loading
    def register_shards(self, names: Sequence[str]) -> List[int]:
        """Create shards in this order on every rank (call with the same list
        everywhere) so raw shard codes can be passed to :meth:`add_memories`."""
        return self._register_shards(names).tolist()

    def add_memories(self, contents: Sequence[str], vectors: torch.Tensor, shard_keys: Optional[Sequence[str]] = None,
                     salience=0.5, now: Optional[float] = None, types="semantic", shard_codes=None) -> torch.Tensor:
        """Collective bulk insert of already-extracted memories (a tenant load
        or a migration): every rank passes its own rows; they get global node
        numbers in rank-major order and stay on the rank that passed them.
        ``shard_keys`` are registered in that global order on every rank so the
        shard codes agree everywhere; ``shard_codes`` (codes of shards created
        by :meth:`register_shards`) skip that exchange for bulk loads.
        Returns this rank's new rows."""
        m = len(contents)
        if shard_codes is None:
            keys_all = [k for ks in self.comm.all_gather_object(list(shard_keys)) for k in ks] \
                if self._coll else list(shard_keys)
        counts = self._gather_rows(torch.tensor([m], dtype=torch.int64, device=self.device)).tolist()
        off = sum(counts[: self.rank])
        codes = self._register_shards(keys_all)[off: off + m] if shard_codes is None else shard_codes
        base = self.next_id
        self.next_id += sum(counts)
        if m == 0:
            return torch.zeros(0, dtype=torch.long, device=self.device)
        nums = torch.arange(base + off + 1, base + off + m + 1, dtype=torch.long, device=self.device)
        ids = self._ids_of_nums(np.arange(base + off + 1, base + off + m + 1))
        now = time.time() if now is None else now
        rows = self.g.add_nodes(ids, list(contents), vectors, shard=codes, types=types, sal=salience, now=now,
                                stored=True)
        self._sync_num()
        self.num[rows] = nums
        self.holder[rows] = self.rank
        self.local.node_counter = self._fact_count
        self._reach_add(rows)
        return rows

    # ------------------------------------------------------------------ scan pruning
    REACH_SLACK = 1e-5  # on the radius cosines: covers fp32 rounding of the row / centroid dots
    REACH_CHUNK = 1 << 18
    FAR_MAX = 1 << 15  # rows bounded exactly instead of by their cluster's cone

    def _row_cos(self, rows: torch.Tensor, C: torch.Tensor, lab: Optional[torch.Tensor] = None):
        """(label, cos) of rows against unit centroids C [K, D] (fp32): the
        given labels, or the nearest centroid. Rows without a vector -> cos -1
        (the cluster's radius becomes 180 degrees: never pruned)."""
        g = self.g
        if lab is not None and g.on_gpu and g.dim % 4 == 0:  # one fused pass over the rows
            cs = T.row_centroid_cos(g.emb32, g.dim, g.sqn, rows, lab, C)
            return lab, cs.double() - self.REACH_SLACK
        labs, coss = [], []
        for a in range(0, rows.numel(), self.REACH_CHUNK):
            r = rows[a: a + self.REACH_CHUNK]
            X = g.emb32[r].float()
            nrm = g.sqn[r].float().sqrt()
            den = torch.where(nrm > 0, nrm, torch.ones_like(nrm))
            if lab is None:
                cs, lb = ((X @ C.T) / den[:, None]).max(1)
            else:  # the labelled centroid only: a row dot, not a [rows, K] GEMM (10M x 4096 after a pass)
                lb = lab[a: a + self.REACH_CHUNK]
                cs = (X * C[lb]).sum(1) / den
            cs = torch.where(nrm > 0, cs, torch.full_like(cs, -1.0))
            labs.append(lb)
            coss.append(cs.double() - self.REACH_SLACK)
        if not labs:
            return rows.new_zeros(0), torch.zeros(0, dtype=torch.float64, device=rows.device)
        return torch.cat(labs), torch.cat(coss)

    def _build_reach(self, collective: bool = True) -> None:
        """Per fine cluster of the hierarchy: unit centroid and the cosine of
        the largest angle between it and a CORE row of this rank (2.0: none).
        The rows farthest from their centroid (at most FAR_MAX / 2 over all
        clusters) are kept out of the radii and bounded exactly instead (the
        "far" rows: each fact's cosine with them is computed), so a few
        outliers do not open a cluster's cone. Rebuilt after every cluster
        pass (and locally when the far set overflows); inserts that fall
        outside their cluster's cone join the far set; deletions leave both
        (still upper bounds)."""
        g = self.g
        h = getattr(g, "hier", None)
        if h is None or h.get("fine_c") is None or g.dim is None:
            self._reach = None
            return
        dev = self.device
        D = g.dim
        C = h["fine_c"][:, :D].float().to(dev)
        C = C / C.norm(dim=1, keepdim=True).clamp_min(1e-30)
        K = C.shape[0]
        n = g.n
        with g.on_stream():
            lab = h["fine"][:n].long().to(dev) if h["fine"].numel() >= n else None
            live = (g.kind[:n] == NODE) & (g.sup[:n] == 0)
            rows = torch.nonzero(live).flatten()
            cosr = torch.full((K,), 2.0, dtype=torch.float64, device=dev)
            far = rows[:0]
            lr = rows[:0]
            if rows.numel():
                lr = lab[rows] if lab is not None else None
                if lr is not None and bool((lr < 0).any()):
                    lr = None  # rows the pass did not label: nearest centroid for all
                lr, cs = self._row_cos(rows, C, lr)
                nf = min(self.FAR_MAX // 2, rows.numel())
                core = torch.ones_like(cs, dtype=torch.bool)
                if nf:
                    fi = torch.topk(cs, nf, largest=False).indices
                    core[fi] = False
                    far = rows[fi]
                cosr.scatter_reduce_(0, lr[core], cs[core], "amin", include_self=True)
        home = self._reach.get("home") if (self._reach is not None and not collective) else None
        self._reach = {"C": C, "Cd": C.double(), "cosr": cosr, "far": far, "far_x": None}
        if home is not None:
            self._reach["home"] = home
        if self.placement == "cluster" and collective:
            cnt = torch.zeros(K, dtype=torch.int64, device=dev)
            if lr.numel():
                cnt.index_add_(0, lr, torch.ones_like(lr))
            allc = self._gather_rows(cnt[None, :])  # [W, K]
            best = torch.argmax(allc, 0)  # first max: the lowest rank on ties
            self._reach["home"] = torch.where(allc.max(0).values > 0, best, torch.arange(K, device=dev) % self.world)

    def _reach_add(self, rows: torch.Tensor) -> None:
        """New live rows of this rank: inside their nearest cluster's cone
        they change nothing; outside they join the far set."""
        r = self._reach
        if r is None or rows.numel() == 0:
            return
        with self.g.on_stream():
            rows = rows.to(self.device).long()
            lr, cs = self._row_cos(rows, r["C"])
            out = cs < r["cosr"][lr]
            if bool(out.any()):
                r["far"] = torch.cat([r["far"], rows[out]])
                r["far_x"] = None
        if r["far"].numel() > self.FAR_MAX:
            self._build_reach(collective=False)

    def _reach_mask(self, Qn: torch.Tensor) -> Optional[torch.Tensor]:
        """Facts (unit float64 rows) that may have a row of this rank at cos >
        LINK_THRESHOLD. Core rows: angle(q, x) >= angle(q, c) - radius(c) for
        every core row x of cluster c, so cos(q, x) <= cos(max(0, angle(q, c)
        - radius(c))). Far rows: the cosine itself (fp32, with slack)."""
        r = self._reach
        if r is None or not self.prune:
            return None
        g = self.g
        sel = torch.zeros(Qn.shape[0], dtype=torch.bool, device=Qn.device)
        cosr = r["cosr"]
        held = cosr <= 1.0
        if bool(held.any()):
            cr = cosr[held].clamp(-1.0, 1.0)
            sr = torch.sqrt((1.0 - cr * cr).clamp_min(0.0))
            ct = (Qn @ r["Cd"][held].T).clamp(-1.0, 1.0)
            st = torch.sqrt((1.0 - ct * ct).clamp_min(0.0))
            bound = torch.where(ct >= cr[None, :], torch.ones_like(ct), ct * cr[None, :] + st * sr[None, :])
            sel |= bound.max(1).values > LINK_THRESHOLD - 1e-6
        far = r["far"]
        if far.numel():
            if r["far_x"] is None:
                X = g.emb32[far].float()
                nrm = g.sqn[far].float().sqrt()
                r["far_x"] = X / torch.where(nrm > 0, nrm, torch.ones_like(nrm))[:, None]
            sel |= (Qn.float() @ r["far_x"].T).max(1).values > LINK_THRESHOLD - self.REACH_SLACK * 10
        return sel

    def _holders(self, Qn: torch.Tensor, origin: torch.Tensor) -> torch.Tensor:
        """Rank that will hold each fact's node: its conversation's rank, or
        (placement="cluster") the home rank of its nearest fine cluster --
        computed identically on every rank (float64, same inputs)."""
        r = self._reach
        if self.placement != "cluster" or r is None or "home" not in r:
            return origin
        return r["home"][torch.argmax(Qn @ r["Cd"].T, 1)]

    # ------------------------------------------------------------------ queries
    def num_nodes(self) -> int:
        return self._sum(self.g.num_nodes())[0]

    def num_edges(self) -> int:
        return self._sum(self.g.num_edges)[0]

    def _candidates(self, Q: torch.Tensor, codes: torch.Tensor):
        """Global (dual) top-3 of every fact over every rank's live nodes:
        local fused scan, all-gather of the lists, merge by (score desc,
        node number asc). Returns ((s, num, shard, rank, row) global,
        (same) same-shard), each s [F, 3] fp64 and ints [F, 3]."""
        g = self.g
        F = Q.shape[0]
        dev = self.device
        k = LINK_TOPK
        live = g.num_nodes() if g.n else 0
        sel = None
        if live:
            Qd = Q.double()
            qn = Qd.norm(dim=1, keepdim=True)
            sel = self._reach_mask(Qd / torch.where(qn > 0, qn, torch.ones_like(qn)))
        n_scan = F if sel is None else int(sel.sum())
        self.last_scan_work = n_scan * live
        self.scan_work += self.last_scan_work
        if live and n_scan:
            n = g.n
            mask = (g.kind[:n] == NODE) & (g.sup[:n] == 0)
            # decisions read only entries above LINK_THRESHOLD (as in _scan_batch)
            if sel is None or n_scan == F:
                (gs, gr), (ws, wr) = g.cos_topk(Q, k, mask, dual_label=codes, min_score=LINK_THRESHOLD)
            else:  # only the facts a cluster held here can reach; the rest get empty lists
                si = torch.nonzero(sel).flatten()
                (gs_, gr_), (ws_, wr_) = g.cos_topk(Q[si], k, mask, dual_label=codes[si],
                                                    min_score=LINK_THRESHOLD)
                gs = torch.full((F, k), NEG_INF, dtype=torch.float64, device=dev)
                ws = gs.clone()
                gr = torch.full((F, k), -1, dtype=torch.long, device=dev)
                wr = gr.clone()
                gs[si], gr[si], ws[si], wr[si] = gs_.to(dev), gr_.to(dev), ws_.to(dev), wr_.to(dev)
        else:
            gs = ws = torch.full((F, k), NEG_INF, dtype=torch.float64, device=dev)
            gr = wr = torch.full((F, k), -1, dtype=torch.long, device=dev)

        def pack(s, r):
            ok = r >= 0
            rr = r.clamp_min(0)
            num = torch.where(ok, self.num[rr], torch.full_like(r, -1))
            sh = torch.where(ok, g.shard[rr].long() if g.n else torch.zeros_like(r), torch.full_like(r, -1))
            own = torch.where(ok, torch.full_like(r, self.rank), torch.full_like(r, -1))
            return s, torch.stack([num, sh, own, torch.where(ok, r, torch.full_like(r, -1))], 2)

        out = []
        for s, r in ((gs, gr), (ws, wr)):
            s, meta = pack(s, r)
            if self._coll:
                s = self._gather_rows(s).view(self.world, F, k).permute(1, 0, 2).reshape(F, -1)
                meta = self._gather_rows(meta).view(self.world, F, k, 4).permute(1, 0, 2, 3).reshape(F, -1, 4)
                key = torch.where(meta[:, :, 0] >= 0, meta[:, :, 0], torch.full_like(meta[:, :, 0], BIG))
                o = torch.argsort(key, dim=1, stable=True)
                s = torch.gather(s, 1, o)
                meta = torch.gather(meta, 1, o[:, :, None].expand(-1, -1, 4))
                o = torch.sort(s, dim=1, descending=True, stable=True).indices[:, :k]
                s = torch.gather(s, 1, o)
                meta = torch.gather(meta, 1, o[:, :, None].expand(-1, -1, 4))
            out.append((s, meta))
        return out

    def search_memories_batch(self, queries: Sequence[str], limit: int = 5) -> List[List[Dict]]:
        """Collective ``search_memories`` over the whole tenant (reference
        :1460-1472): every rank embeds its own queries, the query rows are
        all-gathered, each rank runs the store search (fused scan + fp32
        re-rank, L2) over its rows, the (score, owner, row) lists are merged
        (ties -> lower node number) and the winners' node dicts are returned
        to the rank that asked. Returns this rank's results."""
        g = self.g
        dev = self.device
        qs = list(queries)
        E = self.local._batch_embed_any(qs) if qs else None
        D = g.dim
        E = (E.to(dev, torch.float32) if torch.is_tensor(E) else
             torch.as_tensor(np.asarray(E, np.float32)).to(dev)) if qs else torch.zeros((0, D), device=dev)
        Qa, qcnt = self._gather_var(E)
        nq = Qa.shape[0]
        if nq == 0:
            return [[] for _ in qs]
        if g.n and g.num_nodes():
            sc, rows = g.store_search(Qa.float(), limit, self.local.vector_store.metric)
            sc, rows = sc.to(dev).double(), rows.to(dev).long()
            ok = rows >= 0
            sc = torch.where(ok, sc, torch.full_like(sc, NEG_INF))
            num = torch.where(ok, self.num[rows.clamp_min(0)], torch.full_like(rows, -1))
        else:
            sc = torch.full((nq, limit), NEG_INF, dtype=torch.float64, device=dev)
            rows = num = torch.full((nq, limit), -1, dtype=torch.long, device=dev)
        meta = torch.stack([num, torch.where(num >= 0, torch.full_like(num, self.rank), num), rows], 2)
        if self._coll:
            sc = self._gather_rows(sc).view(self.world, nq, limit).permute(1, 0, 2).reshape(nq, -1)
            meta = self._gather_rows(meta).view(self.world, nq, limit, 3).permute(1, 0, 2, 3).reshape(nq, -1, 3)
            key = torch.where(meta[:, :, 0] >= 0, meta[:, :, 0], torch.full_like(meta[:, :, 0], BIG))
            o = torch.argsort(key, dim=1, stable=True)
            sc, meta = torch.gather(sc, 1, o), torch.gather(meta, 1, o[:, :, None].expand(-1, -1, 3))
            o = torch.sort(sc, dim=1, descending=True, stable=True).indices[:, :limit]
            sc, meta = torch.gather(sc, 1, o), torch.gather(meta, 1, o[:, :, None].expand(-1, -1, 3))
        mh = meta.cpu().numpy()
        sh = sc.cpu().numpy()
        # the node dicts of the winners this rank holds, sent to the asking rank
        qoff = np.cumsum([0] + qcnt)
        mine = {}
        for q in range(nq):
            for j in range(limit):
                if mh[q, j, 0] >= 0 and mh[q, j, 1] == self.rank and np.isfinite(sh[q, j]):
                    mine[(q, j)] = self._node_dict(int(mh[q, j, 2]))
        parts = self.comm.all_gather_object(mine) if self._coll else [mine]
        got = {}
        for p in parts:
            got.update(p)
        q0 = int(qoff[self.rank])
        return [[got[(q0 + i, j)] for j in range(limit) if (q0 + i, j) in got] for i in range(len(qs))]

    def _node_dict(self, r: int) -> Dict:
        g = self.g
        with g.on_stream():
            sal, acc, last, ts, sh = (float(g.sal[r]), int(g.acc[r]), float(g.last[r]), float(g.ts[r]),
                                      int(g.shard[r]))
        return {"id": g.ids[r], "content": g.content[r], "type": g.types[r], "salience": sal,
                "access_count": acc, "last_accessed": last, "timestamp": ts,
                "shard_key": g.shard_names[sh] if 0 <= sh < len(g.shard_names) else None}

    # ------------------------------------------------------------------ consolidation
    def consolidate_batch(self, conversations: Sequence[Sequence[Dict]], embeddings=None,
                          now: Optional[float] = None, cadence: str = "conversation",
                          commit: str = "batch") -> Dict[str, int]:
        """Collective batched ``end_conversation`` (see module doc). Each rank
        passes its own finished conversations' extracted facts (and optionally
        their vectors, aligned with the flattened facts). Returns the counts of
        the WHOLE batch (identical on every rank).

        ``cadence="conversation"`` (default): the reference's per-conversation
        cadence -- the state ``MemorySystem.consolidate_batch`` (same cadence)
        reaches on one process holding the union (:meth:`_consolidate_exact`);
        ``"batch"``: eviction and run_consolidation once per batch.
        ``commit="conversation"`` (with the conversation cadence): every rank
        commits its rows after each conversation of the batch is applied --
        the reference's save per ``end_conversation`` (memory_system.py:648,
        785); ``"batch"``: one commit per rank per batch."""
        if cadence not in ("conversation", "batch"):
            raise ValueError("cadence must be 'conversation' or 'batch'")
        if commit not in ("conversation", "batch"):
            raise ValueError("commit must be 'conversation' or 'batch'")
        self._commit_each = commit == "conversation" and cadence == "conversation"
        self._batch_src = embeddings  # a prefetched batch is keyed by its embeddings object
        g = self.g
        dev = self.device
        flat, conv, idx = [], [], []
        j = 0
        for c, fs in enumerate(conversations):
            for f in fs:
                if isinstance(f, dict) and f.get("content") and len(f["content"]) >= MIN_FACT_LEN:
                    flat.append(f)
                    conv.append(c)
                    idx.append(j)
                j += 1
        # the batch clock: one `now` for every rank (rank 0's)
        t_now = torch.tensor([time.time() if now is None else now], dtype=torch.float64, device=dev)
        if self._coll:
            t_now = self.comm.broadcast(self._to_comm(t_now), 0).to(dev)
        now = float(t_now.item())
        m = len(flat)
        if embeddings is not None and m:
            E = embeddings if torch.is_tensor(embeddings) else torch.as_tensor(np.asarray(embeddings, np.float32))
            E = E[torch.as_tensor(idx, dtype=torch.long).to(E.device)] if len(idx) != len(E) else E
        elif m:
            with tracer.stage("embed_facts", dev):
                E = self.local._batch_embed_any([f["content"] for f in flat])
        else:
            E = None
        if m:
            E, valid = self.local._fact_matrix(E, m)
            vidx = np.nonzero(valid)[0]
            flat = [flat[i] for i in vidx]
            conv = [conv[i] for i in vidx]
            E = E[torch.as_tensor(vidx, dtype=torch.long).to(E.device)].to(dev, torch.float32)
            m = len(flat)
        d = torch.tensor([g.dim or (int(E.shape[1]) if E is not None else 0)], dtype=torch.int64, device=dev)
        if self._coll:
            d = self.comm.all_reduce(self._to_comm(d), "max").to(dev)
        if g.dim is None and int(d.item()):
            g._set_dim(int(d.item()))
        D = g.dim or 0
        if E is None:
            E = torch.zeros((0, D), dtype=torch.float32, device=dev)
        B_loc = len(conversations)
        stats = {"conversations": 0, "facts": 0, "dup": 0, "inserted": 0, "linked": 0, "cross_links": 0,
                 "pruned": 0, "evicted": 0, "consolidations": 0, "fallbacks": 0}
        if cadence == "conversation":
            # one switch to the graph's stream for the whole batch (as the
            # single process): the graph operations inside skip their stream hop
            with self.local._graph_lock, tracer.stage("sharded_consolidate", dev), g.on_stream():
                self._consolidate_exact(flat, conv, E, B_loc, now, stats)
                self.local.node_counter = self._fact_count
                with tracer.stage("persist", "cpu"):
                    self.local._save_to_persistence()
            return stats
        with self.local._graph_lock, tracer.stage("sharded_consolidate", dev):
            self._consolidate(flat, conv, E, B_loc, now, stats)
            self._evict(now, stats)
            c0 = self.conversation_count
            self.conversation_count += stats["conversations"]
            if self.auto_consolidate and (self.conversation_count // self.consolidate_every
                                          > c0 // self.consolidate_every):
                stats["consolidations"] += 1
                with tracer.stage("run_consolidation", dev):
                    self.run_consolidation()
            hp = self.hierarchy_params
            if hp and (self.conversation_count // hp["every"] > c0 // hp["every"]
                       or getattr(g, "hier", None) is None):
                with tracer.stage("cluster", dev):
                    self.cluster_pass()
            self.local.node_counter = self._fact_count
            with tracer.stage("persist", "cpu"):
                self.local._save_to_persistence()
        return stats

    def _consolidate(self, flat, conv, E, B_loc, now, stats) -> None:
        g = self.g
        dev = self.device
        comm = self.comm
        keep = 1.0 - DECAY_RATE
        thr = self.prune_threshold if self.auto_prune else None
        m = len(flat)
        # ---- 1. the global fact batch (rank-major conversation order)
        with tracer.stage("sc_gather", dev):
            bl = self._host_ints(B_loc)[:, 0].tolist()
            B = int(sum(bl))
            c_off = int(sum(bl[: self.rank]))
            keys = [self.local._fact_shard_key(f) for f in flat]
            keys_all = [k for ks in comm.all_gather_object(keys) for k in ks] if self._coll else keys
            sal_l = torch.tensor([float(f.get("salience", 0.5)) for f in flat], dtype=torch.float32, device=dev)
            ct_l = torch.tensor(conv, dtype=torch.long, device=dev) + c_off
            Qa, fcnt = self._gather_var(E)
            sal_in, _ = self._gather_var(sal_l)
            ct, _ = self._gather_var(ct_l)
        stats["conversations"] = B
        F = int(Qa.shape[0])
        stats["facts"] = F
        if F == 0:
            stats["pruned"] += self._sum(g.decay(1.0 - keep, thr, steps=B))[0]
            return
        origin = torch.repeat_interleave(torch.arange(self.world, device=dev),
                                         torch.tensor(fcnt, dtype=torch.long, device=dev))
        origin_conv = origin
        codes = self._register_shards(keys_all)
        code_t = torch.as_tensor(codes).to(dev)
        Q = Qa.float()
        Qd = Q.double()
        qn = Qd.norm(dim=1, keepdim=True)
        Qn = Qd / torch.where(qn > 0, qn, torch.ones_like(qn))
        origin = self._holders(Qn, origin_conv)  # the rank that will hold each fact's node
        if origin is not origin_conv:  # the holders need the contents of facts from other ranks
            flat = [f for part in comm.all_gather_object([{"content": f["content"], "type": f.get("type", "semantic")}
                                                          for f in flat]) for f in part]
            f_off = 0
        else:
            f_off = int(sum(fcnt[: self.rank]))

        # ---- 2. every fact against every rank's rows: local dual scan + merge
        with tracer.stage("sc_scan", dev), g.on_stream():
            (gs, gm), (ws, wm) = self._candidates(Q, code_t)
        gb_s = gs[:, 0]
        gb_node = gm[:, 0, 0] >= 0
        # the dedupe top-1 is the store's, by L2: a super-node (a mean, not a
        # unit row) can beat the list head (single process: _scan_batch)
        sup_win = sup_head = None
        if self.ref_hierarchy:
            srows, scos, sn2, _ = self._stored_supers(Qn)
            if srows.size:
                sup_win, sup_head, sup_cos = self._super_heads(qn, gs, gm, srows, scos, sn2)
                gb_s = torch.where(sup_win, sup_cos, gb_s)
                gb_node = gb_node | sup_win

        # ---- 3. replicated decisions
        with tracer.stage("sc_dedupe", dev):
            S, earlier, dup, batch_best, bb_i, ins = batch_dedupe(Qn, ct, gb_s, gb_node)
        dup_graph = dup & ~batch_best
        dup_batch = dup & batch_best
        sal_dec = salience_decayed(sal_in, (B - ct).double(), keep)

        # ---- 4. decay + prune this rank's edges / node saliences by B conversations
        with tracer.stage("sc_decay", dev):
            stats["pruned"] += self._sum(g.decay(1.0 - keep, thr, steps=B))[0]

        # ---- 5. duplicate merges onto the rows this rank holds
        stats["dup"] += int(dup.sum())
        mine_dup = dup_graph & (gm[:, 0, 2] == self.rank)
        tgt_row = gm[:, 0, 3]
        if sup_win is not None:
            srow_l = self._held_rows(sup_head.clamp_min(0))
            mine_dup = torch.where(sup_win, dup_graph & (srow_l >= 0), mine_dup)
            tgt_row = torch.where(sup_win, srow_l, tgt_row)
        if bool(mine_dup.any()):
            rows = tgt_row[mine_dup]
            with g.on_stream():
                g.sal.scatter_reduce_(0, rows, sal_dec[mine_dup].float(), "amax", include_self=True)
                g.last[rows] = now
                g.acc.index_add_(0, rows, torch.ones_like(rows, dtype=torch.int32))
                g.dirty[rows] = 1
            g._bump()
        sal_new = sal_dec.clone()
        acc_new = torch.zeros(F, dtype=torch.int32, device=dev)
        if bool(dup_batch.any()):
            tgt = bb_i[dup_batch]
            sal_new.scatter_reduce_(0, tgt, sal_dec[dup_batch], "amax", include_self=True)
            acc_new.index_add_(0, tgt, torch.ones_like(tgt, dtype=torch.int32))

        # ---- 6. inserts: kept facts numbered globally in batch order, each
        # held by the rank whose conversation it came from
        kidx = torch.nonzero(ins).flatten()
        K = int(kidx.numel())
        if K == 0:
            return
        base = self.next_id
        self.next_id += K
        stats["inserted"] += K
        new_num = torch.full((F,), -1, dtype=torch.long, device=dev)
        new_num[kidx] = torch.arange(base + 1, base + K + 1, dtype=torch.long, device=dev)
        mk = kidx[origin[kidx] == self.rank]
        row_of_fact = torch.full((F,), -1, dtype=torch.long, device=dev)
        if mk.numel():
            mkh = mk.cpu().numpy()
            nums_h = new_num[mk].cpu().numpy()
            lf = [flat[int(i) - f_off] for i in mkh]
            with tracer.stage("sc_insert", dev):
                rows = g.add_nodes(self._ids_of_nums(nums_h), [f["content"] for f in lf], Q[mk],
                                   shard=codes[mkh], types=[f.get("type", "semantic") for f in lf],
                                   sal=sal_new[mk].float(), acc=acc_new[mk], now=now, stored=True)
            self._sync_num()
            self.num[rows] = new_num[mk]
            self.holder[rows] = self.rank
            row_of_fact[mk] = rows.to(dev)
            self._reach_add(rows)
        if self.local.query_cache:
            self.local.query_cache.invalidate_results()

        # ---- 7. links (global node numbers), kept where this rank holds the source
        with tracer.stage("sc_link", dev):
            plan, _ = batch_link_plan(kidx, new_num, code_t, ct, S, earlier, (ws, wm[:, :, 0]),
                                      (gs, gm[:, :, 0]), keep, B, thr, stats)
            if plan is not None:
                self._apply_edges(plan, new_num, row_of_fact, origin, code_t, (gm, wm), now)

        # ---- 8. the reference hierarchy at the batch end (the single
        # process's coarse path: a shard's super-node over all its members)
        if self.ref_hierarchy:
            with tracer.stage("sc_supers", dev):
                self._make_supers_batch(codes[kidx.cpu().numpy()].tolist(), Q, now)

    def _super_heads(self, qn, gs, gm, srows, scos, sn2):
        """Per fact: whether the best super-node by the store's L2 score
        (2 |q| |x| cos - |x|^2) beats the merged global head, that
        super-node's global row and cosine (a tie: the lower row, as in the
        single process's ``_scan_batch``). The head's |x|^2 (fp32 column)
        comes from its holder (one all-reduce of F doubles)."""
        g = self.g
        dev = self.device
        F = gs.shape[0]
        sc_t = torch.as_tensor(scos, dtype=torch.float64).to(dev)
        n2_t = torch.as_tensor(sn2, dtype=torch.float64).to(dev)
        q = qn.reshape(-1).to(dev, torch.float64)
        l2s = 2.0 * q[:, None] * n2_t.sqrt()[None, :] * sc_t - n2_t[None, :]
        j = torch.argmax(l2s, 1)  # first maximum: the lowest super row on a tie
        sl2 = l2s.gather(1, j[:, None])[:, 0]
        sv = torch.as_tensor(srows, dtype=torch.long).to(dev)[j]
        hr = gm[:, 0, 3]
        mine = (gm[:, 0, 2] == self.rank) & (hr >= 0)
        hn2 = torch.zeros(F, dtype=torch.float64, device=dev)
        if bool(mine.any()):
            with g.on_stream():
                hn2[mine] = g.sqn[hr[mine]].double()
        if self._coll:
            hn2 = self.comm.all_reduce(self._to_comm(hn2)).to(dev)
        hv = gm[:, 0, 0] - 1
        hs = gs[:, 0].to(dev, torch.float64)
        hl2 = torch.where(hv >= 0, 2.0 * q * hs * hn2.sqrt() - hn2, torch.full_like(hs, NEG_INF))
        win = (sl2 > hl2) | ((sl2 == hl2) & (sv < hv))
        return win, torch.where(win, sv, torch.full_like(sv, -1)), sc_t.gather(1, j[:, None])[:, 0]

    def _make_supers_batch(self, kept_codes: List[int], Q: torch.Tensor, now: float) -> None:
        """Batch cadence: a super-node for every shard of the batch's kept
        facts (first-seen order) that passed ``super_node_threshold`` members
        and has none (reference memory_system.py:775-780, 893-933). Collective."""
        g = self.g
        dev = self.device
        order = list(dict.fromkeys(int(c) for c in kept_codes))
        if not order:
            return
        _, _, _, have = self._stored_supers(torch.zeros((0, g.dim), dtype=torch.float64, device=dev))
        have = set(have)
        sc = torch.as_tensor(g.shard_count, dtype=torch.int64).to(dev)
        if self._coll:
            sc = self.comm.all_reduce(self._to_comm(sc)).to(dev)
        sc = sc.cpu().tolist()
        for code in order:
            if sc[code] <= self.super_node_threshold or code in have:
                continue
            children = self._pre_members(code)
            info = self._super_mean(children, np.zeros(0, np.int64), Q, BIG, np.zeros(0, np.int64), [], 0)
            if info is None:
                continue
            sp = {"code": code, "key": int(self.next_id), "children": children}
            self.next_id += 1
            self._sup_v = np.union1d(self._sup_v, np.asarray([sp["key"]], np.int64))
            self._insert_super(sp, info, now)
            have.add(code)

    def _apply_edges(self, plan, new_num, row_of_fact, origin, code_t, hits, now) -> None:
        """Append the planned edges whose source this rank holds; an endpoint
        held elsewhere becomes (or reuses) a ghost row with its id and shard."""
        g = self.g
        dev = self.device
        Sn, Dn, W, H = plan
        base = int(new_num[new_num >= 0].min()) if bool((new_num >= 0).any()) else 0
        # source = a new node: its fact position = kept index
        kept = torch.nonzero(new_num >= 0).flatten()
        src_fact = kept[Sn - base]
        mine = origin[src_fact] == self.rank
        if not bool(mine.any()):
            return
        src_fact, Dn, W, H = src_fact[mine], Dn[mine], W[mine], H[mine]
        src_rows = row_of_fact[src_fact]
        # destination: a new node of this batch (its fact tells the holder and
        # shard) or an existing node from the merged candidate lists
        is_new = Dn >= base
        dst_rows = torch.full_like(Dn, -1)
        dst_shard = torch.full_like(Dn, -1)
        dst_hold = torch.full_like(Dn, -1)
        dst_fact = kept[(Dn - base).clamp_min(0).clamp_max(max(kept.numel() - 1, 0))]
        nf = is_new & (origin[dst_fact] == self.rank)
        dst_rows = torch.where(nf, row_of_fact[dst_fact], dst_rows)
        dst_shard = torch.where(is_new, code_t[dst_fact].long(), dst_shard)
        dst_hold = torch.where(is_new, origin[dst_fact], dst_hold)
        # existing nodes: (number -> shard, holder, row) from the candidate lists
        metas = torch.cat([h.reshape(-1, 4) for h in hits])
        metas = metas[metas[:, 0] >= 0]
        if metas.numel():
            un, first = np.unique(metas[:, 0].cpu().numpy(), return_index=True)
            info = metas[torch.as_tensor(first, dtype=torch.long).to(dev)]
            un_t = torch.as_tensor(un).to(dev)
            pos = torch.searchsorted(un_t, Dn.clamp_max(int(un[-1])))
            hit = (~is_new) & (un_t[pos.clamp_max(un_t.numel() - 1)] == Dn)
            pi = info[pos.clamp_max(un_t.numel() - 1)]
            dst_shard = torch.where(hit, pi[:, 1], dst_shard)
            dst_hold = torch.where(hit, pi[:, 2], dst_hold)
            dst_rows = torch.where(hit & (pi[:, 2] == self.rank), pi[:, 3], dst_rows)
        # remote endpoints -> ghost rows (created once per id)
        need = torch.nonzero(dst_rows < 0).flatten()
        if need.numel():
            dn_h = Dn[need].cpu().numpy()
            sh_h = dst_shard[need].cpu().numpy()
            ho_h = dst_hold[need].cpu().numpy()
            ids = self._ids_of_nums(dn_h)
            have = [g.row_of.get(i, -1) for i in ids]
            fresh = {}
            for i, r, x, s_, h_ in zip(ids, have, dn_h.tolist(), sh_h.tolist(), ho_h.tolist()):
                if r < 0 and i not in fresh:
                    fresh[i] = (s_, h_, x)
            if fresh:
                fid = list(fresh)
                rows_new = g.add_nodes(fid, [""] * len(fid), None, shard=[fresh[i][0] for i in fid], ghost=True,
                                       stored=False, now=now)
                self._sync_num()
                self.num[rows_new] = torch.as_tensor([fresh[i][2] for i in fid], dtype=torch.long).to(dev)
                self.holder[rows_new] = torch.as_tensor([fresh[i][1] for i in fid], dtype=torch.long).to(dev)
            rr = torch.as_tensor([g.row_of[i] for i in ids], dtype=torch.long).to(dev)
            dst_rows[need] = rr
        g.append_edges(src_rows, dst_rows, W.float(), H.to(torch.int32), g.etype("relates_to"), now=now)

    # ------------------------------------------------------------------ reference cadence
    def _vrows(self, rows: torch.Tensor) -> torch.Tensor:
        """Global row number of local rows: node number - 1 -- the row the
        node has in a single process holding the union (nodes only, numbered
        in creation order), so every order key equals the single process's."""
        return torch.where(rows >= 0, self.num[rows.clamp_min(0)] - 1, torch.full_like(rows, -1))

    def _held_rows(self, vrows: torch.Tensor) -> torch.Tensor:
        """Local row of each global row this rank HOLDS live (-1 elsewhere:
        not here, a ghost, or gone)."""
        return self._rows_of_nums(vrows, held=True, add=1)

    def _merge_lists(self, s: torch.Tensor, v: torch.Tensor, k: int):
        """Per fact: top-k of the gathered (score, global row) entries by
        (score desc, row asc); -1 rows last (the single process's order)."""
        key = torch.where(v >= 0, v, torch.full_like(v, BIG))
        o = torch.argsort(key, dim=1, stable=True)
        s, v = torch.gather(s, 1, o), torch.gather(v, 1, o)
        o = torch.sort(s, dim=1, descending=True, stable=True).indices[:, :k]
        s, v = torch.gather(s, 1, o), torch.gather(v, 1, o)
        return s, torch.where(torch.isneginf(s), torch.full_like(v, -1), v)

    def _gather_lists(self, s: torch.Tensor, v: torch.Tensor, k: int):
        F = s.shape[0]
        if self._coll:
            s = self._gather_rows(s.contiguous()).view(self.world, F, k).permute(1, 0, 2).reshape(F, -1)
            v = self._gather_rows(v.contiguous()).view(self.world, F, k).permute(1, 0, 2).reshape(F, -1)
        return self._merge_lists(s, v, k)

    def _exact_lists(self, Q: torch.Tensor, code_t: torch.Tensor, K: int, pf: Optional[Dict] = None):
        """The planner's candidate lists: every fact's global and same-shard
        top-K over every rank's live nodes (the same fused scan + float64
        re-rank per rank, merged by global row). Returns numpy
        ((gs, gv), (ws, wv)), rows as global row numbers. ``pf``: this batch
        was prefetched (:meth:`_launch_prefetch`) -- the facts the scan took
        (those that could reach this rank's rows then) complete it against
        the rows now (TenantGraph.cos_topk_finish); the others could reach
        none of the older rows and look at the rows added since only."""
        g = self.g
        F = Q.shape[0]
        dev = self.device
        live = g.num_nodes() if g.n else 0
        gs = ws = torch.full((F, K), NEG_INF, dtype=torch.float64, device=dev)
        gv = wv = torch.full((F, K), -1, dtype=torch.long, device=dev)
        if pf is not None and pf.get("si") is not None and live:
            si, h, n0 = pf["si"], pf["h"], pf["n0"]
            n = g.n
            mask = (g.kind[:n] == NODE) & (g.sup[:n] == 0) & (self.holder[:n] == self.rank)
            self.last_scan_work = int(si.numel()) * live
            self.scan_work += self.last_scan_work
            gs, ws = gs.clone(), ws.clone()
            gv, wv = gv.clone(), wv.clone()
            with g.on_stream():
                if h is not None:
                    (a, ar), (b, br) = g.cos_topk_finish(h, K, mask)
                    gs[si], ws[si] = a.double(), b.double()
                    gv[si], wv[si] = self._vrows(ar), self._vrows(br)
                rest = torch.ones(F, dtype=torch.bool, device=dev)
                rest[si] = False
                ri = torch.nonzero(rest).flatten()
                if ri.numel() and n > n0:
                    (a, ar), (b, br) = g.cos_topk_new_rows(Q[ri], K, mask, n0, code_t[ri], LINK_THRESHOLD)
                    gs[ri], ws[ri] = a.double(), b.double()
                    gv[ri], wv[ri] = self._vrows(ar), self._vrows(br)
            (gs, gv), (ws, wv) = self._gather_lists(gs, gv, K), self._gather_lists(ws, wv, K)
            return ((gs.cpu().numpy(), gv.cpu().numpy()), (ws.cpu().numpy(), wv.cpu().numpy()))
        sel = None
        if live:
            Qd = Q.double()
            qn = Qd.norm(dim=1, keepdim=True)
            sel = self._reach_mask(Qd / torch.where(qn > 0, qn, torch.ones_like(qn)))
        n_scan = F if sel is None else int(sel.sum())
        self.last_scan_work = n_scan * live
        self.scan_work += self.last_scan_work
        if live and n_scan:
            n = g.n
            mask = (g.kind[:n] == NODE) & (g.sup[:n] == 0) & (self.holder[:n] == self.rank)
            si = torch.arange(F, device=dev) if sel is None else torch.nonzero(sel).flatten()
            with g.on_stream():
                (a, ar), (b, br) = g.cos_topk(Q[si], K, mask, dual_label=code_t[si], min_score=LINK_THRESHOLD)
            gs, ws = gs.clone(), ws.clone()
            gv, wv = gv.clone(), wv.clone()
            gs[si], ws[si] = a.to(dev).double(), b.to(dev).double()
            gv[si], wv[si] = self._vrows(ar.to(dev)), self._vrows(br.to(dev))
        (gs, gv), (ws, wv) = self._gather_lists(gs, gv, K), self._gather_lists(ws, wv, K)
        return ((gs.cpu().numpy(), gv.cpu().numpy()), (ws.cpu().numpy(), wv.cpu().numpy()))

    def _exact_pool(self, B: int, P: int, now: float):
        """This rank's part of the eviction pool (its P lowest rows by
        importance now and after all B decays, as the single process picks
        over the union) -> (global pool rows, local mask or None when every
        evictable row here is in it)."""
        from ..core.consolidation import _lowest_keys
        g = self.g
        n = g.n
        dev = self.device
        local = torch.zeros(0, dtype=torch.long, device=dev)
        mask = None
        if n:
            with g.on_stream():
                held = (self.holder[:n] == self.rank).to(torch.uint8)
                kind = torch.where(held.bool(), g.kind[:n], torch.zeros_like(g.kind[:n]))
                imp0 = T.importance(g.sal[:n], g.acc[:n], g.last[:n], kind, g.sup[:n], now)
                nev = int(torch.isfinite(imp0).sum())
                if P >= nev:
                    local = torch.nonzero(torch.isfinite(imp0)).flatten()
                else:
                    sal = g.sal[:n].clone()
                    empty = {"src": torch.zeros(0, dtype=torch.int32, device=dev),
                             "dst": torch.zeros(0, dtype=torch.int32, device=dev),
                             "w": torch.zeros(0, dtype=torch.float32, device=dev)}
                    T.decay_prune(empty, sal, kind, g.sup[:n], DECAY_RATE, None, steps=B)
                    impB = T.importance(sal, g.acc[:n], g.last[:n], kind, g.sup[:n], now)
                    okey = g.shard[:n].long() * (1 << NUM_BITS) + self._vrows(torch.arange(n, device=dev))
                    mask = torch.zeros(n, dtype=torch.uint8, device=dev)
                    for imp in (imp0, impB):
                        mask[_lowest_keys(imp, okey, P)] = 1
                    local = torch.nonzero(mask).flatten()
        pv, _ = self._gather_var(self._vrows(local))
        return torch.unique(pv).cpu().numpy().astype(np.int64), mask

    def _row_states(self, want: np.ndarray):
        """State (sal, acc, last, shard, super, |x|^2) and holder of global
        rows ``want`` (sorted unique), each supplied by the rank holding it."""
        g = self.g
        dev = self.device
        wt = torch.as_tensor(want, dtype=torch.long).to(dev)
        r = self._held_rows(wt)
        mine = torch.nonzero(r >= 0).flatten()
        rr = r[mine]
        with g.on_stream():
            blk = torch.stack([wt[mine].double(), g.sal[rr].double(), g.acc[rr].double(), g.last[rr].double(),
                               g.shard[rr].double(), g.sup[rr].double(), g.sqn[rr].double(),
                               torch.full_like(rr, self.rank).double()], 1) if mine.numel() else \
                torch.zeros((0, 8), dtype=torch.float64, device=dev)
        allb, _ = self._gather_var(blk)
        allb = allb[torch.argsort(allb[:, 0])] if allb.numel() else allb
        a = allb.cpu().numpy()
        rows = a[:, 0].astype(np.int64)
        cols = (a[:, 1].astype(np.float32), a[:, 2].astype(np.int64), a[:, 3], a[:, 4].astype(np.int64),
                a[:, 5] != 0, a[:, 6])
        return rows, cols, dict(zip(rows.tolist(), a[:, 7].astype(np.int64).tolist()))

    # ------------------------------------------------------------------ reference hierarchy
    def _stored_supers(self, Qn: torch.Tensor):
        """The tenant's super-nodes as the batch planner sees them (the single
        process's ``_plan_inputs``): global rows (ascending), every fact's
        cosine with each (fp32 row, |x| from the stored |x|^2), their |x|^2,
        and the shard codes that have one. Collective (one variable-length
        gather of a few rows); refreshes the id map."""
        g = self.g
        dev = self.device
        F = int(Qn.shape[0])
        n = g.n
        st = torch.zeros(0, dtype=torch.long, device=dev)
        if n and g.n_super:
            with g.on_stream():
                st = torch.nonzero((g.kind[:n] == NODE) & (g.sup[:n] != 0)
                                   & (self.holder[:n] == self.rank)).flatten()
        blk = torch.zeros((st.numel(), 3 + F), dtype=torch.float64, device=dev)
        if st.numel():
            with g.on_stream():
                X = g.emb32[st].double()
                sq = g.sqn[st].double()
                nrm = sq.sqrt()
                blk[:, 0] = self._vrows(st).double()
                blk[:, 1] = g.shard[st].double()
                blk[:, 2] = sq
                if F:
                    blk[:, 3:] = ((Qn @ X.T) / torch.where(nrm > 0, nrm, torch.ones_like(nrm))[None, :]).T
        allb, _ = self._gather_var(blk)
        a = allb.cpu().numpy()
        if a.shape[0]:
            a = a[np.argsort(a[:, 0], kind="stable")]
        rows = a[:, 0].astype(np.int64)
        self._sup_v = np.union1d(self._sup_v, rows)
        cos = np.ascontiguousarray(a[:, 3:].T) if F else np.zeros((0, rows.size))
        return rows, cos, a[:, 2].copy(), sorted(set(a[:, 1].astype(np.int64).tolist()))

    def _pre_members(self, code: int) -> np.ndarray:
        """Global rows (ascending) of shard ``code``'s live non-super nodes
        over every rank -- the planner's ``pre_members`` callback (collective:
        every rank's planner calls it at the same point)."""
        g = self.g
        n = g.n
        v = torch.zeros(0, dtype=torch.long, device=self.device)
        if n:
            with g.on_stream():
                m = (g.kind[:n] == NODE) & (g.sup[:n] == 0) & (g.shard[:n] == int(code)) & \
                    (self.holder[:n] == self.rank)
                v = self._vrows(torch.nonzero(m).flatten())
        allv, _ = self._gather_var(v)
        return np.sort(allv.cpu().numpy().astype(np.int64))

    def _super_mean(self, children: np.ndarray, new_facts: np.ndarray, Q: torch.Tensor, n0: int,
                    origin_h: np.ndarray, flat, f_off: int) -> Optional[Dict]:
        """A planned super-node's mean embedding, holder and the contents of
        its first three children (collective). ``children``: global rows, the
        pre-batch ones (< n0, held anywhere) first, then batch facts
        ``new_facts`` (rows of ``Q``). Every rank sums the fp32 rows it holds
        in float64; the per-rank sums are all-gathered and added in rank
        order, so every rank gets the same mean (the single process sums all
        rows in one pass: the fp32 mean agrees with its to rounding). Holder:
        the rank holding the most children (the lowest on a tie)."""
        g = self.g
        dev = self.device
        D = g.dim
        ch = np.asarray(children, np.int64)
        nf = np.asarray(new_facts, np.int64)
        pre = ch[ch < n0]
        part = torch.zeros((1, D + 1), dtype=torch.float64, device=dev)
        n_held = 0
        if pre.size and g.n:
            loc = self._held_rows(torch.as_tensor(pre).to(dev))
            loc = loc[loc >= 0]
            n_held = int(loc.numel())
            if n_held:
                with g.on_stream():
                    part[0, :D] = g.emb32[loc].double().sum(0)
        if nf.size:
            n_held += int((origin_h[nf] == self.rank).sum())
        part[0, D] = float(n_held)
        allp = self._gather_rows(part)
        tot = allp[0, :D].clone()
        for r in range(1, allp.shape[0]):
            tot += allp[r, :D]
        cnt = int(pre.size + nf.size)
        if nf.size:
            tot += Q[torch.as_tensor(nf, dtype=torch.long).to(Q.device)].to(dev).double().sum(0)
        # first three children's contents, from the rank that has each
        txt = {}
        head = ch[:3]
        hp = head[head < n0]
        if hp.size and g.n:
            lr = self._held_rows(torch.as_tensor(hp).to(dev)).cpu().tolist()
            for i, r in enumerate(lr):
                if r >= 0:
                    txt[i] = g.content[r]
        for i in range(int(hp.size), int(head.size)):
            j = int(nf[i - int(pre.size)])
            if int(origin_h[j]) == self.rank:
                txt[i] = flat[j - f_off]["content"]
        if self._coll:
            for part_ in self.comm.all_gather_object(txt):
                txt.update(part_)
        if cnt == 0:
            return None
        return {"emb": (tot / cnt).float(), "holder": int(torch.argmax(allp[:, D]).item()),
                "contents": [txt[i] for i in range(int(head.size))]}

    def _insert_super(self, sp: Dict, info: Dict, now: float, sal: float = 0.5, acc: int = 0,
                      last: Optional[float] = None) -> None:
        """Apply one planned super-node on every rank (reference
        memory_system.py:893-933): its holder adds the row -- id
        ``super_<shard>_<int(now)>``, the "Topic: ..." summary of the first
        three children, the mean embedding, every child's id; unstored -- and
        every rank holding children points their parent at it (a ghost row of
        the super-node where it is held elsewhere)."""
        g = self.g
        dev = self.device
        code = int(sp["code"])
        key = int(sp["key"])
        skey = g.shard_names[code]
        children = np.asarray(sp["children"], np.int64)
        sid = f"super_{skey}_{int(now)}"
        h = int(info["holder"])
        held = torch.zeros(0, dtype=torch.long, device=dev)
        if children.size and g.n:
            loc = self._held_rows(torch.as_tensor(children).to(dev))
            held = loc[loc >= 0]
        srow = -1
        if self.rank == h:
            summary = f"Topic: {skey}. Contains memories about: " + "; ".join(info["contents"])
            rows = g.add_nodes([sid], [summary], info["emb"][None, :], shard=[code], sup=[1],
                               children={0: self._ids_of_nums(children + 1)}, stored=False, sal=float(sal),
                               acc=int(acc), last=float(now if last is None else last), now=now)
        elif held.numel() and g.row_of.get(sid, -1) < 0:
            rows = g.add_nodes([sid], [""], None, shard=[code], sup=[1], ghost=True, stored=False, now=now)
        else:
            rows = None
        if rows is not None:
            srow = int(rows[0])
            self._sync_num()
            self.num[srow] = key + 1
            self.holder[srow] = h
        elif held.numel():
            srow = int(g.row_of[sid])
        if held.numel():
            with g.on_stream():
                g.parent[held] = srow
                g.dirty[held] = 1
            g._bump()

    def _gather_batch(self, flat, conv, E, B_loc) -> Dict:
        """Step 1 of :meth:`_consolidate_exact` (collective): the global fact
        batch in rank-major conversation order -- fact vectors, saliences,
        conversation indices, shard codes (registered in fact order), the
        rank that will hold each fact's node and the facts' contents where
        holders need them."""
        dev = self.device
        comm = self.comm
        with tracer.stage("sc_gather", dev):
            bl = self._host_ints(B_loc)[:, 0].tolist()
            B = int(sum(bl))
            c_off = int(sum(bl[: self.rank]))
            keys = [self.local._fact_shard_key(f) for f in flat]
            keys_all = [k for ks in comm.all_gather_object(keys) for k in ks] if self._coll else keys
            sal_l = torch.tensor([float(f.get("salience", 0.5)) for f in flat], dtype=torch.float32, device=dev)
            ct_l = torch.tensor(conv, dtype=torch.long, device=dev) + c_off
            Qa, fcnt = self._gather_var(E)
            sal_in, _ = self._gather_var(sal_l)
            ct, _ = self._gather_var(ct_l)
        F = int(Qa.shape[0])
        gb = {"B": B, "F": F}
        if B == 0:
            return gb
        origin = torch.repeat_interleave(torch.arange(self.world, device=dev),
                                         torch.tensor(fcnt, dtype=torch.long, device=dev)) if F else \
            torch.zeros(0, dtype=torch.long, device=dev)
        codes = self._register_shards(keys_all).astype(np.int64)
        code_t = torch.as_tensor(codes).to(dev)
        Q = Qa.float()
        Qd = Q.double()
        qn = Qd.norm(dim=1, keepdim=True)
        Qn = Qd / torch.where(qn > 0, qn, torch.ones_like(qn))
        if F:
            origin_conv = origin
            origin = self._holders(Qn, origin_conv)
            if origin is not origin_conv:  # holders need the contents of facts from other ranks
                flat = [f for part in comm.all_gather_object([{"content": f["content"],
                                                               "type": f.get("type", "semantic")} for f in flat])
                        for f in part]
                f_off = 0
            else:
                f_off = int(sum(fcnt[: self.rank]))
        else:
            f_off = 0
        gb.update(Q=Q, Qn=Qn, qn=qn, code_t=code_t, codes=codes, origin=origin, flat=flat, f_off=f_off,
                  sal_in=sal_in, ct=ct)
        return gb

    _prefetch_next = None
    _prefetched = None
    prefetched_batches = 0  # batches whose gather + local scan ran under the previous batch's apply

    def consolidate_stream(self, batches, cadence: str = "conversation", commit: str = "batch"):
        """Collective :meth:`consolidate_batch` over a stream of batches
        (every rank passes its own, the same number), yielding each batch's
        counts -- exactly the per-batch calls' results. As in
        ``MemorySystem.consolidate_stream``, batch i+1 is gathered and this
        rank's candidate scan of it launched on a side stream once batch i is
        planned; the scan runs under batch i's apply and batch i+1 completes
        it against the rows batch i left. ``batches`` yields
        ``(conversations, embeddings)`` or ``(conversations, embeddings,
        now)``."""
        it = iter(batches)
        cur = next(it, None)
        try:
            while cur is not None:
                nxt = next(it, None)
                self._prefetch_next = nxt
                now = cur[2] if len(cur) > 2 else None
                yield self.consolidate_batch(cur[0], embeddings=cur[1], now=now, cadence=cadence, commit=commit)
                cur = nxt
        finally:
            self._prefetch_next = None
            self._prefetched = None

    def _prep_facts(self, conversations, embeddings):
        """consolidate_batch's local fact preparation: (flat, conv, E)."""
        dev = self.device
        flat, conv, idx = [], [], []
        j = 0
        for c, fs in enumerate(conversations):
            for f in fs:
                if isinstance(f, dict) and f.get("content") and len(f["content"]) >= MIN_FACT_LEN:
                    flat.append(f)
                    conv.append(c)
                    idx.append(j)
                j += 1
        m = len(flat)
        if embeddings is not None and m:
            E = embeddings if torch.is_tensor(embeddings) else torch.as_tensor(np.asarray(embeddings, np.float32))
            E = E[torch.as_tensor(idx, dtype=torch.long).to(E.device)] if len(idx) != len(E) else E
        elif m:
            with tracer.stage("embed_facts", dev):
                E = self.local._batch_embed_any([f["content"] for f in flat])
        else:
            E = None
        if m:
            E, valid = self.local._fact_matrix(E, m)
            vidx = np.nonzero(valid)[0]
            flat = [flat[i] for i in vidx]
            conv = [conv[i] for i in vidx]
            E = E[torch.as_tensor(vidx, dtype=torch.long).to(E.device)].to(dev, torch.float32)
        return flat, conv, E

    def _launch_prefetch(self, pl: Dict) -> None:
        """After batch i's plan (collective: the same point on every rank):
        gather batch i+1 and launch this rank's candidate scan of it on a
        side stream (see :meth:`consolidate_stream`). Not when batch i runs a
        cluster pass (it moves the cluster homes that decide the holders, and
        shares the scan workspaces) or off the GPU -- conditions every rank
        evaluates alike -- and when any rank's next batch has no embeddings
        or the wrong width: those are per-rank, so they are summed over the
        ranks first (one host all-reduce) and every rank skips or runs the
        prefetch's collectives together."""
        from ..core.consolidation import _prefetch_stream
        nxt, self._prefetch_next = self._prefetch_next, None
        self._prefetched = None
        g = self.g
        if not g.on_gpu or g.dim is None or any(seg["cluster"] for seg in pl["segments"]):
            return
        skip = nxt is None or nxt[1] is None
        flat, conv, E = ([], [], None) if skip else self._prep_facts(nxt[0], nxt[1])
        if E is None:
            E = torch.zeros((0, g.dim), dtype=torch.float32, device=self.device)
        n_skip, n_bad = self._sum(int(skip), int(E.shape[1] != g.dim))
        if n_skip or n_bad:
            return
        gb = self._gather_batch(flat, conv, E, len(nxt[0]))
        pf = {"src": nxt[1], "B_loc": len(nxt[0]), "m": len(flat), "gb": gb, "h": None, "si": None, "n0": g.n}
        F = gb["F"]
        K = self.local.BATCH_LIST_K
        if F and g.n and g.dual_prefetch_ok(F, K):
            ps = pl["stats"]
            g.reserve(g.n + int(ps["inserted"]) + len(pl["supers"]) + F + 16)  # ghost rows too: no column moves
            sel = self._reach_mask(gb["Qn"])
            si = torch.arange(F, device=self.device) if sel is None else torch.nonzero(sel).flatten()
            n = g.n
            pf["si"], pf["n0"] = si, n
            if si.numel():
                with g.on_stream():
                    mask = (g.kind[:n] == NODE) & (g.sup[:n] == 0) & (self.holder[:n] == self.rank)
                    pf["h"] = g.cos_topk_prefetch(gb["Q"][si], mask, gb["code_t"][si], LINK_THRESHOLD,
                                                  _prefetch_stream(self.device))
        self._prefetched = pf

    def _consolidate_exact(self, flat, conv, E, B_loc, now, stats) -> None:
        """The reference cadence over the row-sharded buffer: every rank runs
        the SAME native batch planner (core/batch_plan.py) on the global
        inputs -- all-gathered facts, candidate lists merged over the ranks by
        global row, the eviction pool as the union of every rank's lowest
        rows, the touched rows' state from their holders -- so every decision
        of the B conversations is known everywhere without further exchange
        (the planner's exact-fallback callback is itself collective and runs
        at the same point on every rank). The plan is applied in segments:
        each rank applies what it holds (decay, row updates, inserts of the
        facts it will hold, the edges whose source it holds, its victims),
        and the collective ``run_consolidation`` / cluster pass run at the
        segment ends, as in the single-process engine. The eviction pool is
        verified on every rank (tg_evict_verify_kernel keyed by global row)."""
        from ..core.batch_plan import PoolTooSmall, plan
        g = self.g
        dev = self.device
        keep = 1.0 - DECAY_RATE
        thr = self.prune_threshold if self.auto_prune else None
        K = self.local.BATCH_LIST_K
        # ---- 1. the global fact batch (rank-major conversation order)
        pf, self._prefetched = self._prefetched, None
        ok = pf is not None and pf["src"] is getattr(self, "_batch_src", None) and pf["B_loc"] == B_loc \
            and pf["m"] == len(flat)
        if pf is not None and self._sum(0 if ok else 1)[0]:  # every rank uses its prefetch, or none does
            pf = None
        gb = pf["gb"] if pf is not None else self._gather_batch(flat, conv, E, B_loc)
        self.prefetched_batches += pf is not None
        B, F = gb["B"], gb["F"]
        stats["conversations"] = B
        stats["facts"] = F
        if B == 0:
            return
        Q, Qn, qn, code_t, codes = gb["Q"], gb["Qn"], gb["qn"], gb["code_t"], gb["codes"]
        origin, flat, f_off, sal_in, ct = gb["origin"], gb["flat"], gb["f_off"], gb["sal_in"], gb["ct"]
        # ---- 2. candidate lists + the fact x fact block (the single process's formulas)
        with tracer.stage("sc_scan", dev):
            if F and g.dim is not None:
                glob, shard = self._exact_lists(Q, code_t, K, pf=pf)
            else:
                e = (np.full((F, K), NEG_INF), np.full((F, K), -1, np.int64))
                glob, shard = e, e
            if F:
                X = Q.double()
                nrm = (X * X).sum(1).float().double().sqrt()
                S = _host_pinned(self, "_pin_S", (Qn @ X.T) / torch.where(nrm > 0, nrm, torch.ones_like(nrm))[None, :])
                qnorm = qn.flatten().cpu().numpy()
                fact_n2 = (X * X).sum(1).float().double().cpu().numpy()
            else:
                S, qnorm, fact_n2 = np.zeros((0, 0)), np.zeros(0), np.zeros(0)

        def fallback(j, evicted, same_shard):  # collective: every rank calls it at the same point
            n = g.n
            s_ = torch.full((1, K), NEG_INF, dtype=torch.float64, device=dev)
            v_ = torch.full((1, K), -1, dtype=torch.long, device=dev)
            if n and g.dim is not None:
                m = (g.kind[:n] == NODE) & (g.sup[:n] == 0) & (self.holder[:n] == self.rank)
                ev = np.asarray(evicted, np.int64)
                if ev.size:
                    er = self._held_rows(torch.as_tensor(ev).to(dev))
                    er = er[er >= 0]
                    if er.numel():
                        m = m.clone()
                        m[er] = False
                with g.on_stream():
                    if same_shard:
                        a, ar = g._exact_cos(Qn[j:j + 1], m, K, row_label=g.shard[:n],
                                             q_label=code_t[j:j + 1])
                    else:
                        a, ar = g._exact_cos(Qn[j:j + 1], m, K)
                s_, v_ = a.to(dev).double(), self._vrows(ar.to(dev))
            s_, v_ = self._gather_lists(s_, v_, K)
            return s_[0].cpu().numpy(), v_[0].cpu().numpy()

        # ---- the reference hierarchy: stored super-nodes, collective member /
        # mean callbacks for the ones the plan creates
        n0 = int(self.next_id)
        origin_h = origin.cpu().numpy() if F else np.zeros(0, np.int64)
        self._super_plan = {}
        if self.ref_hierarchy:
            sup_rows, sup_cos, sup_n2, super_codes = self._stored_supers(Qn)
        else:
            sup_rows, sup_cos, sup_n2, super_codes = np.zeros(0, np.int64), np.zeros((F, 0)), np.zeros(0), []

        def super_cos(children, new_facts):  # collective, like fallback
            ch = np.asarray(children, np.int64)
            info = self._super_mean(ch, new_facts, Q, n0, origin_h, flat, f_off)
            if info is None:
                return np.full(F, NEG_INF), 1.0
            self._super_plan[tuple(ch.tolist())] = info
            ed = info["emb"].double()
            n2 = float((ed * ed).sum().float())
            en = n2 ** 0.5
            return (((Qn @ ed) / (en if en > 0 else 1.0)).cpu().numpy() if F else np.zeros(0)), n2

        # ---- 3. plan (identical on every rank), eviction pool verified everywhere
        tot = self._sum(g.num_nodes(), *g.shard_count)  # every rank registered the same shards
        node_count, shard_count = tot[0], tot[1:]
        excess0 = max(0, node_count - self.max_buffer_size)
        P = 4 * (F + excess0) + 1024  # per rank (a rank with fewer evictable rows pools them all)
        cl_every = int(self.hierarchy_params["every"]) if self.hierarchy_params else 0
        ct_np = ct.cpu().numpy().astype(np.int64)
        sal_np = sal_in.cpu().numpy().astype(np.float32)
        while True:
            with tracer.stage("sc_pool", dev):
                pool, pmask = self._exact_pool(B, P, now)
                want = np.unique(np.concatenate([pool, glob[1][glob[1] >= 0], shard[1][shard[1] >= 0], sup_rows]))
                rows_v, cols, holder_of = self._row_states(want)
            kw = dict(ct=ct_np, code=codes, sal_in=sal_np, n0=n0, node_count=node_count, shard_count=shard_count,
                      super_codes=super_codes, pre_members=self._pre_members, max_buffer=self.max_buffer_size,
                      super_threshold=self.super_node_threshold, ref_hierarchy=self.ref_hierarchy,
                      prune_thr=thr, keep=keep, now=now, pool=pool, rows=rows_v, cols=cols, glob=glob, shard=shard,
                      sup_rows=sup_rows, sup_cos=sup_cos, sup_n2=sup_n2, qnorm=qnorm,
                      fact_n2=fact_n2, S=S, super_cos=super_cos, fallback=fallback)
            with tracer.stage("cb_plan", "cpu"):
                pl = plan(kw, B, self.conversation_count, self.auto_consolidate, self.consolidate_every, cl_every,
                          native=self.local.NATIVE_PLANNER, seg_each=self._commit_each)
            with tracer.stage("cb_verify", dev):
                ok = True
                if pmask is not None and pl["events"]:
                    n = g.n
                    with g.on_stream():
                        ok = T.evict_verify(g.sal[:n], g.acc[:n], g.last[:n], g.kind[:n], g.sup[:n], g.shard[:n],
                                            pmask, now, keep, pl["events"],
                                            rowkey=self._vrows(torch.arange(n, device=dev)))
                bad, partial = self._sum(0 if ok else 1, 0 if pmask is None else 1)
            if bad == 0:
                break
            if partial == 0:
                raise PoolTooSmall("eviction plan failed verification with every row in the pool")
            stats["pool_retries"] = stats.get("pool_retries", 0) + 1
            P = 4 * P
        ps = pl["stats"]
        for k_ in ("dup", "inserted", "linked", "cross_links", "evicted", "fallbacks"):
            stats[k_] += int(ps[k_])
        if self._prefetch_next is not None:
            with tracer.stage("sc_prefetch", dev):
                self._launch_prefetch(pl)
        pruned = int(ps["pruned_new"])
        fact_key = np.asarray(pl["fact_key"], np.int64)
        supers = pl["supers"]
        if supers:  # node ids of the batch's facts skip the super-node rows
            self._sup_v = np.union1d(self._sup_v, np.asarray([int(sp["key"]) for sp in supers], np.int64))
        # new rows: holder and shard (the ghost rows of edges need them)
        for j in np.nonzero(fact_key >= 0)[0].tolist():
            holder_of[int(fact_key[j])] = int(origin_h[j])
        shard_of = dict(zip(rows_v.tolist(), cols[3].tolist()))
        for j in np.nonzero(fact_key >= 0)[0].tolist():
            shard_of[int(fact_key[j])] = int(codes[j])
        self.next_id = n0 + int(ps["inserted"]) + len(supers)
        count0 = self.conversation_count
        etype = g.etype("relates_to")
        n_fact = n0 - int(np.searchsorted(self._sup_v, n0))
        reach_new: List[torch.Tensor] = []
        cc_w1 = False
        base_ok = self._native_w1_base_ok(pl, thr)
        if base_ok and any(seg["consolidate"] for seg in pl["segments"]) and \
                g.num_edges + sum(len(seg["edge_src"]) for seg in pl["segments"]) > T.dg_small_max_edges():
            # a graph past the one-block digest (the persistent graph): the
            # single tenant's incremental components -- the batch's stable
            # edges labelled once, the points union the volatile suffix inside
            # the native applier (rows are the plan's keys here)
            vic = [np.asarray(seg["victims"], np.int64).reshape(-1) for seg in pl["segments"]]
            with tracer.stage("cc_begin", dev):
                cc_w1 = g.cc_begin(np.concatenate(vic) if vic else np.zeros(0, np.int64), self.prune_threshold,
                                   1.0 - DECAY_RATE, B)
        try:
            if base_ok and self._native_w1_ok(pl, thr, cc_w1, base_checked=True):
                with tracer.stage("cb_apply_native", dev):
                    pruned += self._native_w1(pl, fact_key, codes, Q, flat, f_off, thr, now, count0, stats,
                                              reach_new)
                pl = {"segments": []}  # applied
        finally:
            if cc_w1:
                g.cc_end()
        with tracer.stage("sc_digest_base", dev):
            self._dcc_begin(pl)
            if any(s["consolidate"] for s in pl["segments"]):
                self._check_num_mono()
        try:
            for seg in pl["segments"]:
                with tracer.stage("cb_apply", dev):
                    pruned_local = self._apply_exact_segment(seg, supers, fact_key, origin_h, codes, Q, flat, f_off,
                                                             holder_of, shard_of, thr, now, etype, reach_new)
                if self._dcc is not None:
                    self._dcc["steps"] += int(seg["c1"]) - int(seg["c0"]) + 1
                pruned += self._sum(pruned_local)[0]
                self.conversation_count = count0 + int(seg["c1"]) + 1
                if seg["consolidate"]:
                    stats["consolidations"] += 1
                    with tracer.stage("run_consolidation", dev):
                        self.run_consolidation()
                if seg["cluster"]:
                    if reach_new:  # the pass rebuilds the cones from every row
                        self._reach_add(torch.cat(reach_new))
                        reach_new.clear()
                    with tracer.stage("cluster", dev):
                        self.cluster_pass()
                if self._commit_each:  # the counter as of this conversation
                    n_fact += int((np.asarray(seg["ins_kind"]) == 0).sum())
                    self.local.node_counter = n_fact
                    with tracer.stage("commit", "cpu"):
                        self.local._save_to_persistence()
        finally:
            self._dcc_end()
            self._num_mono = False
        stats["pruned"] += pruned
        if reach_new:
            self._reach_add(torch.cat(reach_new))
        if self.hierarchy_params and getattr(g, "hier", None) is None:
            self.cluster_pass()
        if self.local.query_cache:
            self.local.query_cache.invalidate_results()

    # one rank (no collectives, every row held here): the plan's segments
    # through the native applier (csrc/kernels/apply.hip) like the single
    # process; False: the per-segment path
    NATIVE_W1 = True
    native_w1_runs = 0  # batches applied natively (tests)

    def _native_w1_ok(self, pl: Dict, thr, cc: bool = False, base_checked: bool = False) -> bool:
        """The native applier applies the plan of a one-rank buffer exactly
        when the tenant's rows are its global node numbers (rows appended in
        number order, no ghost rows -- then every key of the plan is a row),
        no super-node is created (the reference hierarchy's ghost-free super
        rows are the per-segment path's), the decay prunes, and the graph's
        edges fit the one-block digest for the whole batch (the digest of
        :meth:`_digest_world1` on a tenant without super-nodes)."""
        g = self.g
        if not (base_checked or self._native_w1_base_ok(pl, thr)):
            return False
        app = sum(len(seg["edge_src"]) for seg in pl["segments"])
        if cc:
            # the partitioned batch (TenantGraph.cc_begin): every point takes the
            # incremental digest inside the applier
            c = g._cc
            ns = c.get("ns") if c is not None else None
            n_end = g.n + sum(len(seg["ins_kind"]) for seg in pl["segments"])
            if ns is None or ns <= T.dg_small_max_edges() or 16 * ns <= n_end:
                return False
        elif g.num_edges + app > T.dg_small_max_edges():
            return False
        return True

    def _native_w1_base_ok(self, pl: Dict, thr) -> bool:
        """The conditions of :meth:`_native_w1_ok` that do not depend on the
        graph's edges."""
        from ..core.consolidation import ConsolidationMixin
        from ..engine import native_apply as NA
        from ..engine import tenant_graph as TG
        g = self.g
        if not (self.NATIVE_W1 and ConsolidationMixin.NATIVE_APPLY and self.world == 1 and not self._coll
                and g.on_gpu and thr is not None and not self._commit_each and not pl["supers"]
                and g.n_super == 0 and TG.SEG_END_KERNEL and TG.SET_ROWS_KERNEL and not g._digest_sorted
                and NA.available() and self._sup_v.size == 0):
            return False
        if g.emb8 is not None and g.emb8.dtype != torch.int8:
            return False
        if g.dim is None or g.dim > 1024 or PROFILE_CONTENTS > 64:
            return False
        n = g.n
        if int(self.next_id) - sum(len(seg["ins_kind"]) for seg in pl["segments"]) != n:
            return False
        # every row is its node number (number = row + 1): one pass, one read
        with g.on_stream():
            ident = bool((self.num[:n] == torch.arange(1, n + 1, device=self.device)).all()) if n else True
        return ident

    def _native_w1(self, pl, fact_key, codes, Q, flat, f_off, thr, now, count0, stats, reach_new) -> int:
        """:meth:`_apply_exact_segment` for every segment of the plan through
        one native call per run of segments (a run ends at a cluster pass),
        rows = plan keys; then the host bookkeeping, the new rows' numbers,
        and run_consolidation's profile prompts (digest / first rows captured
        at each point, read after the run -- the profile sees the same
        contents: no content changes inside a batch without super-nodes).
        Returns the edges the segments' decays pruned."""
        from ..engine.native_apply import SegmentProgram
        g = self.g
        ms = self.local
        segs = pl["segments"]
        pruned = 0
        self.native_w1_runs += 1
        i = 0
        while i < len(segs):
            j = i
            while j < len(segs) - 1 and not segs[j]["cluster"]:
                j += 1
            run = segs[i:j + 1]
            etype = g.etype("relates_to") if any(len(s["edge_src"]) for s in run) else 0
            prog = SegmentProgram(g, now, thr if thr > 0.0 else float("-inf"), 1.0 - DECAY_RATE, etype,
                                  PROFILE_CONTENTS)
            n0 = g.n
            g.reserve(n0 + sum(len(s["ins_kind"]) for s in run))
            n = n0
            prog.n(n)
            host = []
            for seg in run:
                prog.decay(int(seg["c1"]) - int(seg["c0"]) + 1)
                tr = np.asarray(seg["tch_rows"], np.int64)
                if tr.size:
                    prog.touch_rows(tr, seg["tch_sal"], seg["tch_acc"], seg["tch_last"])
                kinds = np.asarray(seg["ins_kind"], np.int64).reshape(-1)
                idx = np.asarray(seg["ins_idx"], np.int64).reshape(-1)
                isal = np.asarray(seg["ins_sal"], np.float32)
                iacc = np.asarray(seg["ins_acc"], np.int32)
                ilast = np.asarray(seg["ins_last"], np.float64)
                ins = []
                if idx.size:  # (no super-nodes: every insert is a fact, in key order)
                    keys = fact_key[idx]
                    if not np.array_equal(keys, np.arange(n, n + keys.size)):
                        raise RuntimeError("native apply: plan keys are not the next rows")
                    sh = codes[idx].astype(np.int32)
                    prog.insert_rows(n, int(idx.size), {"sal": isal, "acc": iacc, "last": ilast, "shard": sh}, True)
                    prog.embeddings(idx.tolist(), n)
                    cnt = np.bincount(sh[sh >= 0], minlength=1)
                    for c in np.nonzero(cnt)[0].tolist():
                        prog.shard_delta(c, int(cnt[c]))
                    lf = [flat[int(x) - f_off] for x in idx]
                    ins = (self._ids_of_nums(keys + 1), [f["content"] for f in lf],
                           [f.get("type", "semantic") for f in lf], sh, n)
                    n += int(idx.size)
                    prog.n(n)
                es = np.asarray(seg["edge_src"], np.int64)
                if es.size:
                    prog.append_edges(es, seg["edge_dst"], seg["edge_w"], seg["edge_code"])
                vic = sorted({int(r) for r in np.asarray(seg["victims"], np.int64).tolist() if 0 <= r < n})
                prog.segment_end(vic)
                if seg["consolidate"]:
                    prog.point()
                host.append((ins, vic))
            res = prog.run(g.shard_count, Q, g._cc)
            p = 0
            gone = []
            for s, (seg, (ins, vic)) in enumerate(zip(run, host)):
                steps = int(seg["c1"]) - int(seg["c0"]) + 1
                g.decay_log += steps * math.log1p(-DECAY_RATE)
                if g._cc is not None:
                    g._cc["steps"] += steps
                g._bump(edges=True)
                if ins:
                    ids, contents, types, sh, r0 = ins
                    m = len(ids)
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
                    if not g._dv_acc_pending:
                        g._norm_dev_pending.append(g._dv_acc[0])
                        g._dv_acc_pending = True
                    g._bump(store=True)
                    self._sync_num()
                    rows = torch.arange(r0, r0 + m, device=self.device)
                    self.num[r0:r0 + m] = rows + 1
                    self.holder[r0:r0 + m] = self.rank
                    reach_new.append(rows)
                gone += [g.ids[r] for r in vic]
                pruned += prog.finish_segment(res, s)
                self.conversation_count = count0 + int(seg["c1"]) + 1
                if seg["consolidate"]:
                    stats["consolidations"] += 1
                    dig, first = prog.captures(res, p)
                    p += 1
                    self._rc_w1_host(dig, first)
            if gone:
                ms._store_delete(gone, graph_unstored=True)
            if list(res["shard_count"][:len(g.shard_count)]) != list(g.shard_count):
                raise RuntimeError("native segment apply diverged from the host shard counts")
            if run[-1]["cluster"]:
                if reach_new:  # the pass rebuilds the cones from every row
                    self._reach_add(torch.cat(reach_new))
                    reach_new.clear()
                with tracer.stage("cluster", self.device):
                    self.cluster_pass()
            i = j + 1
        return pruned

    def _rc_w1_host(self, dig, first) -> None:
        """:meth:`run_consolidation`'s host side on one rank from the native
        run's captures: the profile prompt of every qualifying component,
        else of the first shard rows (no prune: the segment end already
        dropped every edge under the threshold)."""
        ms = self.local
        g = self.g
        updates = 0
        for rows in dig.get():
            r = ms._extract_profile_from_contents([g.content[int(x)] for x in rows.tolist()])
            if "Updated" in r:
                updates += 1
        if updates == 0:
            contents = [g.content[int(r)] for r in first.get().tolist()]
            if len(contents) >= 3:
                ms._extract_profile_from_contents(contents)

    def _apply_exact_segment(self, seg, supers, fact_key, origin_h, codes, Q, flat, f_off, holder_of, shard_of, thr,
                             now, etype, reach_new) -> int:
        """This rank's part of one plan segment (see :meth:`_consolidate_exact`).
        Returns the local edges the segment's decay pruned."""
        g = self.g
        dev = self.device
        me = self.rank
        steps = int(seg["c1"]) - int(seg["c0"]) + 1
        tok = g.segment_begin(DECAY_RATE, thr, steps)
        tr = np.asarray(seg["tch_rows"], np.int64)
        if tr.size:
            loc = self._held_rows(torch.as_tensor(tr).to(dev))
            if g.on_gpu:
                # one launch over every touched row, rows held elsewhere (-1)
                # skipped in the kernel: no host read of which rows are local
                m = int(tr.size)
                blk = torch.empty(7 + 3 * m, dtype=torch.float64).pin_memory()
                bn = blk.numpy()
                bn[:7] = 0.0
                for j, c in enumerate((seg["tch_sal"], seg["tch_acc"], seg["tch_last"])):
                    bn[7 + j * m: 7 + (j + 1) * m] = np.asarray(c, dtype=np.float64).reshape(-1)
                with g.on_stream():
                    T.set_rows(g, loc.contiguous(), blk.to(dev, non_blocking=True), 0b111 | (0b1111000 << 8), -1, -1)
                g._bump()
            else:
                keep_ = torch.nonzero(loc >= 0).flatten()
                if keep_.numel():
                    k_h = keep_.cpu().numpy()
                    rt = loc[keep_]
                    with g.on_stream():
                        g.sal[rt] = torch.as_tensor(np.asarray(seg["tch_sal"])[k_h], dtype=torch.float32).to(dev)
                        g.acc[rt] = torch.as_tensor(np.asarray(seg["tch_acc"])[k_h], dtype=torch.int32).to(dev)
                        g.last[rt] = torch.as_tensor(np.asarray(seg["tch_last"])[k_h], dtype=torch.float64).to(dev)
                        g.dirty[rt] = 1
                    g._bump()
        kinds = np.asarray(seg["ins_kind"], np.int64).reshape(-1)
        idx_all = np.asarray(seg["ins_idx"], np.int64).reshape(-1)
        fpos = np.nonzero(kinds == 0)[0]
        idx = idx_all[fpos]
        if idx.size:
            sel_ = origin_h[idx] == me
            mine = idx[sel_]
            if mine.size:
                pos = fpos[sel_]
                keys = fact_key[mine]
                lf = [flat[int(j) - f_off] for j in mine]
                rows = g.add_nodes(self._ids_of_nums(keys + 1), [f["content"] for f in lf],
                                   Q[torch.as_tensor(mine, dtype=torch.long).to(dev)], shard=codes[mine].astype(np.int32),
                                   types=[f.get("type", "semantic") for f in lf],
                                   sal=torch.as_tensor(np.asarray(seg["ins_sal"], np.float32)[pos]),
                                   acc=torch.as_tensor(np.asarray(seg["ins_acc"], np.int32)[pos]),
                                   last=torch.as_tensor(np.asarray(seg["ins_last"], np.float64)[pos]), now=now,
                                   stored=True)
                self._sync_num()
                self.num[rows] = torch.as_tensor(keys + 1, dtype=torch.long).to(dev)
                self.holder[rows] = me
                reach_new.append(rows)  # cone test once per batch (the next batch's scan reads it)
        # super-nodes after the facts: their children (earlier keys) all exist
        for p in np.nonzero(kinds != 0)[0].tolist():
            sp = supers[int(idx_all[p])]
            info = self._super_plan[tuple(np.asarray(sp["children"], np.int64).tolist())]
            self._insert_super(sp, info, now, sal=float(np.asarray(seg["ins_sal"])[p]),
                               acc=int(np.asarray(seg["ins_acc"])[p]), last=float(np.asarray(seg["ins_last"])[p]))
        es = np.asarray(seg["edge_src"], np.int64)
        if es.size:
            ed = np.asarray(seg["edge_dst"], np.int64)
            ew = np.asarray(seg["edge_w"], np.float32)
            ec = np.asarray(seg["edge_code"], np.int64)
            sel = np.asarray([holder_of.get(int(x), -1) == me for x in es.tolist()], bool)
            if sel.any():
                es, ed, ew, ec = es[sel], ed[sel], ew[sel], ec[sel]
                src = self._held_rows(torch.as_tensor(es).to(dev))
                dst = self._held_rows(torch.as_tensor(ed).to(dev))
                # endpoints held elsewhere (known on the host): only then look
                # for the missing rows on the device (a host read)
                remote = any(holder_of.get(int(x), -1) != me for x in ed.tolist())
                need = torch.nonzero(dst < 0).flatten() if remote else None
                if need is not None and need.numel():  # endpoints held elsewhere: ghost rows (created once per node)
                    dv = ed[need.cpu().numpy()]
                    ids = self._ids_of_nums(dv + 1)
                    fresh = {}
                    for i, x in zip(ids, dv.tolist()):
                        if g.row_of.get(i, -1) < 0 and i not in fresh:
                            fresh[i] = (int(shard_of[int(x)]), int(holder_of[int(x)]), int(x) + 1)
                    if fresh:
                        fid = list(fresh)
                        rn = g.add_nodes(fid, [""] * len(fid), None, shard=[fresh[i][0] for i in fid], ghost=True,
                                         stored=False, now=now)
                        self._sync_num()
                        self.num[rn] = torch.as_tensor([fresh[i][2] for i in fid], dtype=torch.long).to(dev)
                        self.holder[rn] = torch.as_tensor([fresh[i][1] for i in fid], dtype=torch.long).to(dev)
                    dst[need] = torch.as_tensor([g.row_of[i] for i in ids], dtype=torch.long).to(dev)
                g.append_edges(src, dst, torch.as_tensor(ew).to(dev), torch.as_tensor(ec, dtype=torch.int32).to(dev),
                               etype, now=now)
        vic = np.asarray(seg["victims"], np.int64)
        loc_v = []
        other = np.zeros(0, np.int64)
        if vic.size:
            hv = np.asarray([holder_of.get(int(x), -1) for x in vic.tolist()], np.int64)
            mv = vic[hv == me]
            if mv.size:  # victims are live fact nodes held here: their rows by id, no device read
                ro = g.row_of
                loc_v = [r for r in (ro.get(i, -1) for i in self._ids_of_nums(mv + 1)) if r >= 0]
            other = vic[hv != me]
        ids = [g.ids[r] for r in loc_v]
        pruned = g.segment_end(tok, loc_v, unstore=True)
        if ids:
            self.local._store_delete(ids, graph_unstored=True)
        if other.size and g.num_edges:  # edges here that point at a victim held elsewhere
            rows = self._rows_of_nums(torch.as_tensor(other + 1).to(dev))
            rows = rows[rows >= 0]
            if rows.numel():
                with g.on_stream():
                    rm = torch.zeros(g.n, dtype=torch.uint8, device=dev)
                    rm[rows] = 1
                    g.e, k_, dropped = T.remove_edges_of(g.e, rm, g.shard[: g.n], want_dropped=g.track)
                if dropped is not None and k_:
                    g._note_dropped(*dropped)
                g._bump(edges=True)
        return int(pruned)

    # ------------------------------------------------------------------ eviction
    def _evict(self, now: float, stats: Dict[str, int]) -> None:
        """Global buffer limit (reference :535-578 over the whole tenant)."""
        g = self.g
        dev = self.device
        total = self._sum(g.num_nodes())[0]
        excess = total - self.max_buffer_size
        if excess <= 0:
            return
        with tracer.stage("sc_evict", dev):
            n = g.n
            m = min(excess, n)
            cand_s = torch.full((excess,), float("inf"), dtype=torch.float64, device=dev)
            cand_k = torch.full((excess,), BIG, dtype=torch.long, device=dev)
            cand_r = torch.full((excess,), -1, dtype=torch.long, device=dev)
            if m:
                with g.on_stream():
                    score = T.importance(g.sal[:n], g.acc[:n], g.last[:n], g.kind[:n], g.sup[:n], now)
                    okey = (g.shard[:n].long() + 1) * (1 << NUM_BITS) + self.num[:n]
                    # this rank's m lowest (score, shard, number): a top-k for the
                    # threshold, then the tied rows by key (no full sort)
                    t = torch.topk(score, m, largest=False, sorted=False).values.max()
                    lt = torch.nonzero(score < t).flatten()
                    rest = m - int(lt.numel())
                    tie = torch.where(score == t, okey, torch.full_like(okey, BIG))
                    tv, ti = torch.topk(tie, rest, largest=False, sorted=True) if rest > 0 else (tie[:0], lt[:0])
                    cand = torch.cat([lt, ti[tv != BIG]])
                    cand = cand[torch.isfinite(score[cand])]
                    c = int(cand.numel())
                    cand_s[:c] = score[cand]
                    cand_k[:c] = okey[cand]
                    cand_r[:c] = cand
            alls = self._gather_rows(cand_s)
            allk = self._gather_rows(cand_k)
            o = torch.argsort(allk, stable=True)
            o = o[torch.sort(alls[o], stable=True).indices][:excess]
            o = o[torch.isfinite(alls[o])]
            stats["evicted"] += int(o.numel())
            if o.numel() == 0:
                return
            owner = o // excess
            pos = o % excess
            mine = cand_r[pos[owner == self.rank]]
            victims = mine.tolist()
            if victims:
                g.remove_nodes(victims, drop_edges=True, unstore=True)
                self.local._store_delete([g.ids[r] for r in victims])
            # edges held here that point at a victim held elsewhere: the
            # victim's shard drops them (its ghost row carries that shard)
            other = allk[o[owner != self.rank]] & ((1 << NUM_BITS) - 1)
            if other.numel() and g.num_edges:
                rows = self._rows_of_nums(other)
                rows = rows[rows >= 0]
                if rows.numel():
                    with g.on_stream():
                        rm = torch.zeros(g.n, dtype=torch.uint8, device=dev)
                        rm[rows] = 1
                        g.e, k, dropped = T.remove_edges_of(g.e, rm, g.shard[: g.n], want_dropped=g.track)
                    if dropped is not None and k:
                        g._note_dropped(*dropped)
                    g._bump(edges=True)

    # ------------------------------------------------------------------ re-shard
    def rebalance(self) -> Dict[str, int]:
        """Collective all-to-all re-shard: move live rows
        from ranks above the even share to ranks below it -- inserts land on
        the rank whose conversation made them and eviction is global, so the
        split drifts. A moved node takes its vector, scalars, content and its
        outgoing edges (edges live with their source) to the new holder; the old
        row becomes a ghost, ghost rows everywhere learn the new holder (one
        all-gather of the moved numbers). Node numbers do not change, so every
        later decision is unchanged. Returns {"moved": rows moved in total}."""
        g = self.g
        dev = self.device
        W = self.world
        if not self._coll:
            return {"moved": 0}
        counts = self._gather_rows(torch.tensor([g.num_nodes()], dtype=torch.int64, device=dev)).tolist()
        T_ = sum(counts)
        tgt = [T_ // W + (1 if r < T_ % W else 0) for r in range(W)]
        sur = [c - t for c, t in zip(counts, tgt)]
        moves = [[0] * W for _ in range(W)]
        need = [[r, -x] for r, x in enumerate(sur) if x < 0]
        j = 0
        for r, x in enumerate(sur):
            while x > 0 and j < len(need):
                k = min(x, need[j][1])
                moves[r][need[j][0]] += k
                x -= k
                need[j][1] -= k
                if need[j][1] == 0:
                    j += 1
        total_moved = sum(map(sum, moves))
        if total_moved == 0:
            return {"moved": 0}
        n = g.n
        D = g.dim
        n_out = sum(moves[self.rank])
        if n_out:
            with g.on_stream():
                live = (g.kind[:n] == NODE) & (g.sup[:n] == 0)
                key = torch.where(live, self.num[:n], torch.full((n,), -1, dtype=torch.long, device=dev))
                _, rows_out = torch.topk(key, n_out)  # the most recent nodes move
                rows_out = rows_out[torch.argsort(self.num[rows_out])]
            dest = torch.repeat_interleave(torch.arange(W, device=dev),
                                           torch.tensor(moves[self.rank], dtype=torch.long, device=dev))
        else:
            rows_out = torch.zeros(0, dtype=torch.long, device=dev)
            dest = torch.zeros(0, dtype=torch.long, device=dev)
        ro = rows_out
        num_f = torch.stack([self.num[ro].double(), g.shard[ro].double(), g.sal[ro].double(), g.acc[ro].double(),
                             g.last[ro], g.ts[ro]], 1) if n_out else torch.zeros((0, 6), dtype=torch.float64,
                                                                                   device=dev)
        emb = g.emb32[ro] if n_out else torch.zeros((0, D), dtype=torch.float32, device=dev)
        rh = ro.tolist()
        texts = [[] for _ in range(W)]
        for r_, d_ in zip(rh, dest.tolist()):
            texts[d_].append([g.content[r_], g.types[r_]])
        # outgoing edges of the moved rows travel with them
        if n_out and g.num_edges:
            mv = torch.zeros(n, dtype=torch.bool, device=dev)
            mv[ro] = True
            dest_of = torch.full((n,), -1, dtype=torch.long, device=dev)
            dest_of[ro] = dest
            e = g.e
            eidx = torch.nonzero(mv[e["src"].long()]).flatten()
            s_, d_ = e["src"][eidx].long(), e["dst"][eidx].long()
            edge_f = torch.stack([self.num[s_].double(), self.num[d_].double(),
                                  (e["meta"][eidx] & SHARD_MASK).double(),
                                  ((e["meta"][eidx] >> TYPE_SHIFT) & TYPE_MASK).double(), e["w"][eidx].double(),
                                  e["co"][eidx].double(), e["lu"][eidx], g.shard[d_].double(),
                                  self.holder[d_].double()], 1)
            edest = dest_of[s_]
        else:
            eidx = torch.zeros(0, dtype=torch.long, device=dev)
            edge_f = torch.zeros((0, 9), dtype=torch.float64, device=dev)
            edest = torch.zeros(0, dtype=torch.long, device=dev)
        cd = self.comm.device
        r_num, r_emb = (x.to(dev) for x in self.comm.reshard(dest.to(cd), num_f.to(cd), emb.to(cd)))
        (r_edge,) = (x.to(dev) for x in self.comm.reshard(edest.to(cd), edge_f.to(cd)))
        got_txt = self.comm.exchange_objects(texts)
        # sender: the moved rows become ghosts held elsewhere, their edges leave
        if n_out:
            if eidx.numel():
                g.remove_edges(eidx)
            g.remove_nodes(rh, drop_edges=False, unstore=True)
            self.holder[ro] = dest
        # receiver: the rows arrive (a ghost row of the same id turns live)
        m_in = int(r_num.shape[0])
        if m_in:
            txt = [t for part in got_txt if part for t in part]
            nums = r_num[:, 0].long()
            rows = g.add_nodes(self._ids_of_nums(nums.tolist()), [t[0] for t in txt], r_emb,
                               shard=r_num[:, 1].int(), types=[t[1] for t in txt], sal=r_num[:, 2].float(),
                               acc=r_num[:, 3].int(), last=r_num[:, 4], ts=r_num[:, 5], stored=True)
            self._sync_num()
            self.num[rows] = nums
            self.holder[rows] = self.rank
            self._reach_add(rows)
        if r_edge.shape[0]:
            src = self._rows_of_nums(r_edge[:, 0].long())
            dn = r_edge[:, 1].long()
            dst = self._rows_of_nums(dn)
            miss = torch.nonzero(dst < 0).flatten()
            if miss.numel():
                un, first = np.unique(dn[miss].cpu().numpy(), return_index=True)
                fi = miss[torch.as_tensor(first, dtype=torch.long).to(dev)]
                rows_g = g.add_nodes(self._ids_of_nums(un), [""] * len(un), None,
                                     shard=r_edge[fi, 7].int(), ghost=True, stored=False)
                self._sync_num()
                self.num[rows_g] = torch.as_tensor(un).to(dev)
                self.holder[rows_g] = r_edge[fi, 8].long()
                dst = self._rows_of_nums(dn)
            et = r_edge[:, 3].long()
            for t in torch.unique(et).tolist():
                sel = et == t
                g.append_edges(src[sel], dst[sel], r_edge[sel, 4].float(), r_edge[sel, 2].int(), int(t),
                               co=r_edge[sel, 5].int(), lu=r_edge[sel, 6])
        # every ghost row of a moved node learns its new holder
        moved = torch.stack([self.num[ro] if n_out else torch.zeros(0, dtype=torch.long, device=dev), dest], 1)
        allm, _ = self._gather_var(moved)
        if allm.numel():
            rr = self._rows_of_nums(allm[:, 0])
            ok = rr >= 0
            self.holder[rr[ok]] = allm[ok, 1]
        return {"moved": total_moved}

    # ------------------------------------------------------------------ deep consolidation
    # Up to this many edges over all ranks the digest replicates them (one
    # all-gather of 24 B per edge) and every rank runs the single-graph digest
    # kernels on the endpoints; above it the boundary-label exchange keeps the
    # work and the bytes distributed (the 20M-edge persistent graph per rank).
    DIGEST_REPLICATE_MAX = 1 << 22

    def _digest_world1(self, min_size: int, min_avg_w: float, take: int) -> List[List[str]]:
        """:meth:`component_digest` of a one-rank tenant on the GPU: the local
        rows are the whole tenant (no ghosts), rows are appended in node-number
        order (a fact's number and row both follow the plan's insertion
        order), so the single-graph digest kernels run on the rows directly --
        super-node rows passed as non-candidate members, as the distributed
        form counts them (they are not first-member keys)."""
        g = self.g
        n = g.n
        sup = g.sup[:n]
        kind = torch.where((g.kind[:n] == NODE) & (sup != 0), torch.full_like(g.kind[:n], GHOST), g.kind[:n])
        e = g.e
        if g.num_edges <= T.dg_small_max_edges():
            res = T.component_digest_small(e["src"], e["dst"], e["w"], kind, sup, g.shard[:n], n, min_size,
                                           min_avg_w, take)
        else:
            res = T.component_digest_local(e["src"], e["dst"], e["w"], kind, sup, g.shard[:n], min_size, min_avg_w,
                                           take)
        return [[g.content[int(r)] for r in rows] for rows in T.digest_lists(res.cpu().numpy())]

    def _digest_replicated(self, cnt: List[int], min_size: int, min_avg_w: float, take: int) -> List[List[str]]:
        """:meth:`component_digest` over the replicated edge list, four
        collectives in all (edge counts, edges, the endpoints' liveness, the
        selected contents) instead of the boundary-label rounds and five
        routed exchanges. Every rank renumbers the endpoints' node numbers
        0 .. U-1 in number order (identical on every rank: same edges, same
        order), the holders fill in which endpoints are live shard nodes and
        their shard (one all-reduce), and the digest runs on that compact
        graph -- on the GPU the one-block ``dg_small`` kernel or the O(edges)
        renumbered digest (tenant_ops), no host synchronisation before the
        selected rows. The renumbering is monotone in the node number, so the
        components, their (shard, number) first-member order and each
        component's first ``take`` live members are those of the distributed
        form."""
        g = self.g
        dev = self.device
        ne = cnt[self.rank] if self._coll else cnt[0]
        if ne:
            ed = torch.stack([self.num[g.e["src"].long()], self.num[g.e["dst"].long()],
                              g.e["w"].float().contiguous().view(torch.int32).long()], 1)
        else:
            ed = torch.zeros((0, 3), dtype=torch.long, device=dev)
        if self._coll:
            mx = max(cnt)
            pad = torch.zeros((mx, 3), dtype=torch.long, device=dev)
            pad[:ne] = ed
            allr = self._gather_rows(pad)
            ed = torch.cat([allr[r * mx: r * mx + c] for r, c in enumerate(cnt) if c])
        E = int(ed.shape[0])
        if E == 0:
            return []
        nl = 2 * E
        ep = ed[:, :2].reshape(-1)
        srt, perm = torch.sort(ep)
        newf = torch.ones(nl, dtype=torch.bool, device=dev)
        newf[1:] = srt[1:] != srt[:-1]
        uid = torch.cumsum(newf, 0) - 1
        local = torch.empty(nl, dtype=torch.int64, device=dev)
        local[perm] = uid
        numof = torch.full((nl,), -1, dtype=torch.long, device=dev)  # compact id -> node number
        numof[uid] = srt
        valid = numof >= 0
        rows = self._rows_of_nums(numof.clamp_min(0))
        rc = rows.clamp_min(0)
        mine = valid & (rows >= 0) & (self.holder[rc] == self.rank) & (g.kind[rc] == NODE) & (g.sup[rc] == 0)
        attr = torch.where(mine, g.shard[rc].long() + 1, torch.zeros_like(rows))  # one holder per node
        if self._coll:
            attr = self.comm.all_reduce(self._to_comm(attr)).to(dev)
        live = attr > 0
        lsrc, ldst = local[0::2].contiguous(), local[1::2].contiguous()
        w = ed[:, 2].to(torch.int32).view(torch.float32)
        if dev.type == "cuda":
            kind_c = torch.where(valid, torch.where(live, 1, 2), 0).to(torch.uint8)
            sup_c = torch.zeros(nl, dtype=torch.uint8, device=dev)
            shard_c = (attr - 1).clamp_min(0).to(torch.int32)
            if E <= T.dg_small_max_edges():
                res = T.component_digest_small(lsrc, ldst, w, kind_c, sup_c, shard_c, nl, min_size, min_avg_w, take)
            else:
                res = T.component_digest_local(lsrc, ldst, w, kind_c, sup_c, shard_c, min_size, min_avg_w, take)
        else:
            res = _digest_compact_host(lsrc, ldst, w, valid, live, attr - 1, nl, min_size, min_avg_w, take)
        return self._digest_contents(res, numof)

    def _digest_contents(self, res, numof: torch.Tensor) -> List[List[str]]:
        """The digest's (order key, compact id) pairs as content lists: ids to
        node numbers (``numof``), the holders fill in the contents (one object
        all-gather), rank 0 groups them by key."""
        g = self.g
        ok = res[1] >= 0
        nums = torch.where(ok, numof[res[1].clamp_min(0)], torch.full_like(res[1], -1))
        rr = self._rows_of_nums(nums.clamp_min(0))
        own = ok & (rr >= 0) & (self.holder[rr.clamp_min(0)] == self.rank)
        kr = torch.stack([res[0], nums, torch.where(own, rr, torch.full_like(rr, -1))]).cpu().numpy()
        mine_c = [(int(k), int(v), g.content[int(r)]) for k, v, r in zip(kr[0], kr[1], kr[2]) if r >= 0]
        parts = self.comm.all_gather_object(mine_c) if self._coll else [mine_c]
        if self.rank != 0:
            return []
        out: List[List[str]] = []
        last = None
        for f_, _, c in sorted(x for p in parts for x in p):
            if f_ != last:
                out.append([])
                last = f_
            out[-1].append(c)
        return out

    # ---- incremental digest over the ranks. Within one batch of the
    # reference cadence the digest at every run_consolidation point is the
    # batch's STABLE base -- the edges that exist at every point: none incident
    # to a victim of the plan, none that the batch's decays (or a
    # run_consolidation prune) can bring under the threshold -- plus the few
    # volatile edges (TenantGraph.cc_begin's definition, per rank). The base is
    # all-gathered and labelled ONCE per batch (union-find over the replicated
    # stable edges), its endpoints' liveness / shard fixed for the batch (no
    # base endpoint is a victim); each point all-gathers only the volatile
    # edges, replays the decay rounds since the batch start on the replicated
    # base weights (the same tg_decay rounds every rank ran on its own edges,
    # bit for bit), unions the volatile edges on top of the base labels and
    # runs the digest kernels -- instead of all-gathering every edge of every
    # rank at every point (~43 per step) or the boundary-label rounds above
    # DIGEST_REPLICATE_MAX. Vertex ids are a batch-wide universe in node-number
    # order (the base endpoints, the volatile ones, every endpoint the plan
    # will link), so first-member keys order components as the full digest
    # does. Reference: buffer_graph.py:99-120, memory_system.py:967-985.
    DIGEST_INCREMENTAL = True
    DIGEST_INCREMENTAL_MIN = 1 << 16  # edges over all ranks at the batch start
    _dcc = None
    dcc_points = 0  # points served by the incremental digest (tests)
    dcc_base_max = 0  # the largest replicated base (edges) so far (tests)

    def _dcc_begin(self, pl: Dict) -> None:
        """Set up a batch's incremental digest (collective; every rank decides
        alike from all-gathered counts)."""
        self._dcc = None
        segs = pl["segments"]
        g = self.g
        if not (self.DIGEST_INCREMENTAL and any(s["consolidate"] for s in segs)):
            return
        dev = self.device
        ne = int(g.num_edges) if g.n else 0
        tot = self._sum(ne)[0]
        if tot < max(1, self.DIGEST_INCREMENTAL_MIN):
            return
        if self.world == 1 and g.on_gpu and tot <= T.dg_small_max_edges():
            return  # one GPU rank, a few edges: the one-block row digest (_digest_world1)
        keep = 1.0 - DECAY_RATE
        steps = sum(int(s["c1"]) - int(s["c0"]) + 1 for s in segs)
        t0 = NEG_INF
        if self.prune_threshold > 0.0:  # the segments' decay-prune and run_consolidation's prune
            t0 = float(self.prune_threshold) * keep ** (-steps) * (1.0 + 1e-4) + 1e-12
        vic = [np.asarray(s["victims"], np.int64).reshape(-1) for s in segs]
        vic = np.concatenate(vic) if vic else np.zeros(0, np.int64)
        ns = 0
        if ne:
            vmark = torch.zeros(g.n, dtype=torch.uint8, device=dev)
            if vic.size:
                vr = self._rows_of_nums(torch.as_tensor(vic + 1).to(dev))  # live and ghost rows of the victims
                vr = vr[vr >= 0]
                if vr.numel():
                    vmark[vr] = 1
            with g.on_stream():
                p = g._partition_stable(vmark, t0)
            ns = 0 if p is None else int(p)
            if ns:  # the stable prefix stays in place: segment ends compact the suffix only
                g._cc = {"ns": ns, "steps": 0, "sharded": True}
        # the replicated base: (number, number, weight bits), rank order
        e = g.e
        if ns:
            loc = torch.stack([self.num[e["src"][:ns].long()], self.num[e["dst"][:ns].long()],
                               e["w"][:ns].float().contiguous().view(torch.int32).long()], 1)
        else:
            loc = torch.zeros((0, 3), dtype=torch.long, device=dev)
        base, _ = self._gather_var(loc)
        # volatile endpoints now, every endpoint the plan links: the universe
        if ne > ns:
            vol = torch.cat([self.num[e["src"][ns:].long()], self.num[e["dst"][ns:].long()]])
        else:
            vol = torch.zeros(0, dtype=torch.long, device=dev)
        vol, _ = self._gather_var(vol)
        planned = [np.asarray(s[k], np.int64).reshape(-1) for s in segs for k in ("edge_src", "edge_dst")]
        planned = np.concatenate(planned) + 1 if planned else np.zeros(0, np.int64)
        A = torch.unique(torch.cat([base[:, 0], base[:, 1], vol, torch.as_tensor(planned).to(dev)]))
        nl = int(A.numel())
        bs = torch.searchsorted(A, base[:, 0].contiguous())
        bd = torch.searchsorted(A, base[:, 1].contiguous())
        nb = int(bs.numel())
        inb = torch.zeros(nl, dtype=torch.bool, device=dev)
        inb[bs] = True
        inb[bd] = True
        # base endpoints: liveness and shard are fixed for the batch (one all-reduce)
        attr = torch.zeros(nl, dtype=torch.long, device=dev)
        bidx = torch.nonzero(inb).flatten()
        if bidx.numel():
            attr[bidx] = self._attr_of(A[bidx])
        # stats arrays: the base as the prefix, room behind it for the volatile edges
        cap = nb + max(1024, 2 * int(vol.numel()) // 2 + 2 * int(planned.size))
        src = torch.empty(cap, dtype=torch.int32, device=dev)
        dst = torch.empty(cap, dtype=torch.int32, device=dev)
        w = torch.empty(cap, dtype=torch.float32, device=dev)
        src[:nb] = bs.to(torch.int32)
        dst[:nb] = bd.to(torch.int32)
        w[:nb] = base[:, 2].to(torch.int32).view(torch.float32)
        lab = None
        if dev.type == "cuda" and nb:
            from ..ops.graph_ops import components_sel
            zero = torch.zeros(nl, dtype=torch.uint8, device=dev)
            lab = components_sel(src[:nb], dst[:nb], nl, None, NEG_INF, zero, nl, 0)
        self.dcc_base_max = max(self.dcc_base_max, nb)
        self._dcc = {"ns": ns, "A": A, "nl": nl, "nb": nb, "src": src, "dst": dst, "w": w, "lab": lab,
                     "attr": attr, "dyn": torch.nonzero(~inb).flatten(), "steps": 0, "wsteps": 0}

    def _dcc_end(self) -> None:
        if self._dcc is not None and self.g._cc is not None and self.g._cc.get("sharded"):
            self.g._cc = None
        self._dcc = None

    def _attr_of(self, nums: torch.Tensor) -> torch.Tensor:
        """shard + 1 of the live shard nodes among ``nums`` (0: not a live
        shard node anywhere), from their holders: one all-reduce."""
        g = self.g
        rows = self._rows_of_nums(nums)
        rc = rows.clamp_min(0)
        mine = (rows >= 0) & (self.holder[rc] == self.rank) & (g.kind[rc] == NODE) & (g.sup[rc] == 0)
        attr = torch.where(mine, g.shard[rc].long() + 1, torch.zeros_like(rows))
        if self._coll:
            attr = self.comm.all_reduce(self._to_comm(attr)).to(self.device)
        return attr

    def _digest_incremental(self, min_size: int, min_avg_w: float, take: int) -> Optional[List[List[str]]]:
        """:meth:`component_digest` at a point of a batch with the incremental
        base (:meth:`_dcc_begin`); None when a volatile endpoint fell outside
        the batch's universe (every rank sees the same gathered edges, so every
        rank falls back alike)."""
        d = self._dcc
        g = self.g
        dev = self.device
        nb, nl, A = d["nb"], d["nl"], d["A"]
        k = d["steps"] - d["wsteps"]
        if k > 0 and nb:  # the decay rounds every rank ran on its own stable edges since the batch start
            T.decay_prune({"src": d["src"][:nb], "w": d["w"][:nb]}, None, None, None, DECAY_RATE, None, False,
                          steps=k)
        d["wsteps"] = d["steps"]
        ns = d["ns"]
        e = g.e
        ne = int(g.num_edges) if g.n else 0
        if ne > ns:
            loc = torch.stack([self.num[e["src"][ns:].long()], self.num[e["dst"][ns:].long()],
                               e["w"][ns:].float().contiguous().view(torch.int32).long()], 1)
        else:
            loc = torch.zeros((0, 3), dtype=torch.long, device=dev)
        vol, _ = self._gather_var(loc)
        m = int(vol.shape[0])
        vs = torch.searchsorted(A, vol[:, 0].contiguous()).clamp_max(max(nl - 1, 0))
        vd = torch.searchsorted(A, vol[:, 1].contiguous()).clamp_max(max(nl - 1, 0))
        if m and nl == 0:
            return None
        if m and not bool(((A[vs] == vol[:, 0]) & (A[vd] == vol[:, 1])).all()):
            return None
        if nb + m > d["src"].numel():  # grow the volatile room (the base prefix is copied once)
            cap = nb + 2 * m
            for key, dt in (("src", torch.int32), ("dst", torch.int32), ("w", torch.float32)):
                buf = torch.empty(cap, dtype=dt, device=dev)
                buf[:nb] = d[key][:nb]
                d[key] = buf
        src, dst, w = d["src"], d["dst"], d["w"]
        src[nb:nb + m] = vs.to(torch.int32)
        dst[nb:nb + m] = vd.to(torch.int32)
        w[nb:nb + m] = vol[:, 2].to(torch.int32).view(torch.float32)
        E = nb + m
        if E == 0:
            return []
        attr = d["attr"].clone()
        dyn = d["dyn"]
        if dyn.numel():  # endpoints outside the base: victims, new facts (their liveness changes)
            attr[dyn] = self._attr_of(A[dyn])
        live = attr > 0
        if dev.type == "cuda":
            kind_c = torch.where(live, 1, 2).to(torch.uint8)
            sup_c = torch.zeros(nl, dtype=torch.uint8, device=dev)
            shard_c = (attr - 1).clamp_min(0).to(torch.int32)
            if d["lab"] is not None:
                from ..ops.graph_ops import components_sel
                z = d.get("zero")
                if z is None:
                    z = d["zero"] = torch.zeros(nl, dtype=torch.uint8, device=dev)
                lab = components_sel(src[nb:E], dst[nb:E], nl, None, NEG_INF, z, nl, 0, parent=d["lab"].clone())
            else:
                lab = None
            res = T.component_digest(src[:E], dst[:E], w[:E], kind_c, sup_c, shard_c, nl, min_size, min_avg_w, take,
                                     lab=lab)
        else:
            s_, d_ = src[:E].long(), dst[:E].long()
            valid = torch.zeros(nl, dtype=torch.bool, device=dev)
            valid[s_] = True
            valid[d_] = True
            res = _digest_compact_host(s_, d_, w[:E], valid, live & valid, attr - 1, nl, min_size, min_avg_w, take)
        self.dcc_points += 1
        return self._digest_contents(res, A)

    def component_digest(self, min_size: int = 3, min_avg_w: float = 0.3,
                         take: int = PROFILE_CONTENTS) -> List[List[str]]:
        """``run_consolidation``'s component view of the WHOLE tenant
        (reference :967-990; single-process ``TenantGraph.component_digest``):
        components over every rank's edges with >= ``min_size`` members and
        mean edge weight > ``min_avg_w``, ordered by their first member in the
        reference node order, each as the contents of its first ``take`` live
        nodes. Collective; rank 0 gets the list, the others []."""
        g = self.g
        dev = self.device
        W = self.world
        n = g.n
        ne = int(g.num_edges) if n else 0
        if self._dcc is not None:
            out = self._digest_incremental(min_size, min_avg_w, take)
            if out is not None:
                return out
        if W == 1 and g.on_gpu and ne:
            return self._digest_world1(min_size, min_avg_w, take)
        cnt = self._host_ints(ne)[:, 0].tolist()
        if sum(cnt) <= self.DIGEST_REPLICATE_MAX:
            return self._digest_replicated(cnt, min_size, min_avg_w, take)
        if ne:
            s_num = self.num[g.e["src"].long()]
            d_num = self.num[g.e["dst"].long()]
            w = g.e["w"].double()
        else:
            s_num = d_num = torch.zeros(0, dtype=torch.long, device=dev)
            w = torch.zeros(0, dtype=torch.float64, device=dev)
        cdev = self.comm.device if self._coll else dev
        verts, lab = distributed_components(self.comm, s_num.to(cdev), d_num.to(cdev), force=self._coll)
        verts, lab = verts.to(dev), lab.to(dev)

        def home(t):
            return (t % W) if self._coll else torch.zeros_like(t)

        def route(dest, rows):
            if not self._coll:
                return rows
            got, _ = _route(self.comm, dest.to(cdev), rows.to(cdev))
            return got.to(dev)

        # members: every distinct vertex (live node or ghost endpoint), counted at its home rank
        got = route(home(verts), torch.stack([verts, lab], 1))
        if got.numel():
            uv, first = np.unique(got[:, 0].cpu().numpy(), return_index=True)
            vl = got[torch.as_tensor(first, dtype=torch.long).to(dev), 1]
            ul, cnt = torch.unique(vl, return_counts=True)
            part_size = torch.stack([ul, cnt], 1)
        else:
            part_size = torch.zeros((0, 2), dtype=torch.long, device=dev)
        # edge weight sums by the source's label; first member key by live nodes
        if s_num.numel():
            el = lab[torch.searchsorted(verts, s_num)]
            ul, inv = torch.unique(el, return_inverse=True)
            ws, wc = _seg_sum_count(inv, w, ul.numel())  # sort + scan: no contended fp64 atomics
            wc = wc.double()
            part_w = torch.stack([ul.double(), ws, wc], 1)
        else:
            part_w = torch.zeros((0, 3), dtype=torch.float64, device=dev)
        # the live nodes this rank holds that any rank's edges touch: a rank
        # touching a node through a ghost row sends (vertex, label) to the
        # ghost's holder
        rows_t = self._rows_of_nums(verts)
        hold = torch.where(rows_t >= 0, self.holder[rows_t.clamp_min(0)], torch.full_like(rows_t, -1))
        rem = (hold >= 0) & (hold != self.rank)
        got = route(hold[rem], torch.stack([verts[rem], lab[rem]], 1)) if self._coll else \
            torch.zeros((0, 2), dtype=torch.long, device=dev)
        if got.numel():
            vv = torch.cat([verts[~rem], got[:, 0]])
            ll = torch.cat([lab[~rem], got[:, 1]])
            vv, o = torch.unique(vv, return_inverse=True)
            verts, lab = vv, torch.zeros_like(vv).scatter_(0, o, ll)
        else:
            verts, lab = verts[~rem], lab[~rem]
        if verts.numel():
            rows_l = self._rows_of_nums(verts)
            okr = rows_l >= 0
            rr = rows_l.clamp_min(0)
            live = okr & (g.kind[rr] == NODE) & (g.sup[rr] == 0)
            key = (g.shard[rr].long() + 1) * (1 << NUM_BITS) + verts
            lv = torch.nonzero(live).flatten()
            ul, inv = torch.unique(lab[lv], return_inverse=True)
            fk = _seg_min(inv, key[lv], ul.numel(), BIG)
            part_f = torch.stack([ul, fk], 1)
        else:
            lv = torch.zeros(0, dtype=torch.long, device=dev)
            rows_l = key = torch.zeros(0, dtype=torch.long, device=dev)
            part_f = torch.zeros((0, 2), dtype=torch.long, device=dev)
        ps = route(home(part_size[:, 0]), part_size)
        pw = route(home(part_w[:, 0].long()), part_w)
        pf = route(home(part_f[:, 0]), part_f)
        labels = torch.unique(torch.cat([ps[:, 0], pw[:, 0].long(), pf[:, 0]]))
        qual = torch.zeros((0, 2), dtype=torch.long, device=dev)
        if labels.numel():
            L = labels.numel()
            size = torch.zeros(L, dtype=torch.long, device=dev).index_add_(0, torch.searchsorted(labels, ps[:, 0].contiguous()),
                                                                           ps[:, 1])
            wi = torch.searchsorted(labels, pw[:, 0].long())
            wsum = torch.zeros(L, dtype=torch.float64, device=dev).index_add_(0, wi, pw[:, 1])
            wcnt = torch.zeros(L, dtype=torch.float64, device=dev).index_add_(0, wi, pw[:, 2])
            fst = torch.full((L,), BIG, dtype=torch.long, device=dev).scatter_reduce_(
                0, torch.searchsorted(labels, pf[:, 0].contiguous()), pf[:, 1], "amin")
            ok = (size >= min_size) & (wcnt > 0) & (wsum / wcnt.clamp_min(1) > min_avg_w) & (fst < BIG)
            qual = torch.stack([labels[ok], fst[ok]], 1)
        qual, _ = self._gather_var(qual)  # every qualifying (label, first key), replicated
        if qual.numel() == 0:
            return []
        # each rank's first `take` live members (node-number order) per qualifying component
        mine = []
        if lv.numel():
            ql = qual[:, 0]
            o = torch.argsort(ql)
            ql_s, qf_s = ql[o], qual[o, 1]
            li = torch.searchsorted(ql_s, lab[lv]).clamp_max(ql_s.numel() - 1)
            inq = ql_s[li] == lab[lv]
            sel = lv[inq]
            if sel.numel():
                fk = qf_s[li[inq]]
                vn = verts[sel]
                oo = torch.argsort(vn)
                oo = oo[torch.sort(fk[oo], stable=True).indices]
                fk, vn, rsel = fk[oo], vn[oo], rows_l[sel][oo]
                newg = torch.ones_like(fk, dtype=torch.bool)
                newg[1:] = fk[1:] != fk[:-1]
                gstart = torch.nonzero(newg).flatten()[torch.cumsum(newg.long(), 0) - 1]
                rank_in = torch.arange(fk.numel(), device=dev) - gstart
                keepm = rank_in < take
                for f_, v_, r_ in zip(fk[keepm].tolist(), vn[keepm].tolist(), rsel[keepm].tolist()):
                    mine.append((f_, v_, g.content[r_]))
        parts = self.comm.all_gather_object(mine) if self._coll else [mine]
        if self.rank != 0:
            return []
        allm = sorted(x for p in parts for x in p)
        out: List[List[str]] = []
        last = None
        for f_, _, c in allm:
            if f_ != last:
                out.append([])
                last = f_
            if len(out[-1]) < take:
                out[-1].append(c)
        return out

    _num_mono = False  # inside a batch: live shard nodes' numbers ascend with the row

    def _check_num_mono(self) -> None:
        g = self.g
        n = g.n
        self._num_mono = False
        if n and g.on_gpu:
            with g.on_stream():
                live = torch.nonzero((g.kind[:n] == NODE) & (g.sup[:n] == 0)).flatten()
                nums = self.num[live]
                self._num_mono = bool((nums[1:] > nums[:-1]).all()) if nums.numel() > 1 else True

    def _first_contents(self, take: int = PROFILE_CONTENTS) -> List[str]:
        """Contents of the tenant's first ``take`` live nodes in the reference
        node order (shard creation order, then insertion). Rank 0 gets them."""
        g = self.g
        n = g.n
        mine = []
        if n and g.on_gpu and self._num_mono:
            # live shard nodes in number order along the rows (checked at the
            # batch start; a batch appends larger numbers): the first rows by
            # (shard, row) are the first by (shard, number) -- the one-block
            # tg_first_rows kernel, no pass over the tenant's rows
            with g.on_stream():
                r = g.first_node_rows_dev(min(take, n), super_=False)
                key = (g.shard[r].long() + 1) * (1 << NUM_BITS) + self.num[r]
                vr = torch.stack([key, r]).cpu().tolist()
                mine = [(int(a), g.content[int(b)]) for a, b in zip(*vr)]
        elif n:
            with g.on_stream():
                live = (g.kind[:n] == NODE) & (g.sup[:n] == 0)
                key = torch.where(live, (g.shard[:n].long() + 1) * (1 << NUM_BITS) + self.num[:n],
                                  torch.full((n,), BIG, dtype=torch.long, device=self.device))
                k = min(take, n)
                v, r = torch.topk(key, k, largest=False, sorted=True)
                vr = torch.stack([v, r]).cpu().tolist()  # one device read
                mine = [(int(a), g.content[int(b)]) for a, b in zip(*vr) if a < BIG]
        parts = self.comm.all_gather_object(mine) if self._coll else [mine]
        return [c for _, c in sorted(x for p in parts for x in p)[:take]] if self.rank == 0 else []

    def run_consolidation(self) -> str:
        """Collective deep consolidation (reference :935-1010) over the whole
        tenant: component digest (distributed CC), profile extraction on rank 0
        (the tenant's profile is broadcast afterwards), prune of every rank's
        weak edges. The reference's merge step is its no-op default."""
        ms = self.local
        results = []
        with tracer.stage("components", self.device):
            digest = self.component_digest(3, 0.3, PROFILE_CONTENTS)
        updates = 0
        for cs in digest:
            r = ms._extract_profile_from_contents(cs)
            if "Updated" in r:
                updates += 1
                results.append(r)
        pruned = self._sum(self.g.prune(self.prune_threshold))[0]
        if pruned > 0:
            results.append(f"✓ Pruned {pruned} weak edges")
        upd = self._sum(updates)[0]
        if upd > 0:
            results.append(f"✓ Updated {upd} profile domains")
        else:
            contents = self._first_contents(PROFILE_CONTENTS)
            if self.rank == 0 and len(contents) >= 3:
                r = ms._extract_profile_from_contents(contents)
                if "Updated" in r:
                    results.append(r)
        if self._coll:
            prof = self.comm.all_gather_object(dict(ms.profile.data) if self.rank == 0 else None)[0]
            for k, v in prof.items():
                if ms.profile.data.get(k) != v:
                    ms.profile.update_domain(k, v)
        if not results:
            results.append("✓ No consolidation actions needed")
        return "\n".join(results)

    def cluster_pass(self) -> Dict:
        hp = self.hierarchy_params or {"fine": 4096, "top": 64, "iters": 2}
        out = self.g.cluster_pass(hp["fine"], hp["top"], hp["iters"], comm=self.comm if self._coll else None)
        self._build_reach()
        return out

    @property
    def profile(self):
        return self.local.profile

    def get_stats(self) -> Dict:
        nodes, edges = self._sum(self.g.num_nodes(), self.g.num_edges)
        return {"user_id": self.user_id, "ranks": self.world, "total_nodes": nodes, "total_edges": edges,
                "local_nodes": self.g.num_nodes(), "local_edges": self.g.num_edges,
                "conversations": self.conversation_count, "next_node_id": self.next_id}

    def close(self) -> None:
        self.local.close()
