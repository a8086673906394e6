"""DeviceGraph: an HBM-resident memory graph for consolidation at scale
(BASELINE.json config 4; SURVEY.md §3.3 hot loops).

The reference keeps the graph as Python objects and runs every consolidation
step as Python loops (dedupe :719-742, linking :797-889, decay/prune
memory_shard.py:64-84, eviction :535-578, components buffer_graph.py:99-120,
super-nodes :893-933). Here one tenant's (or one GPU's share of a) buffer is
structure-of-arrays in HBM and every step is a kernel:

  ingest(facts)   dedupe = fused MFMA top-1 (K5) -> append rows -> chain edges
                  -> within-shard top-3 (label-filtered, K6) + global top-3 (K6)
  maintain()      decay + prune with stable compaction (K10) -> importance
                  select + tombstone + dead-edge compaction (K11)
  components()    hook/compress label propagation (K9)
  cluster()       k-means super-nodes: assign = fused top-1, update = segmented
                  mean (K16/K8), see :mod:`lazzaro_amd.index.kmeans`
  boost(seeds)    CSR neighbour boost (K12)

Semantics follow the reference's constants (App. B): dedupe cos > 0.95
(salience=max, access+1), link top-3 cos > 0.5 with w = 0.8*cos, chain edge
0.5, decay 0.01/conversation with salience floor 0.2, prune w < 0.5, eviction
importance 0.5*sal + 0.3*min(1, acc/10) + 0.2/(1+days).
"""
from __future__ import annotations

import time
from typing import Dict, Optional, Tuple

import torch

from ..ops import graph_ops as G
from ..ops.search import flat_topk, flat_topk_dual

NEG_INF = float("-inf")


def _pad64(d):
    return (d + 63) // 64 * 64


def csr_undirected(src: torch.Tensor, dst: torch.Tensor, n: int):
    """Undirected CSR built with tensor ops on the tensors' device: arcs
    ordered per source by edge index, self-loops once -- the same layout as
    the native host build (csrc/runtime/graph_host.cpp build_csr).
    Returns (off int64 [n+1], adj int32, eid int32)."""
    dev = src.device
    s, d = src.long(), dst.long()
    ne = s.numel()
    frm = torch.stack([s, d], 1).reshape(-1)
    to = torch.stack([d, s], 1).reshape(-1)
    eid = torch.arange(ne, device=dev).repeat_interleave(2)
    ok = torch.ones(2 * ne, dtype=torch.bool, device=dev)
    ok[1::2] = s != d
    frm, to, eid = frm[ok], to[ok], eid[ok]
    order = torch.sort(frm, stable=True).indices
    off = torch.zeros(n + 1, dtype=torch.int64, device=dev)
    off[1:] = torch.cumsum(torch.bincount(frm, minlength=n)[:n], 0)
    return off, to[order].to(torch.int32), eid[order].to(torch.int32)


class DeviceGraph:
    def __init__(self, dim: int, device=None, capacity: int = 1 << 16, edge_capacity: int = 1 << 18):
        self.device = torch.device(device) if device is not None else torch.device("cpu")
        self.dim = dim
        self.Dp = _pad64(dim) if self.device.type == "cuda" else dim
        self.cap = 0
        self.n = 0
        self._alloc(capacity)
        z = lambda dt: torch.zeros(0, dtype=dt, device=self.device)  # noqa: E731
        self.edges: Dict[str, torch.Tensor] = {"src": z(torch.int32), "dst": z(torch.int32),
                                               "w": z(torch.float32), "co": z(torch.int32),
                                               "lu": z(torch.float64)}
        self.stats = {"deduped": 0, "inserted": 0, "linked": 0, "pruned": 0, "evicted": 0}

    # ------------------------------------------------------------------ storage
    def _alloc(self, cap: int) -> None:
        dev, n = self.device, self.n
        dt = torch.bfloat16 if dev.type == "cuda" else torch.float32
        new = {
            "emb": torch.zeros((cap, self.Dp), dtype=dt, device=dev),
            "sal": torch.zeros(cap, dtype=torch.float32, device=dev),
            "acc": torch.zeros(cap, dtype=torch.int32, device=dev),
            "last": torch.zeros(cap, dtype=torch.float64, device=dev),
            "ts": torch.zeros(cap, dtype=torch.float64, device=dev),
            "shard": torch.full((cap,), -1, dtype=torch.int32, device=dev),
            "alive": torch.zeros(cap, dtype=torch.uint8, device=dev),
            "super": torch.zeros(cap, dtype=torch.uint8, device=dev),
            "bias": torch.full((cap,), NEG_INF, dtype=torch.float32, device=dev),
        }
        if self.cap:
            for k, v in new.items():
                v[:n] = getattr(self, k)[:n]
        for k, v in new.items():
            setattr(self, k, v)
        self.cap = cap

    def reserve(self, n: int) -> None:
        if n > self.cap:
            self._alloc(max(n, int(self.cap * 1.5) + 1))

    @property
    def num_edges(self) -> int:
        return int(self.edges["src"].numel())

    def num_alive(self) -> int:
        return int(self.alive[: self.n].sum().item())

    def add_nodes(self, emb: torch.Tensor, shard: torch.Tensor, salience: torch.Tensor,
                  now: Optional[float] = None, is_super: bool = False) -> torch.Tensor:
        """Append unit-norm rows; returns their row indices."""
        m = emb.shape[0]
        now = time.time() if now is None else now
        self.reserve(self.n + m)
        r0, r1 = self.n, self.n + m
        self.emb[r0:r1, : emb.shape[1]] = emb.to(self.emb.dtype)
        self.sal[r0:r1] = salience.to(self.device, torch.float32)
        self.acc[r0:r1] = 0
        self.last[r0:r1] = now
        self.ts[r0:r1] = now
        self.shard[r0:r1] = shard.to(self.device, torch.int32)
        self.alive[r0:r1] = 1
        self.super[r0:r1] = 1 if is_super else 0
        self.bias[r0:r1] = NEG_INF if is_super else 0.0
        self.n = r1
        return torch.arange(r0, r1, device=self.device)

    def add_edges(self, src, dst, w, now: Optional[float] = None) -> None:
        if src.numel() == 0:
            return
        now = time.time() if now is None else now
        e = self.edges
        e["src"] = torch.cat([e["src"], src.to(torch.int32)])
        e["dst"] = torch.cat([e["dst"], dst.to(torch.int32)])
        e["w"] = torch.cat([e["w"], w.to(torch.float32)])
        e["co"] = torch.cat([e["co"], torch.ones_like(src, dtype=torch.int32)])
        e["lu"] = torch.cat([e["lu"], torch.full((src.numel(),), now, dtype=torch.float64, device=self.device)])

    # ------------------------------------------------------------------ search
    def _search(self, q: torch.Tensor, k: int, row_label=None, q_label=None, bias=None):
        n = self.n
        if n == 0:
            m = q.shape[0]
            return (torch.full((m, k), NEG_INF, device=self.device),
                    torch.full((m, k), -1, dtype=torch.long, device=self.device))
        b = self.bias[:n] if bias is None else bias
        return flat_topk(self.emb[:n], q, k, bias=b, row_label=row_label, q_label=q_label)

    # ------------------------------------------------------------------ ingest
    def ingest(self, q: torch.Tensor, shard: torch.Tensor, salience: torch.Tensor,
               now: Optional[float] = None, dedupe_thr: float = 0.95, link_k: int = 3,
               link_thr: float = 0.5, link_scale: float = 0.8, chain_w: float = 0.5,
               dedupe: bool = True, global_links: bool = True, shard_hits=None) -> Dict[str, int]:
        """One consolidation batch of M facts (unit rows ``q`` [M, Dp]).

        All searches run over the rows that existed before the batch (the
        reference links new facts to EXISTING memories, memory_system.py:
        816-821, 842-847) and come from ONE scan (``flat_topk_dual``): the
        unfiltered top-k gives dedupe (top-1 > 0.95) and global links, the
        shard-filtered top-k gives within-shard links.
        ``dedupe``/``global_links`` False when a sharded caller already did the
        global search; it may then pass its shard-filtered hits (``shard_hits``
        = (scores, rows) aligned with ``q``) from the same fused scan."""
        now = time.time() if now is None else now
        q = q.to(self.emb.dtype)
        M = q.shape[0]
        if M == 0:
            return {"deduped": 0, "inserted": 0, "linked": 0}
        sh_all = shard.to(self.device).to(torch.int32)
        if shard_hits is not None:
            sw_all, rw_all = shard_hits
            sg_all = rg_all = None
        elif dedupe or global_links:
            (sg_all, rg_all), (sw_all, rw_all) = self._search_dual(q, link_k, sh_all)
        else:
            sw_all, rw_all = self._search(q, link_k, row_label=self.shard[: self.n], q_label=sh_all)
            sg_all = rg_all = None
        if dedupe:
            s1, r1 = sg_all[:, 0], rg_all[:, 0]
            dup = (r1 >= 0) & (s1 > dedupe_thr)
        else:
            dup = torch.zeros(M, dtype=torch.bool, device=self.device)
            r1 = torch.full((M,), -1, dtype=torch.long, device=self.device)
        if bool(dup.any()):
            rows = r1[dup]
            self.sal.scatter_reduce_(0, rows, salience.to(self.device)[dup].float(), "amax", include_self=True)
            self.acc.index_add_(0, rows, torch.ones_like(rows, dtype=torch.int32))
            self.last[rows] = now
        keep = ~dup
        nk = int(keep.sum().item())
        out = {"deduped": M - nk, "inserted": nk, "linked": 0}
        if nk == 0:
            return out
        qn, sh, sl = q[keep], sh_all[keep], salience.to(self.device)[keep]
        rows = self.add_nodes(qn, sh, sl, now)
        sw, rw = sw_all[keep], rw_all[keep]
        if global_links and sg_all is not None:
            sg, rg = sg_all[keep], rg_all[keep]
        else:
            sg = torch.full_like(sw, NEG_INF)
            rg = torch.full_like(rw, -1)
        src = rows[:, None].expand(-1, link_k)
        mw = (rw >= 0) & (sw > link_thr)
        mg = (rg >= 0) & (sg > link_thr)
        key_w = src[mw] * (1 << 32) + rw[mw]
        key_g = src[mg] * (1 << 32) + rg[mg]
        mg_new = ~torch.isin(key_g, key_w)  # skip pairs already linked in-shard
        es = torch.cat([src[mw], src[mg][mg_new]])
        ed = torch.cat([rw[mw], rg[mg][mg_new]])
        ew = torch.cat([sw[mw], sg[mg][mg_new]]) * link_scale
        # chain edges between consecutive new facts of the same shard
        if nk > 1:
            same = sh[1:] == sh[:-1]
            es = torch.cat([es, rows[:-1][same]])
            ed = torch.cat([ed, rows[1:][same]])
            ew = torch.cat([ew, torch.full((int(same.sum()),), chain_w, device=self.device)])
        self.add_edges(es, ed, ew, now)
        out["linked"] = int(es.numel())
        for k_ in out:
            self.stats[k_] += out[k_]
        return out

    def ingest_fixed(self, q: torch.Tensor, shard: torch.Tensor, salience: torch.Tensor, dead: torch.Tensor,
                     shard_hits, global_hits=None, now: Optional[float] = None, link_k: int = 3,
                     link_thr: float = 0.5, link_scale: float = 0.8, chain_w: float = 0.5,
                     invalid_w: float = -1.0) -> Dict[str, torch.Tensor]:
        """Host-sync-free form of :meth:`ingest` for a pipelined caller that
        already searched (``shard_hits`` / ``global_hits`` = (scores, rows)
        aligned with ``q``) and decided the duplicates (``dead`` bool [M]).

        Every shape is fixed by M, so no step waits for a device count: all M
        facts get rows, the duplicates' rows are tombstoned at once (alive 0,
        bias -inf: invisible to search, eviction and links), and all M*(2k+1)
        candidate edges are appended with weight ``invalid_w`` where the link
        is not taken -- the next decay/prune compaction removes them, exactly
        as it removes weak edges. Same links as :meth:`ingest`: top-k in-shard
        and global hits above ``link_thr`` (w = link_scale*cos, a global hit
        already linked in-shard is skipped), chain edges between consecutive
        KEPT facts of the same shard. Returns device counts (no .item())."""
        now = time.time() if now is None else now
        M = q.shape[0]
        dev = self.device
        if M == 0:
            z = torch.zeros((), dtype=torch.int64, device=dev)
            return {"deduped": z, "inserted": z, "linked": z, "placeholders": z}
        dead = dead.to(dev).bool()
        keep = ~dead
        sh = shard.to(dev).to(torch.int32)
        rows = self.add_nodes(q.to(self.emb.dtype), sh, salience.to(dev), now)
        self.alive[rows] = keep.to(torch.uint8)
        self.bias[rows] = torch.where(keep, 0.0, NEG_INF)
        sw, rw = shard_hits
        src = rows[:, None].expand(-1, link_k)
        mw = (rw >= 0) & (sw > link_thr) & keep[:, None]
        es, ed, ew = [src.reshape(-1)], [rw.reshape(-1)], [torch.where(mw, sw * link_scale, invalid_w).reshape(-1)]
        n_link = mw.sum()
        if global_hits is not None:
            sg, rg = global_hits
            mg = (rg >= 0) & (sg > link_thr) & keep[:, None]
            in_shard = ((rg[:, :, None] == rw[:, None, :]) & mw[:, None, :]).any(dim=2)
            mg = mg & ~in_shard
            es.append(src.reshape(-1))
            ed.append(rg.reshape(-1))
            ew.append(torch.where(mg, sg * link_scale, invalid_w).reshape(-1))
            n_link = n_link + mg.sum()
        # chain: each kept fact to the previous kept fact of the batch, same shard
        idx = torch.arange(M, device=dev)
        prev = torch.cummax(torch.where(keep, idx, -1), 0).values
        prev = torch.cat([torch.full((1,), -1, dtype=prev.dtype, device=dev), prev[:-1]])
        pc = prev.clamp_min(0)
        mc = keep & (prev >= 0) & (sh[pc] == sh)
        es.append(rows[pc])
        ed.append(rows)
        ew.append(torch.where(mc, torch.full_like(salience.to(dev).float(), chain_w), invalid_w))
        n_link = n_link + mc.sum()
        self.add_edges(torch.cat(es), torch.cat(ed), torch.cat(ew).float(), now)
        n_keep = keep.sum()
        appended = sum(int(t.numel()) for t in es)
        return {"deduped": M - n_keep, "inserted": n_keep, "linked": n_link, "placeholders": appended - n_link}

    def _search_dual(self, q: torch.Tensor, k: int, q_label: torch.Tensor):
        n = self.n
        if n == 0:
            m = q.shape[0]
            e = (torch.full((m, k), NEG_INF, device=self.device),
                 torch.full((m, k), -1, dtype=torch.long, device=self.device))
            return e, e
        return flat_topk_dual(self.emb[:n], q, k, bias=self.bias[:n], row_label=self.shard[:n], q_label=q_label)

    # ------------------------------------------------------------------ maintenance
    def decay_prune(self, rate: float = 0.01, threshold: float = 0.5, conversations: int = 1) -> int:
        """Apply ``conversations`` rounds of decay in one pass (exact for both
        the edge product and the salience floor recurrence), then prune."""
        eff = 1.0 - (1.0 - rate) ** conversations
        n = self.n
        live_sal = self.sal[:n]
        self.edges, pruned = G.decay_prune(self.edges, live_sal, self.alive[:n], eff, threshold)
        self.stats["pruned"] += pruned
        return pruned

    def enforce_limit(self, max_nodes: int, now: Optional[float] = None, alive_upper: Optional[int] = None) -> int:
        """``alive_upper``: a host-side upper bound on live rows (e.g. rows ever
        added); when it is within the limit the device count is not read."""
        if alive_upper is not None and alive_upper <= max_nodes:
            return 0
        n_alive = self.num_alive()
        excess = n_alive - max_nodes
        if excess <= 0:
            return 0
        now = time.time() if now is None else now
        n = self.n
        score = G.importance(self.sal[:n], self.acc[:n], self.last[:n], self.alive[:n], self.super[:n], now)
        victims = G.select_lowest(score, excess)
        G.mark_dead(self.alive, victims)
        self.bias[victims] = NEG_INF
        self.edges = G.drop_dead_edges(self.edges, self.alive[:n])
        self.stats["evicted"] += int(victims.numel())
        return int(victims.numel())

    def components(self, min_w: float = 0.0) -> torch.Tensor:
        e = self.edges
        return G.connected_components(e["src"], e["dst"], self.n, e["w"], min_w)

    def csr(self):
        """Undirected CSR, per-source arcs in edge-index order (self-loops once).
        Device graphs build it in HBM (stable sort of the arc sources + bincount
        scan, no host round trip); CPU graphs use the native runtime build."""
        e = self.edges
        if self.device.type == "cuda":
            return csr_undirected(e["src"], e["dst"], self.n)
        from ..store.colstore import _rt
        off, adj, eid = _rt().build_csr(e["src"].cpu().numpy(), e["dst"].cpu().numpy(), self.n, True)
        t = lambda a: torch.from_numpy(a).to(self.device)  # noqa: E731
        return t(off), t(adj), t(eid)

    def boost(self, seeds: torch.Tensor, now: Optional[float] = None, csr=None) -> int:
        now = time.time() if now is None else now
        off, adj, eid = csr if csr is not None else self.csr()
        return G.neighbor_boost(off, adj, eid, self.edges["w"], seeds.to(self.device), self.sal, self.last, now)

    def search(self, q: torch.Tensor, k: int = 10):
        return self._search(q.to(self.emb.dtype), k)
