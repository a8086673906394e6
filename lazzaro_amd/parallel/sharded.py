"""Row-sharded search and distributed graph maintenance.

* :class:`ShardedIndex` -- one logical index whose rows are split across ranks
  (a tenant larger than one GPU, or a global cross-tenant index). Search is
  local fused top-k (K1) -> all-gather of (score, global id) candidates (C1,
  Q*k*12 bytes per rank: latency-bound, tens of microseconds on xGMI) -> merge
  (K2). Every rank gets the same exact global top-k.
* :func:`distributed_components` -- connected components over edges spread
  across ranks (C5): local hook/compress once, then boundary-label exchange
  (all-to-all-v of only the shared vertices whose label changed).
"""
from __future__ import annotations

from typing import Optional, Tuple

import torch

from ..index.arena import VectorArena
from ..ops import graph_ops as G
from ..ops.search import flat_topk
from .comm import Communicator

NEG_INF = float("-inf")


def merge_topk(scores: torch.Tensor, ids: torch.Tensor, k: int) -> Tuple[torch.Tensor, torch.Tensor]:
    """Merge candidate lists [nq, C] -> top-k by (score desc, id asc).

    Device tensors (k <= 32) run the K2 ``topk_merge64_kernel`` (search.hip):
    one wave per query, no sort of the gathered lists. Empty slots (id < 0)
    sort last and come back as (-inf, -1) in both paths."""
    if scores.is_cuda and 0 < k <= 32 and scores.shape[1] >= k:
        from ..ops import _lib

        nq, nc = scores.shape
        s = scores.float().contiguous()
        i = ids.long().contiguous()
        os_ = torch.empty((nq, k), dtype=torch.float32, device=s.device)
        oi = torch.empty((nq, k), dtype=torch.long, device=s.device)
        _lib.check(_lib.lib().lzk_topk_merge64(s.data_ptr(), i.data_ptr(), nc, nq, k, os_.data_ptr(), oi.data_ptr(),
                                               _lib.stream_ptr(s.device)), "lzk_topk_merge64")
        return os_, oi
    big = torch.iinfo(torch.int64).max
    key_ids = torch.where(ids < 0, torch.full_like(ids, big), ids)
    o = torch.argsort(key_ids, dim=1, stable=True)
    s = torch.gather(scores, 1, o)
    i = torch.gather(ids, 1, o)
    o = torch.argsort(-s, dim=1, stable=True)[:, :k]
    return torch.gather(s, 1, o), torch.gather(i, 1, o)


class ShardedIndex:
    """Rows [offset, offset + n_local) of a global index live on this rank."""

    def __init__(self, comm: Communicator, X: torch.Tensor, row_offset: int, bias: Optional[torch.Tensor] = None):
        self.comm = comm
        self.X = X
        self.offset = int(row_offset)
        self.bias = bias

    @classmethod
    def partition(cls, comm: Communicator, X_full: torch.Tensor) -> "ShardedIndex":
        """Evenly split a full matrix (test helper: every rank holds X_full)."""
        n = X_full.shape[0]
        per = (n + comm.world - 1) // comm.world
        lo, hi = comm.rank * per, min(n, (comm.rank + 1) * per)
        return cls(comm, X_full[lo:hi].contiguous(), lo)

    def search(self, Q: torch.Tensor, k: int) -> Tuple[torch.Tensor, torch.Tensor]:
        s, i = flat_topk(self.X, Q, k, bias=self.bias, idx_offset=self.offset)
        if self.comm.world == 1:
            return s, i
        nq = Q.shape[0]
        gs = self.comm.all_gather_rows(s)  # [world*nq, k]
        gi = self.comm.all_gather_rows(i)
        gs = gs.view(self.comm.world, nq, k).permute(1, 0, 2).reshape(nq, -1)
        gi = gi.view(self.comm.world, nq, k).permute(1, 0, 2).reshape(nq, -1)
        return merge_topk(gs, gi, k)


def _route(comm: Communicator, dest: torch.Tensor, rows: torch.Tensor) -> Tuple[torch.Tensor, torch.Tensor]:
    """Send ``rows[i]`` to rank ``dest[i]`` (one all-to-all-v). Returns the
    rows received and the source rank of each."""
    world = comm.world
    order = torch.argsort(dest, stable=True)
    counts = torch.bincount(dest, minlength=world).to(torch.int64)
    rc = comm.exchange_counts(counts.to(comm.device)).cpu()
    got = comm.all_to_all_v(rows[order].to(comm.device), counts.tolist(), rc.tolist()).to(rows.device)
    return got, torch.repeat_interleave(torch.arange(world, device=rows.device), rc.to(rows.device))


def distributed_components(comm: Communicator, src: torch.Tensor, dst: torch.Tensor, n_global: Optional[int] = None,
                           w: Optional[torch.Tensor] = None, min_w: float = 0.0, max_rounds: int = 1 << 20,
                           stats: Optional[dict] = None, force: bool = False) -> Tuple[torch.Tensor, torch.Tensor]:
    """Connected components of a graph whose edges are spread over ranks
    (the reference's single-process DFS is
    buffer_graph.py:99-120). Returns ``(verts, labels)``: the vertices this
    rank's edges touch (sorted global ids) and their global component label
    (the smallest vertex id of the component).

    Boundary-label exchange, no replicated state: each rank contracts its own
    edges once (device hook/compress CC over compact local ids); every vertex
    is owned by rank ``v % world``. Round 0 sends each touched vertex's label
    to its owner, which learns the vertices that several ranks touch (the
    boundary) and who subscribes to them. Every later round sends only
    boundary vertices whose label went down, the owner forwards new minima to
    the subscribers, and each rank re-propagates inside its local components
    (a segmented min). Per-round traffic is O(changed boundary vertices), not
    O(n_global); the round count is bounded by the diameter of the graph of
    local components. ``n_global`` is accepted for API compatibility."""
    dev = src.device
    s, d = src.long(), dst.long()
    if w is not None:
        keep = w >= min_w
        s, d = s[keep], d[keep]
    E = s.numel()
    verts, inv = torch.unique(torch.cat([s, d]), return_inverse=True)
    nl = verts.numel()
    comp = G.connected_components(inv[:E].to(torch.int32), inv[E:].to(torch.int32), nl).to(dev).long() \
        if nl else torch.zeros(0, dtype=torch.long, device=dev)
    big = torch.iinfo(torch.int64).max

    from ..engine.tenant_graph import _seg_min

    def propagate(lab):  # segmented min by sorts: a giant local component is one key
        return _seg_min(comp, lab, nl, big)[comp]

    label = propagate(verts.clone())
    st = {"rounds": 0, "rows_sent": 0, "first_round_rows": int(nl)}
    world = comm.world
    if world == 1 and not force:  # (force: the exchange rounds run even at world 1)
        if stats is not None:
            stats.update(st)
        return verts, label
    # round 0: subscribe every touched vertex at its owner
    got, frm = _route(comm, verts % world, torch.stack([verts, label], 1))
    uv, uinv = torch.unique(got[:, 0], return_inverse=True)
    cur = torch.full((uv.numel(),), big, dtype=torch.int64, device=dev).scatter_reduce(0, uinv, got[:, 1], "amin")
    shared = torch.bincount(uinv, minlength=uv.numel()) >= 2
    sub = shared[uinv]
    sub_v, sub_rank = uinv[sub], frm[sub]  # subscriptions to boundary vertices
    o = torch.argsort(sub_v, stable=True)
    sub_v, sub_rank = sub_v[o], sub_rank[o]
    reply = torch.stack([uv[sub_v], cur[sub_v]], 1)
    back, _ = _route(comm, sub_rank, reply)
    bpos = torch.searchsorted(verts, back[:, 0])  # this rank's boundary vertices
    is_b = torch.zeros(nl, dtype=torch.bool, device=dev)
    is_b[bpos] = True
    bnd = torch.nonzero(is_b).flatten()
    for rnd in range(max_rounds):
        new = label.clone().scatter_reduce_(0, bpos, back[:, 1], "amin")
        new = propagate(new)
        dec = bnd[new[bnd] < label[bnd]]
        label = new
        msg = torch.stack([verts[dec], label[dec]], 1)
        st["rounds"] = rnd + 1
        st["rows_sent"] += int(dec.numel())
        flag = torch.tensor([int(dec.numel())], dtype=torch.int64, device=comm.device)
        comm.all_reduce(flag, "max")
        if int(flag.item()) == 0:
            break
        got, _ = _route(comm, msg[:, 0] % world, msg)
        gi = torch.searchsorted(uv, got[:, 0])
        nxt = cur.clone().scatter_reduce_(0, gi, got[:, 1], "amin")
        chg = nxt < cur
        cur = nxt
        sel = chg[sub_v]
        back, _ = _route(comm, sub_rank[sel], torch.stack([uv[sub_v[sel]], cur[sub_v[sel]]], 1))
        bpos = torch.searchsorted(verts, back[:, 0])
    if stats is not None:
        stats.update(st)
    return verts, label
