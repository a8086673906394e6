"""Row-sharded search and distributed graph maintenance.

* :class:`ShardedIndex` -- one logical index whose rows are split across ranks
  (a tenant larger than one GPU, or a global cross-tenant index). Search is
  local fused top-k (K1) -> all-gather of (score, global id) candidates (C1,
  Q*k*12 bytes per rank: latency-bound, tens of microseconds on xGMI) -> merge
  (K2). Every rank gets the same exact global top-k.
* :func:`distributed_components` -- connected components over edges spread
  across ranks (C5): local hook/compress on a replicated parent array, then an
  all-reduce(MIN) of the parents until no rank changes anything.
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
    """Merge candidate lists [nq, C] -> top-k by (score desc, id asc)."""
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


def distributed_components(comm: Communicator, src: torch.Tensor, dst: torch.Tensor, n_global: int,
                           w: Optional[torch.Tensor] = None, min_w: float = 0.0, max_rounds: int = 64) -> torch.Tensor:
    """Global component labels (min node id) for edges partitioned across ranks."""
    label = G.connected_components(src, dst, n_global, w, min_w).to(torch.int64)
    for _ in range(max_rounds):
        before = label.clone()
        comm.all_reduce(label, "min")
        # re-hook locally: edges whose endpoints now carry different labels
        ls = label[src.long()]
        ld = label[dst.long()]
        s2 = torch.cat([ls, torch.arange(n_global, device=label.device)])
        d2 = torch.cat([ld, label])
        label = G.connected_components(s2.to(torch.int32), d2.to(torch.int32), n_global).to(torch.int64)
        changed = torch.tensor([int(not torch.equal(label, before))], device=label.device)
        comm.all_reduce(changed, "max")
        if int(changed.item()) == 0:
            break
    return label
