"""HBM vector arena: the device-resident replacement for a LanceDB vector column.

One :class:`VectorArena` holds one tenant's (or one shard's) vectors as a
contiguous ``[capacity, Dpad]`` bf16 matrix on the GPU (Dpad = D rounded up to
64 so the MFMA kernel's K loop needs no tail), plus

* ``sqn``   fp32 squared norms (exact, computed from the fp32 input) -> L2 bias
* ``bias``  fp32 0 / -inf per row: tombstones cost nothing in the scan
* ``X32``   optional exact fp32 copy used to re-rank the kernel's candidates so
            results match an fp32 reference bit-for-bit in ordering

Capacity grows geometrically (amortised O(1) appends); deletes are tombstones,
compaction runs when more than half the rows are dead. Rows map to string ids
(duplicates allowed, like repeated LanceDB ``add`` calls).

Search = ``ops.flat_topk`` (hand-written MFMA kernel) for k <= 16, candidate
width min(16, 4k) then an fp32 re-rank of those few rows.
"""
from __future__ import annotations

from typing import Dict, Iterable, List, Optional, Sequence, Tuple

import numpy as np
import torch

from ..ops import search as S
from ..utils.device import default_device

NEG_INF = float("-inf")


def _pad64(d: int) -> int:
    return (d + 63) // 64 * 64


def multi_arena_search(arenas: Sequence["VectorArena"], queries, k: int, metric: str = "l2"):
    """Query q searches arenas[q] only; one segment-kernel launch for the
    whole batch (ops.search.segment_topk). Returns (scores, rows) like
    :meth:`VectorArena.search_rows` (score = -L2^2 / cosine / dot)."""
    nq = len(arenas)
    qf = torch.as_tensor(np.asarray(queries, dtype=np.float32)) if not torch.is_tensor(queries) else queries.float()
    dev = arenas[0].device if nq else torch.device("cpu")
    qf = qf.to(dev)
    if metric == "cosine":
        qf = qf / qf.norm(dim=1, keepdim=True).clamp_min(1e-30)
    segs = [a.segment(metric) for a in arenas]
    rows = [s[0] for s in segs]
    dt = rows[0].dtype if nq else torch.float32
    width = max(r.shape[1] for r in rows) if nq else 0
    D = qf.shape[1]
    ok = all(r.dtype == dt and (r.shape[0] == 0 or r.shape[1] == width) for r in rows)
    if not ok:
        raise ValueError("multi_arena_search: arenas of different dtype / width in one batch")
    Q = torch.zeros((nq, width), dtype=dt, device=dev)
    Q[:, :D] = qf.to(dt)
    # empty segments still need a row pointer of the common stride
    filler = next((r for r in rows if r.shape[0] > 0), None)
    if filler is None:
        return (torch.full((nq, k), NEG_INF, device=dev), torch.full((nq, k), -1, dtype=torch.long, device=dev))
    rows = [r if r.shape[0] > 0 else filler[:0] for r in rows]
    zero = torch.zeros(1, dtype=torch.float32, device=dev)
    biases = [s[1] if s[1] is not None else zero for s in segs]
    scales = [s[2] if s[2] is not None else torch.ones(max(1, r.shape[0]), device=dev)
              for s, r in zip(segs, rows)] if metric == "cosine" else None
    alpha = 2.0 if metric == "l2" else 1.0
    qbias = -(qf * qf).sum(1) if metric == "l2" else None
    return S.segment_topk(rows, Q, k, biases=biases, scales=scales, alpha=alpha, qbias=qbias)


class VectorArena:
    def __init__(self, dim: Optional[int] = None, device=None, capacity: int = 256,
                 keep_fp32: bool = True, store_dtype: Optional[torch.dtype] = None):
        self.device = torch.device(device) if device is not None else default_device()
        self.on_gpu = self.device.type == "cuda"
        self.store_dtype = store_dtype or (torch.bfloat16 if self.on_gpu else torch.float32)
        self.keep_fp32 = keep_fp32 and self.on_gpu
        self.dim = dim
        self.cap = 0
        self.n = 0
        self.n_dead = 0
        self.ids: List[Optional[str]] = []
        self.rows_of: Dict[str, List[int]] = {}
        self.X = self.X32 = self.sqn = self.bias = None
        self._init_cap = capacity
        self.version = 0  # bumps on every mutation (cache invalidation)
        self.layout_epoch = 0  # bumps when row indices change (clear / compact)
        self.ivf: Optional["ArenaIVF"] = None

    # ------------------------------------------------------------------ alloc
    def _alloc(self, cap: int) -> None:
        D = self.dim
        Dp = _pad64(D) if self.on_gpu else D
        X = torch.zeros((cap, Dp), dtype=self.store_dtype, device=self.device)
        sqn = torch.zeros(cap, dtype=torch.float32, device=self.device)
        bias = torch.full((cap,), NEG_INF, dtype=torch.float32, device=self.device)
        X32 = torch.zeros((cap, D), dtype=torch.float32, device=self.device) if self.keep_fp32 else None
        if self.cap:
            X[: self.n] = self.X[: self.n]
            sqn[: self.n] = self.sqn[: self.n]
            bias[: self.n] = self.bias[: self.n]
            if X32 is not None:
                X32[: self.n] = self.X32[: self.n]
        self.X, self.sqn, self.bias, self.X32 = X, sqn, bias, X32
        self.cap = cap

    def reserve(self, n: int) -> None:
        if n > self.cap:
            self._alloc(max(n, self._init_cap, int(self.cap * 1.5) + 1))

    # -------------------------------------------------------------- mutation
    def add(self, ids: Sequence[str], vecs) -> None:
        if len(ids) == 0:
            return
        v = torch.as_tensor(np.asarray(vecs, dtype=np.float32)) if not torch.is_tensor(vecs) else vecs.float()
        if v.dim() == 1:
            v = v[None, :]
        if self.dim is None:
            self.dim = int(v.shape[1])
        if v.shape[1] != self.dim:
            raise ValueError(f"vector dim {v.shape[1]} != arena dim {self.dim}")
        m = v.shape[0]
        self.reserve(self.n + m)
        v = v.to(self.device, non_blocking=True)
        r0, r1 = self.n, self.n + m
        self.X[r0:r1, : self.dim] = v.to(self.store_dtype)
        if self.X32 is not None:
            self.X32[r0:r1] = v
        self.sqn[r0:r1] = (v.double() ** 2).sum(1).float()
        self.bias[r0:r1] = 0.0
        for j, i in enumerate(ids):
            self.ids.append(i)
            self.rows_of.setdefault(i, []).append(r0 + j)
        self.n = r1
        self.version += 1

    def delete(self, ids: Iterable[str]) -> int:
        rows = []
        for i in ids:
            rs = self.rows_of.pop(i, None)
            if rs:
                rows.extend(rs)
        if not rows:
            return 0
        for r in rows:
            self.ids[r] = None
        t = torch.as_tensor(rows, dtype=torch.long, device=self.device)
        self.bias[t] = NEG_INF
        self.n_dead += len(rows)
        self.version += 1
        if self.n_dead * 2 > self.n and self.n > 64:
            self.compact()
        return len(rows)

    def clear(self) -> None:
        self.n = self.n_dead = 0
        self.ids = []
        self.rows_of = {}
        if self.bias is not None:
            self.bias.fill_(NEG_INF)
        self.version += 1
        self.layout_epoch += 1

    def compact(self) -> None:
        live = [r for r in range(self.n) if self.ids[r] is not None]
        idx = torch.as_tensor(live, dtype=torch.long, device=self.device)
        m = len(live)
        self.X[:m] = self.X[idx]
        self.sqn[:m] = self.sqn[idx]
        self.bias[:m] = 0.0
        self.bias[m: self.n] = NEG_INF
        if self.X32 is not None:
            self.X32[:m] = self.X32[idx]
        self.ids = [self.ids[r] for r in live]
        self.rows_of = {}
        for r, i in enumerate(self.ids):
            self.rows_of.setdefault(i, []).append(r)
        self.n, self.n_dead = m, 0
        self.version += 1
        self.layout_epoch += 1

    def __len__(self) -> int:
        return self.n - self.n_dead

    # ---------------------------------------------------------------- search
    def _queries(self, q) -> torch.Tensor:
        qt = torch.as_tensor(np.asarray(q, dtype=np.float32)) if not torch.is_tensor(q) else q.float()
        if qt.dim() == 1:
            qt = qt[None, :]
        if qt.shape[1] != self.dim:
            raise ValueError(f"query dim {qt.shape[1]} != arena dim {self.dim}")
        return qt.to(self.device)

    def search_rows(self, q, k: int, metric: str = "l2") -> Tuple[torch.Tensor, torch.Tensor]:
        """Top-k rows per query. Returns (score, row) with score = -L2^2 for
        ``l2``, cosine for ``cosine``, dot for ``ip`` (higher = closer)."""
        qf = self._queries(q)
        nq = qf.shape[0]
        if self.n == 0 or len(self) == 0:
            return (torch.full((nq, k), NEG_INF, device=self.device),
                    torch.full((nq, k), -1, dtype=torch.long, device=self.device))
        if self.ivf is not None and len(self) >= self.ivf.min_rows:
            return self.ivf.search(qf, k, metric)
        n = self.n
        if metric == "cosine":
            qn = qf / qf.norm(dim=1, keepdim=True).clamp_min(1e-30)
        else:
            qn = qf
        if not self.on_gpu:
            Xf = self.X[:n]
            if metric == "cosine":
                norms = self.sqn[:n].sqrt().clamp_min(1e-30)
                s = (qn @ Xf.T) / norms[None, :] + self.bias[:n][None, :]
            elif metric == "l2":
                s = 2.0 * (qn @ Xf.T) - self.sqn[:n][None, :] + self.bias[:n][None, :] - (qn * qn).sum(1, keepdim=True)
            else:
                s = qn @ Xf.T + self.bias[:n][None, :]
            return _stable_topk(s, k)
        # GPU: fused MFMA scan over bf16 rows, then exact fp32 re-rank
        kc = min(16, max(k, 4 * k)) if k <= 16 else k
        Qb = torch.zeros((nq, self.X.shape[1]), dtype=torch.bfloat16, device=self.device)
        if metric == "cosine":
            Qb[:, : self.dim] = qn.to(torch.bfloat16)
            inv = self.sqn[:n].sqrt().clamp_min(1e-30).reciprocal()
            # cosine = <q, x>/|x|: fold 1/|x| by scanning normalised rows would
            # need a second arena; approximate with ip + rerank below.
            bias = self.bias[:n]
            alpha = 1.0
        elif metric == "l2":
            Qb[:, : self.dim] = qn.to(torch.bfloat16)
            bias = (self.bias[:n] - self.sqn[:n]).contiguous()
            alpha = 2.0
        else:
            Qb[:, : self.dim] = qn.to(torch.bfloat16)
            bias = self.bias[:n]
            alpha = 1.0
        Xv = self.X[:n]
        if kc <= 16 and metric != "cosine":
            cs, cr = S.flat_topk(Xv, Qb, kc, bias=bias, alpha=alpha)
        else:
            # cosine on unnormalised rows / very large k: scale rows on the fly
            Xs = (self.X32[:n] if self.X32 is not None else Xv.float())
            if metric == "cosine":
                sc = (qn @ Xs.T) * inv[None, :] + self.bias[:n][None, :]
            else:
                sc = alpha * (qn @ Xs.T) + bias[None, :]
            return _stable_topk(sc, k)
        return self._rerank(qn, cs, cr, k, metric)

    def _rerank(self, qn, cs, cr, k, metric):
        if self.X32 is None:
            return cs[:, :k], cr[:, :k]
        valid = cr >= 0
        rows = cr.clamp_min(0)
        xs = self.X32[rows]  # [nq, kc, D]
        dot = torch.einsum("qd,qkd->qk", qn, xs)
        if metric == "l2":
            s = 2.0 * dot - self.sqn[rows] - (qn * qn).sum(1, keepdim=True)
        elif metric == "cosine":
            s = dot / self.sqn[rows].sqrt().clamp_min(1e-30)
        else:
            s = dot
        s = s + self.bias[rows]
        s = torch.where(valid, s, torch.full_like(s, NEG_INF))
        # order by (score desc, row asc)
        key_rows = torch.where(valid, cr, torch.full_like(cr, 1 << 62))
        o = torch.argsort(key_rows, dim=1, stable=True)
        s = torch.gather(s, 1, o)
        r = torch.gather(cr, 1, o)
        o = torch.argsort(-s, dim=1, stable=True)[:, :k]
        return torch.gather(s, 1, o), torch.gather(r, 1, o)

    def enable_ivf(self, nlist: int = 4096, m: int = 64, nprobe: int = 32, min_rows: int = 1_000_000,
                   candidates: int = 256) -> None:
        """Serve this arena's searches from an IVF-PQ index once it holds
        ``min_rows`` live rows (BASELINE config 5: tenants too large for an
        exhaustive scan per query). Candidates come from the PQ scan kernel,
        the final top-k is re-ranked EXACTLY on the arena's rows."""
        self.ivf = ArenaIVF(self, nlist, m, nprobe, min_rows, candidates)

    def _metric_scores(self, qn: torch.Tensor, rows: torch.Tensor, metric: str) -> torch.Tensor:
        """Exact scores of candidate ``rows`` [nq, c] (-1 = none) for queries qn."""
        valid = rows >= 0
        rr = rows.clamp_min(0)
        xs = self.X32[rr] if self.X32 is not None else self.X[rr, : self.dim].float()
        dot = torch.einsum("qd,qkd->qk", qn, xs)
        if metric == "l2":
            s = 2.0 * dot - self.sqn[rr] - (qn * qn).sum(1, keepdim=True)
        elif metric == "cosine":
            s = dot / self.sqn[rr].sqrt().clamp_min(1e-30)
        else:
            s = dot
        s = s + self.bias[rr]
        return torch.where(valid, s, torch.full_like(s, NEG_INF))

    def segment(self, metric: str = "l2"):
        """(rows, bias, scale) describing this arena for the multi-tenant
        segment kernel: exact fp32 rows when kept (no re-rank needed), the
        metric folded into a per-row bias / scale (cached per version)."""
        key = (metric, self.version, self.n)
        c = getattr(self, "_seg_cache", None)
        if c is not None and c[0] == key:
            return c[1]
        n = self.n
        if n == 0 or self.X is None:
            rows = torch.zeros((0, _pad64(self.dim or 64) if self.on_gpu else (self.dim or 1)),
                               dtype=self.store_dtype, device=self.device)
            out = (rows, None, None)
        else:
            use32 = self.X32 is not None and self.dim % 32 == 0
            rows = self.X32[:n] if use32 else self.X[:n]
            if metric == "l2":
                bias = (self.bias[:n] - self.sqn[:n]).contiguous()
            else:
                bias = self.bias[:n].contiguous()
            scale = self.sqn[:n].sqrt().clamp_min(1e-30).reciprocal().contiguous() if metric == "cosine" else None
            out = (rows, bias, scale)
        self._seg_cache = (key, out)
        return out

    def search(self, q, k: int, metric: str = "l2") -> List[List[str]]:
        s, r = self.search_rows(q, k, metric)
        r = r.cpu().tolist()
        s = s.cpu().tolist()
        out = []
        for rs, ss in zip(r, s):
            out.append([self.ids[x] for x, v in zip(rs, ss) if x >= 0 and v != NEG_INF and self.ids[x] is not None])
        return out

    def vectors(self, ids: Sequence[str]) -> torch.Tensor:
        """fp32 vectors of the first row of each id (device tensor)."""
        rows = [self.rows_of[i][0] for i in ids]
        t = torch.as_tensor(rows, dtype=torch.long, device=self.device)
        if self.X32 is not None:
            return self.X32[t]
        return self.X[t, : self.dim].float()


class ArenaIVF:
    """IVF-PQ acceleration attached to one :class:`VectorArena`.

    Row indices of the arena are the index ids, so the PQ candidates are
    re-ranked exactly against the arena's rows (fp32 copy when kept) with the
    arena's metric and tombstones. Appends are encoded incrementally; a clear
    or compaction (row indices change) triggers a rebuild on the next search.
    """

    def __init__(self, arena: VectorArena, nlist: int, m: int, nprobe: int, min_rows: int, candidates: int):
        self.arena, self.nlist, self.m, self.nprobe = arena, nlist, m, nprobe
        self.min_rows, self.candidates = min_rows, candidates
        self.idx = None
        self.epoch = -1
        self.covered = 0

    def _rows(self, r0: int, r1: int) -> torch.Tensor:
        a = self.arena
        return a.X32[r0:r1] if a.X32 is not None else a.X[r0:r1, : a.dim].float()

    def sync(self) -> None:
        from .ivfpq import IVFPQIndex
        a = self.arena
        if self.idx is None or self.epoch != a.layout_epoch or a.n < self.covered:
            m = self.m if a.dim % self.m == 0 else next(d for d in (64, 48, 32, 16, 8, 4, 2, 1) if a.dim % d == 0)
            nlist = max(16, min(self.nlist, len(a) // 64))
            self.idx = IVFPQIndex(a.dim, nlist=nlist, m=m, device=a.device)
            live = torch.nonzero(torch.isfinite(a.bias[: a.n])).flatten()
            g = torch.Generator(device="cpu").manual_seed(0)
            pick = live[torch.randperm(live.numel(), generator=g)[: min(live.numel(), 262144)].to(live.device)]
            self.idx.train(self._rows(0, a.n)[pick], iters=8, pq_iters=8)
            self.covered = 0
            self.epoch = a.layout_epoch
        step = 1 << 20
        while self.covered < a.n:
            r1 = min(a.n, self.covered + step)
            self.idx.add(self._rows(self.covered, r1), ids=torch.arange(self.covered, r1))
            self.covered = r1

    def search(self, qf: torch.Tensor, k: int, metric: str):
        self.sync()
        a = self.arena
        qn = qf / qf.norm(dim=1, keepdim=True).clamp_min(1e-30) if metric == "cosine" else qf
        kc = max(self.candidates, 4 * k)
        _, rows = self.idx.search(qf, kc, nprobe=self.nprobe)
        s = a._metric_scores(qn, rows.to(a.device), metric)
        vs, o = _stable_topk_rows(s, rows.to(a.device), k)
        return vs, o


def _stable_topk_rows(s: torch.Tensor, rows: torch.Tensor, k: int):
    """Top-k of candidate scores ordered (score desc, row asc)."""
    key = torch.where(rows >= 0, rows, torch.full_like(rows, 1 << 62))
    o = torch.argsort(key, dim=1, stable=True)
    s, rows = torch.gather(s, 1, o), torch.gather(rows, 1, o)
    vs, j = _stable_topk(s, k)
    r = torch.where(j >= 0, torch.gather(rows, 1, j.clamp_min(0)), j)
    return vs, r


def _stable_topk(s: torch.Tensor, k: int):
    n = s.shape[1]
    kk = min(k, n)
    o = torch.argsort(-s, dim=1, stable=True)[:, :kk]
    vs = torch.gather(s, 1, o)
    if kk < k:
        pad = k - kk
        vs = torch.cat([vs, torch.full((s.shape[0], pad), NEG_INF, device=s.device)], 1)
        o = torch.cat([o, torch.full((s.shape[0], pad), -1, dtype=torch.long, device=s.device)], 1)
    o = torch.where(torch.isneginf(vs), torch.full_like(o, -1), o)
    return vs, o
