"""IVF-PQ index (BASELINE config 5).

Memory: ``M`` bytes of PQ code + 20 bytes of list id / position / id per
vector, so one MI355X (288 GB HBM) holds ~3 billion 1024-d vectors at M=64
codes-only, ~200M with an fp8 re-rank copy -- vs 2 KB/vector for bf16 flat
storage. Inner-product metric on unit vectors (cosine).

* train: coarse k-means (``kmeans``: fused MFMA top-1 assign + segmented mean)
  and ``M`` residual sub-quantisers of 256 codewords each
* add:   coarse assign (fused top-1), residual PQ encode (batched GEMM +
         argmax per sub-space), then codes are kept sorted by list (CSR)
* search: coarse probe (top-nprobe centroids), per-query LUT
          ``<q_j, codebook_j[c]>`` (one batched GEMM), HIP ``ivfpq_scan``
          kernel per (query, probed list) with a fused top-k, shared
          ``topk_merge`` kernel; deep lists (re-rank depth > 16) from
          ``ivfpq_scan_deep`` (each wave's best rows per list); optional exact
          re-rank of the candidates against kept bf16/fp8 rows.
CPU tensors run a torch reference of the same pipeline (tests).
"""
from __future__ import annotations

from typing import Optional, Tuple

import numpy as np
import torch

from ..ops import _lib
from ..ops.search import _ws, flat_topk
from .kmeans import assign as coarse_assign
from .kmeans import kmeans

_lib.register("lzk_ivfpq_scan", _lib.I, [_lib.P, _lib.P, _lib.P, _lib.P, _lib.P, _lib.I, _lib.I, _lib.I, _lib.I,
                                          _lib.P, _lib.P, _lib.P])

_lib.register("lzk_ivfpq_scan_deep", _lib.I, [_lib.P, _lib.P, _lib.P, _lib.P, _lib.P, _lib.I, _lib.I, _lib.I,
                                               _lib.P, _lib.P, _lib.P])
_lib.register("lzk_ivfpq_deep_width", _lib.I, [])
_lib.register("lzk_ivfpq_scan_thresh", _lib.I, [_lib.P, _lib.P, _lib.P, _lib.P, _lib.P, _lib.P, _lib.I, _lib.I,
                                                _lib.I, _lib.I, _lib.P, _lib.P, _lib.P, _lib.P])

_lib.register("lzk_rerank", _lib.I, [_lib.P, _lib.L, _lib.I, _lib.P, _lib.P, _lib.I, _lib.I, _lib.P, _lib.I,
                                      _lib.I, _lib.I, _lib.P, _lib.P, _lib.P])

KSLOTS = (1, 4, 10, 16)


def _kslot(k: int) -> int:
    for s in KSLOTS:
        if k <= s:
            return s
    raise ValueError("k <= 16 per IVF-PQ pass")


def _unit(x):
    return x / x.norm(dim=1, keepdim=True).clamp_min(1e-30)


class IVFPQIndex:
    def __init__(self, dim: int, nlist: int = 1024, m: int = 64, device=None, keep_vectors=False):
        """keep_vectors: False (codes only, m+20 bytes/vector), True / "bf16"
        (exact re-rank copy, 2*Dp bytes/vector), "int8" or "fp8" (re-rank
        copy with a per-row scale, D+4 bytes/vector -- the layout that fills
        288 GB with ~200M 1024-d vectors and still re-ranks PQ candidates;
        int8's uniform grid is ~3x finer than e4m3 on embedding rows, so it
        is the one to use for recall).

        Storage is preallocated (:meth:`reserve`) and written in place. Code
        rows (``codes``, ``list_of``) are kept sorted by list (CSR) and carry
        ``pos`` = the insertion row of each; the re-rank copy and the ids stay
        in insertion order, so sorting never moves the big vector copy."""
        assert dim % m == 0, "dim must be divisible by m"
        self.dim, self.nlist, self.m, self.dsub = dim, nlist, m, dim // m
        self.device = torch.device(device) if device is not None else torch.device("cpu")
        self.Dp = (dim + 63) // 64 * 64
        self.centroids = None      # fp32 [nlist, dim]
        self.centroids16 = None    # bf16 [nlist, Dp] (GPU assign)
        self.codebooks = None      # fp32 [m, 256, dsub]
        self.keep_vectors = "bf16" if keep_vectors is True else (keep_vectors or False)
        if self.keep_vectors not in (False, "bf16", "fp8", "int8"):
            raise ValueError("keep_vectors must be False, True/'bf16', 'int8' or 'fp8'")
        self.n = 0
        self.cap = 0
        z = lambda *s, dt: torch.zeros(s, dtype=dt, device=self.device)  # noqa: E731
        self._codes = z(0, m, dt=torch.uint8)
        self._list = z(0, dt=torch.int32)
        self._pos = z(0, dt=torch.int64)
        self._vids = z(0, dt=torch.int64)
        self._vec = None
        self._vscale = None
        self.list_off = z(nlist + 1, dt=torch.int64)
        self._dirty = False

    # ------------------------------------------------------------------ storage
    def reserve(self, n: int) -> None:
        """Capacity for ``n`` vectors (grows by copying; call once up front to
        build a large index without reallocations)."""
        if n <= self.cap:
            return
        cap = max(n, int(self.cap * 1.5) + 1)
        k = self.n

        def grow(t, shape, dt):
            new = torch.zeros(shape, dtype=dt, device=self.device)
            if t is not None and k:
                new[:k] = t[:k]
            return new
        self._codes = grow(self._codes, (cap, self.m), torch.uint8)
        self._list = grow(self._list, (cap,), torch.int32)
        self._pos = grow(self._pos, (cap,), torch.int64)
        self._vids = grow(self._vids, (cap,), torch.int64)
        if self.keep_vectors == "bf16":
            w = self.Dp if self.device.type == "cuda" else self.dim
            self._vec = grow(self._vec, (cap, w), torch.bfloat16 if self.device.type == "cuda" else torch.float32)
        elif self.keep_vectors in ("fp8", "int8"):
            self._vec = grow(self._vec, (cap, self.dim), torch.uint8)
            self._vscale = grow(self._vscale, (cap,), torch.float32)
        self.cap = cap

    # views of the live rows (code order) -- and setters for hand-built indexes
    @property
    def codes(self) -> torch.Tensor:
        return self._codes[: self.n]

    @codes.setter
    def codes(self, v: torch.Tensor) -> None:
        self._codes, self.n, self.cap = v.to(self.device), v.shape[0], v.shape[0]
        self._pos = torch.arange(self.n, device=self.device)

    @property
    def list_of(self) -> torch.Tensor:
        return self._list[: self.n]

    @list_of.setter
    def list_of(self, v: torch.Tensor) -> None:
        self._list = v.to(self.device, torch.int32)

    @property
    def ids(self) -> torch.Tensor:
        """ids in code order."""
        return self._vids[self._pos[: self.n]]

    @ids.setter
    def ids(self, v: torch.Tensor) -> None:
        self._vids = v.to(self.device, torch.int64)
        self._pos = torch.arange(v.shape[0], device=self.device)

    @property
    def vectors(self):
        return None if self._vec is None else self._vec[: self.n]

    @property
    def vscale(self):
        return None if self._vscale is None else self._vscale[: self.n]

    # ------------------------------------------------------------------ train
    def _pad(self, x: torch.Tensor) -> torch.Tensor:
        if self.device.type != "cuda":
            return x.float()
        out = torch.zeros((x.shape[0], self.Dp), dtype=torch.bfloat16, device=self.device)
        out[:, : self.dim] = x.to(torch.bfloat16)
        return out

    def train(self, x: torch.Tensor, iters: int = 10, pq_iters: int = 12, seed: int = 0) -> None:
        x = _unit(x.to(self.device).float())
        c32, _, lab = kmeans(self._pad(x), self.nlist, iters=iters, seed=seed)
        self.centroids = c32[:, : self.dim].contiguous()
        self.centroids16 = self._pad(self.centroids)
        res = x - self.centroids[lab.long()]
        self.codebooks = self._train_pq(res, pq_iters, seed)

    def _train_pq(self, res: torch.Tensor, iters: int, seed: int) -> torch.Tensor:
        n = res.shape[0]
        g = torch.Generator(device="cpu").manual_seed(seed + 1)
        sub = res.view(n, self.m, self.dsub).transpose(0, 1).contiguous()  # [m, n, dsub]
        init = torch.randperm(n, generator=g)[:256].to(res.device)
        cb = sub[:, init].clone()  # [m, 256, dsub]
        for _ in range(iters):
            code = self._encode_sub(sub, cb)  # [m, n]
            sums = torch.zeros_like(cb).scatter_add_(1, code[..., None].expand(-1, -1, self.dsub).long(), sub)
            cnt = torch.zeros((self.m, 256), device=res.device).scatter_add_(
                1, code.long(), torch.ones_like(code, dtype=torch.float32))
            upd = sums / cnt.clamp_min(1)[..., None]
            cb = torch.where((cnt > 0)[..., None], upd, cb)
        return cb

    @staticmethod
    def _encode_sub(sub: torch.Tensor, cb: torch.Tensor, chunk: int = 16384) -> torch.Tensor:
        # argmin ||r - c||^2 = argmax (2 r.c - |c|^2), batched over sub-spaces,
        # chunked over rows so the [m, rows, 256] score block stays ~1 GB
        cn = (cb * cb).sum(-1)[:, None, :]
        out = torch.empty(sub.shape[:2], dtype=torch.uint8, device=sub.device)
        for r0 in range(0, sub.shape[1], chunk):
            score = 2.0 * torch.bmm(sub[:, r0:r0 + chunk], cb.transpose(1, 2)) - cn
            out[:, r0:r0 + chunk] = score.argmax(-1).to(torch.uint8)
        return out

    # ------------------------------------------------------------------ add
    def encode(self, x: torch.Tensor) -> Tuple[torch.Tensor, torch.Tensor]:
        x = _unit(x.to(self.device).float())
        if self.device.type == "cuda":
            lab, _ = coarse_assign(self._pad(x), self.centroids16)
        else:
            lab = (x @ self.centroids.T).argmax(1).to(torch.int32)
        res = x - self.centroids[lab.long()]
        sub = res.view(-1, self.m, self.dsub).transpose(0, 1).contiguous()
        codes = self._encode_sub(sub, self.codebooks).T.contiguous()  # [n, m]
        return lab, codes

    def add(self, x: torch.Tensor, ids: Optional[torch.Tensor] = None, batch: int = 1 << 18) -> None:
        n0 = self.n
        n = x.shape[0]
        self.reserve(n0 + n)
        ids = torch.arange(n0, n0 + n, dtype=torch.int64) if ids is None else ids.to(torch.int64)
        self._vids[n0:n0 + n] = ids.to(self.device)
        self._pos[n0:n0 + n] = torch.arange(n0, n0 + n, device=self.device)
        for r0 in range(0, n, batch):
            r1 = min(n, r0 + batch)
            xb = _unit(x[r0:r1].to(self.device).float())
            lab, codes = self.encode(xb)
            self._list[n0 + r0:n0 + r1] = lab
            self._codes[n0 + r0:n0 + r1] = codes
            if self.keep_vectors == "bf16":
                self._vec[n0 + r0:n0 + r1] = self._pad(xb) if self.device.type == "cuda" else xb
            elif self.keep_vectors == "fp8":
                from ..ops.encoder_ops import quantize_fp8_rows
                v = xb.to(torch.bfloat16) if self.device.type == "cuda" else xb
                q8, sc = quantize_fp8_rows(v.contiguous())
                self._vec[n0 + r0:n0 + r1] = q8
                self._vscale[n0 + r0:n0 + r1] = sc
            elif self.keep_vectors == "int8":
                sc = xb.abs().amax(1).clamp_min(1e-30) / 127.0
                q = torch.round(xb / sc[:, None]).clamp_(-127, 127).to(torch.int8)
                self._vec[n0 + r0:n0 + r1] = q.view(torch.uint8)
                self._vscale[n0 + r0:n0 + r1] = sc
        self.n = n0 + n
        self._dirty = True

    def _finalize(self, chunk: int = 1 << 24) -> None:
        """Sort the code rows by list id (CSR) -- amortised over a batch of
        adds; the codes are permuted in chunks into one new buffer, the
        vectors never move (``pos`` follows the codes)."""
        if not self._dirty:
            return
        n = self.n
        o = torch.argsort(self._list[:n], stable=True)
        codes = torch.empty_like(self._codes)
        for c0 in range(0, n, chunk):
            c1 = min(n, c0 + chunk)
            codes[c0:c1] = self._codes[o[c0:c1]]
        self._codes = codes
        self._list[:n] = self._list[:n][o]
        self._pos[:n] = self._pos[:n][o]
        cnt = torch.bincount(self._list[:n].long(), minlength=self.nlist)
        self.list_off = torch.zeros(self.nlist + 1, dtype=torch.int64, device=self.device)
        self.list_off[1:] = torch.cumsum(cnt, 0)
        self._dirty = False

    def __len__(self) -> int:
        return int(self.n)

    def memory_bytes(self) -> int:
        b = self.n * (self.m + 4 + 8 + 8)  # codes, list id, pos, id
        if self._vec is not None:
            b += self.n * self._vec.shape[1] * self._vec.element_size()
        return b + (self.n * 4 if self._vscale is not None else 0)

    # ------------------------------------------------------------------ search
    def search(self, q: torch.Tensor, k: int = 10, nprobe: int = 16, rerank: int = 0):
        """Returns (scores fp32 [nq, k], ids int64 [nq, k]). ``rerank`` > 0:
        the best ``rerank`` PQ candidates are re-scored exactly against the
        kept copy (scores then are exact inner products)."""
        self._finalize()
        qf = _unit(q.to(self.device).float())
        nq = qf.shape[0]
        nprobe = min(nprobe, self.nlist)
        cs = qf @ self.centroids.T
        coarse, probes = torch.topk(cs, nprobe, dim=1)
        lut = torch.einsum("qmd,mcd->qmc", qf.view(nq, self.m, self.dsub), self.codebooks).contiguous()
        kk = max(k, rerank) if rerank else k
        if self.device.type != "cuda":
            s, rows = self._scan_ref(probes, coarse, lut, kk)
        elif rerank and self._vec is not None and kk > KSLOTS[-1]:
            s, rows = self._scan_candidates(probes.to(torch.int32).contiguous(), coarse.contiguous(), lut, kk)
        elif kk <= KSLOTS[-1]:
            s, rows = self._scan_gpu(probes.to(torch.int32).contiguous(), coarse.contiguous(), lut, kk)
        else:
            s, rows = self._scan_deep(probes.to(torch.int32).contiguous(), coarse.contiguous(), lut, kk)
        if rerank and self._vec is not None:
            vrows = torch.where(rows >= 0, self._pos[rows.clamp_min(0)], torch.full_like(rows, -1))
            if self._rerank_gpu_ok(k):
                s, vr = self._rerank_gpu(qf, vrows.contiguous(), k)
            else:
                valid = vrows >= 0
                vv = vrows.clamp_min(0)
                if self._vscale is not None:  # fp8 / int8 copy: dequantise the gathered candidates only
                    dt = torch.int8 if self.keep_vectors == "int8" else torch.float8_e4m3fn
                    v = self._vec[vv].view(dt).float() * self._vscale[vv][..., None]
                else:
                    v = self._vec[vv].float()[..., : self.dim]
                sc = torch.einsum("qd,qkd->qk", qf, v)
                sc = torch.where(valid, sc, torch.full_like(sc, float("-inf")))
                s, o = torch.sort(sc, dim=1, descending=True, stable=True)
                vr = torch.gather(vrows, 1, o)
            s, vr = s[:, :k], vr[:, :k]
            return s, torch.where(vr >= 0, self._vids[vr.clamp_min(0)], torch.full_like(vr, -1))
        s, rows = s[:, :k], rows[:, :k]
        ids = torch.where(rows >= 0, self._vids[self._pos[rows.clamp_min(0)]], torch.full_like(rows, -1))
        return s, ids

    def candidate_ids(self, q: torch.Tensor, R: int, nprobe: int = 16) -> torch.Tensor:
        """The ids of the exact PQ top-``R`` rows over the ``nprobe`` probed
        lists per query ([nq, R] int64, -1 padded) -- for a caller that
        re-ranks with its own exact vectors (TenantGraph's fp32 rows)."""
        self._finalize()
        qf = _unit(q.to(self.device).float())
        nq = qf.shape[0]
        nprobe = min(nprobe, self.nlist)
        coarse, probes = torch.topk(qf @ self.centroids.T, nprobe, dim=1)
        lut = torch.einsum("qmd,mcd->qmc", qf.view(nq, self.m, self.dsub), self.codebooks).contiguous()
        if self.device.type != "cuda":
            _, rows = self._scan_ref(probes, coarse, lut, R)
        elif R <= KSLOTS[-1]:
            _, rows = self._scan_gpu(probes.to(torch.int32).contiguous(), coarse.contiguous(), lut, R)
        else:
            _, rows = self._scan_candidates(probes.to(torch.int32).contiguous(), coarse.contiguous(), lut, R)
        rows = rows.long()
        return torch.where(rows >= 0, self._vids[self._pos[rows.clamp_min(0)]], torch.full_like(rows, -1))

    def _rerank_gpu_ok(self, k: int) -> bool:
        if self.device.type != "cuda" or k > KSLOTS[-1]:
            return False
        w = self._vec.shape[1]
        row_bytes = w if self._vscale is not None else 2 * w
        return row_bytes % 256 == 0

    def _rerank_gpu(self, qf: torch.Tensor, rows: torch.Tensor, k: int):
        """Fused exact re-rank over the kept copy (csrc/kernels/ivfpq.hip
        rerank_kernel): no dequantised [nq, R, D] intermediate. ``rows`` are
        vector (insertion) rows; returns (scores, vector rows)."""
        nq, R = rows.shape
        fmt = {"fp8": 1, "int8": 2}.get(self.keep_vectors, 0)
        w = self._vec.shape[1]
        Q = torch.zeros((nq, w), dtype=torch.float32, device=self.device)
        Q[:, : qf.shape[1]] = qf
        ks = _kslot(k)
        os_ = torch.empty((nq, k), dtype=torch.float32, device=self.device)
        oi = torch.empty((nq, k), dtype=torch.long, device=self.device)
        ldv = self._vec.stride(0) * self._vec.element_size()
        _lib.check(_lib.lib().lzk_rerank(self._vec.data_ptr(), ldv, fmt, _lib.ptr(self._vscale),
                                         rows.data_ptr(), nq, R, Q.data_ptr(), w, ks, k, os_.data_ptr(),
                                         oi.data_ptr(), _lib.stream_ptr(self.device)), "lzk_rerank")
        return os_, oi

    def _scan_ref(self, probes, coarse, lut, k):
        nq = probes.shape[0]
        out_s = torch.full((nq, k), float("-inf"), device=self.device)
        out_r = torch.full((nq, k), -1, dtype=torch.long, device=self.device)
        ar = torch.arange(self.m, device=self.device)
        codes = self.codes
        for qi in range(nq):
            cand_s, cand_r = [], []
            for p in range(probes.shape[1]):
                l = int(probes[qi, p])
                r0, r1 = int(self.list_off[l]), int(self.list_off[l + 1])
                if r1 == r0:
                    continue
                c = codes[r0:r1].long()
                cand_s.append(coarse[qi, p] + lut[qi][ar[None, :], c].sum(1))
                cand_r.append(torch.arange(r0, r1, device=self.device))
            if not cand_s:
                continue
            cs_, cr_ = torch.cat(cand_s), torch.cat(cand_r)
            o = torch.argsort(-cs_, stable=True)[:k]
            out_s[qi, : o.numel()] = cs_[o]
            out_r[qi, : o.numel()] = cr_[o]
        return out_s, out_r

    def _scan_deep(self, probes, coarse, lut, k):
        """Deep candidate lists (re-rank depth >> 16): each (query, probed
        list) block emits its waves' best rows (``ivfpq_scan_deep_kernel``,
        4 x 128 per list), then a top-k over the query's nprobe x 512 PQ scores."""
        nq, nprobe = probes.shape
        L = _lib.lib()
        W = L.lzk_ivfpq_deep_width()
        os_ = torch.empty((nq, nprobe * W), dtype=torch.float32, device=self.device)
        oi = torch.empty((nq, nprobe * W), dtype=torch.int32, device=self.device)
        _lib.check(L.lzk_ivfpq_scan_deep(self._codes.data_ptr(), self.list_off.data_ptr(), probes.data_ptr(),
                                         coarse.data_ptr(), lut.data_ptr(), nq, nprobe, self.m, os_.data_ptr(),
                                         oi.data_ptr(), _lib.stream_ptr(self.device)), "lzk_ivfpq_scan_deep")
        kk = min(k, os_.shape[1])
        s, j = torch.topk(os_, kk, dim=1)
        rows = torch.gather(oi, 1, j).long()
        rows = torch.where(torch.isneginf(s), torch.full_like(rows, -1), rows)
        if kk < k:
            s = torch.cat([s, torch.full((nq, k - kk), float("-inf"), device=self.device)], 1)
            rows = torch.cat([rows, torch.full((nq, k - kk), -1, dtype=torch.long, device=self.device)], 1)
        return s, rows

    # threshold-pass buffer: CAND_CAP x the requested depth (at least
    # CAND_MIN): with weak PQ codes a crowded list makes the pooled threshold
    # loose, and everything above it must fit before the PQ top-R is taken
    CAND_CAP = 16
    CAND_MIN = 32768

    def _scan_candidates(self, probes, coarse, lut, R):
        """Re-rank candidates: the exact PQ top-R over the probed lists (plus
        ties). Pass 1 (``ivfpq_scan_deep``) pools each list's best rows; the
        R-th best pooled score is a lower bound of the true R-th best; pass 2
        (``ivfpq_scan_thresh``) appends EVERY probed row at or above it, so a
        query whose neighbours crowd into one list still gets all of them.
        Returns (PQ scores, code rows) [nq, R] of the collected rows' PQ
        top-R, -1 padded."""
        nq, nprobe = probes.shape
        ps, _ = self._scan_deep(probes, coarse, lut, R)
        thr = ps[:, R - 1].contiguous()  # -inf when the pools hold fewer than R rows: take everything
        cap = max(self.CAND_CAP * R, self.CAND_MIN)
        L = _lib.lib()
        cnt = torch.zeros(nq, dtype=torch.int32, device=self.device)
        os_ = torch.empty((nq, cap), dtype=torch.float32, device=self.device)
        oi = torch.empty((nq, cap), dtype=torch.int32, device=self.device)
        _lib.check(L.lzk_ivfpq_scan_thresh(self._codes.data_ptr(), self.list_off.data_ptr(), probes.data_ptr(),
                                           coarse.data_ptr(), lut.data_ptr(), thr.data_ptr(), nq, nprobe, self.m,
                                           cap, cnt.data_ptr(), os_.data_ptr(), oi.data_ptr(),
                                           _lib.stream_ptr(self.device)), "lzk_ivfpq_scan_thresh")
        self.last_candidates = cnt  # per-query count (> cap: overflowed, kept the first cap)
        valid = torch.arange(cap, device=self.device)[None, :] < cnt.clamp(max=cap)[:, None]
        sc = torch.where(valid, os_, torch.full_like(os_, float("-inf")))
        ts, j = torch.topk(sc, min(R, cap), dim=1)
        rows = torch.gather(oi, 1, j).long()
        return ts, torch.where(torch.isneginf(ts), torch.full_like(rows, -1), rows)

    def _scan_gpu(self, probes, coarse, lut, k):
        nq, nprobe = probes.shape
        ks = _kslot(k)
        part = nq * nprobe * ks
        ws = _ws.get(self.device, part * 8)
        ps = ws[: part * 4].view(torch.float32)
        pi = ws[part * 4: part * 8].view(torch.int32)
        st = _lib.stream_ptr(self.device)
        L = _lib.lib()
        _lib.check(L.lzk_ivfpq_scan(self._codes.data_ptr(), self.list_off.data_ptr(), probes.data_ptr(),
                                    coarse.data_ptr(), lut.data_ptr(), nq, nprobe, self.m, ks, ps.data_ptr(),
                                    pi.data_ptr(), st), "lzk_ivfpq_scan")
        os_ = torch.empty((nq, k), dtype=torch.float32, device=self.device)
        oi = torch.empty((nq, k), dtype=torch.long, device=self.device)
        _lib.check(L.lzk_topk_merge(ps.data_ptr(), pi.data_ptr(), nprobe * ks, nq, ks, k, 0, os_.data_ptr(),
                                    oi.data_ptr(), st), "lzk_topk_merge")
        return os_, oi


def recall_at_k(found: torch.Tensor, truth: torch.Tensor) -> float:
    f, t = found.cpu().numpy(), truth.cpu().numpy()
    k = t.shape[1]
    return float(np.mean([len(set(a) & set(b)) / k for a, b in zip(f, t)]))
