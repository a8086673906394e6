"""IVF-PQ index (BASELINE config 5).

Memory: ``M`` bytes of PQ code + 8 bytes of id per vector, so one MI355X
(288 GB HBM) holds ~3.5 billion 1024-d vectors at M=64 -- vs 2 KB/vector for
bf16 flat storage. Inner-product metric on unit vectors (cosine).

* train: coarse k-means (``kmeans``: fused MFMA top-1 assign + segmented mean)
  and ``M`` residual sub-quantisers of 256 codewords each
* add:   coarse assign (fused top-1), residual PQ encode (batched GEMM +
         argmax per sub-space), then codes are kept sorted by list (CSR)
* search: coarse probe (top-nprobe centroids), per-query LUT
          ``<q_j, codebook_j[c]>`` (one batched GEMM), HIP ``ivfpq_scan``
          kernel per (query, probed list) with a fused top-k, shared
          ``topk_merge`` kernel; optional exact re-rank of the candidates
          against kept bf16/fp8 rows.
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

_lib.register("lzk_ivfpq_dense", _lib.I, [_lib.P, _lib.P, _lib.P, _lib.P, _lib.P, _lib.I, _lib.I, _lib.I,
                                           _lib.I, _lib.P, _lib.P])

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
        """keep_vectors: False (codes only, 8+m bytes/vector), True / "bf16"
        (exact re-rank copy, 2*Dp bytes/vector) or "fp8" (OCP e4m3 re-rank copy
        with a per-row scale, D+4 bytes/vector -- the layout that fills 288 GB
        with ~250M 1024-d vectors and still re-ranks PQ candidates)."""
        assert dim % m == 0, "dim must be divisible by m"
        self.dim, self.nlist, self.m, self.dsub = dim, nlist, m, dim // m
        self.device = torch.device(device) if device is not None else torch.device("cpu")
        self.Dp = (dim + 63) // 64 * 64
        self.centroids = None      # fp32 [nlist, dim]
        self.centroids16 = None    # bf16 [nlist, Dp] (GPU assign)
        self.codebooks = None      # fp32 [m, 256, dsub]
        self.codes = torch.zeros((0, m), dtype=torch.uint8, device=self.device)
        self.ids = torch.zeros(0, dtype=torch.int64, device=self.device)
        self.list_of = torch.zeros(0, dtype=torch.int32, device=self.device)
        self.list_off = torch.zeros(nlist + 1, dtype=torch.int64, device=self.device)
        self.keep_vectors = "bf16" if keep_vectors is True else (keep_vectors or False)
        if self.keep_vectors not in (False, "bf16", "fp8"):
            raise ValueError("keep_vectors must be False, True/'bf16' or 'fp8'")
        self.vectors = None
        self.vscale = None
        self._dirty = False

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
        n0 = self.ids.numel()
        n = x.shape[0]
        ids = torch.arange(n0, n0 + n, dtype=torch.int64) if ids is None else ids.to(torch.int64)
        labs, codes = [], []
        for r0 in range(0, n, batch):
            l, c = self.encode(x[r0:r0 + batch])
            labs.append(l)
            codes.append(c)
        lab = torch.cat(labs)
        self.codes = torch.cat([self.codes, torch.cat(codes)])
        self.ids = torch.cat([self.ids, ids.to(self.device)])
        self.list_of = torch.cat([self.list_of, lab])
        if self.keep_vectors == "bf16":
            v = self._pad(_unit(x.to(self.device).float()))
            self.vectors = v if self.vectors is None else torch.cat([self.vectors, v])
        elif self.keep_vectors == "fp8":
            from ..ops.encoder_ops import quantize_fp8_rows
            qs, ss = [], []
            for r0 in range(0, n, batch):
                v = _unit(x[r0:r0 + batch].to(self.device).float())
                v = v.to(torch.bfloat16) if self.device.type == "cuda" else v
                q8, sc = quantize_fp8_rows(v.contiguous())
                qs.append(q8)
                ss.append(sc)
            q8, sc = torch.cat(qs), torch.cat(ss)
            self.vectors = q8 if self.vectors is None else torch.cat([self.vectors, q8])
            self.vscale = sc if self.vscale is None else torch.cat([self.vscale, sc])
        self._dirty = True

    def _finalize(self) -> None:
        """Sort rows by list id (CSR) -- amortised over a batch of adds."""
        if not self._dirty:
            return
        o = torch.argsort(self.list_of, stable=True)
        self.codes = self.codes[o].contiguous()
        self.ids = self.ids[o]
        self.list_of = self.list_of[o]
        if self.vectors is not None:
            self.vectors = self.vectors[o]
        if self.vscale is not None:
            self.vscale = self.vscale[o]
        cnt = torch.bincount(self.list_of.long(), minlength=self.nlist)
        self.list_off = torch.zeros(self.nlist + 1, dtype=torch.int64, device=self.device)
        self.list_off[1:] = torch.cumsum(cnt, 0)
        self._dirty = False

    def __len__(self) -> int:
        return int(self.ids.numel())

    def memory_bytes(self) -> int:
        b = self.codes.numel() + self.ids.numel() * 8
        b += self.vectors.numel() * self.vectors.element_size() if self.vectors is not None else 0
        return b + (self.vscale.numel() * 4 if self.vscale is not None else 0)

    # ------------------------------------------------------------------ search
    def search(self, q: torch.Tensor, k: int = 10, nprobe: int = 16, rerank: int = 0):
        """Returns (scores fp32 [nq, k], ids int64 [nq, k])."""
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
        elif kk <= KSLOTS[-1]:
            s, rows = self._scan_gpu(probes.to(torch.int32).contiguous(), coarse.contiguous(), lut, kk)
        else:
            s, rows = self._scan_dense(probes.to(torch.int32).contiguous(), coarse.contiguous(), lut, kk)
        if rerank and self.vectors is not None and self._rerank_gpu_ok(k):
            s, rows = self._rerank_gpu(qf, rows.contiguous(), k)
        elif rerank and self.vectors is not None:
            valid = rows >= 0
            rr = rows.clamp_min(0)
            if self.vscale is not None:  # fp8 copy: dequantise the gathered candidates only
                v = self.vectors[rr].view(torch.float8_e4m3fn).float() * self.vscale[rr][..., None]
            else:
                v = self.vectors[rr].float()[..., : self.dim]
            s = torch.einsum("qd,qkd->qk", qf, v)
            s = torch.where(valid, s, torch.full_like(s, float("-inf")))
            s, o = torch.sort(s, dim=1, descending=True, stable=True)
            rows = torch.gather(rows, 1, o)
        s, rows = s[:, :k], rows[:, :k]
        ids = torch.where(rows >= 0, self.ids[rows.clamp_min(0)], torch.full_like(rows, -1))
        return s, ids

    def _rerank_gpu_ok(self, k: int) -> bool:
        if self.device.type != "cuda" or k > KSLOTS[-1]:
            return False
        w = self.vectors.shape[1]
        row_bytes = w if self.vscale is not None else 2 * w
        return row_bytes % 256 == 0

    def _rerank_gpu(self, qf: torch.Tensor, rows: torch.Tensor, k: int):
        """Fused exact re-rank over the kept copy (csrc/kernels/ivfpq.hip
        rerank_kernel): no dequantised [nq, R, D] intermediate."""
        nq, R = rows.shape
        fp8 = self.vscale is not None
        w = self.vectors.shape[1]
        Q = torch.zeros((nq, w), dtype=torch.float32, device=self.device)
        Q[:, : qf.shape[1]] = qf
        ks = _kslot(k)
        os_ = torch.empty((nq, k), dtype=torch.float32, device=self.device)
        oi = torch.empty((nq, k), dtype=torch.long, device=self.device)
        ldv = self.vectors.stride(0) * self.vectors.element_size()
        _lib.check(_lib.lib().lzk_rerank(self.vectors.data_ptr(), ldv, int(fp8), _lib.ptr(self.vscale),
                                         rows.data_ptr(), nq, R, Q.data_ptr(), w, ks, k, os_.data_ptr(),
                                         oi.data_ptr(), _lib.stream_ptr(self.device)), "lzk_rerank")
        return os_, oi

    def _scan_ref(self, probes, coarse, lut, k):
        nq = probes.shape[0]
        out_s = torch.full((nq, k), float("-inf"), device=self.device)
        out_r = torch.full((nq, k), -1, dtype=torch.long, device=self.device)
        ar = torch.arange(self.m, device=self.device)
        for qi in range(nq):
            cand_s, cand_r = [], []
            for p in range(probes.shape[1]):
                l = int(probes[qi, p])
                r0, r1 = int(self.list_off[l]), int(self.list_off[l + 1])
                if r1 == r0:
                    continue
                c = self.codes[r0:r1].long()
                cand_s.append(coarse[qi, p] + lut[qi][ar[None, :], c].sum(1))
                cand_r.append(torch.arange(r0, r1, device=self.device))
            if not cand_s:
                continue
            cs_, cr_ = torch.cat(cand_s), torch.cat(cand_r)
            o = torch.argsort(-cs_, stable=True)[:k]
            out_s[qi, : o.numel()] = cs_[o]
            out_r[qi, : o.numel()] = cr_[o]
        return out_s, out_r

    def _scan_dense(self, probes, coarse, lut, k):
        """Deep candidate lists: dense PQ scores per probed list (HIP kernel),
        then a library top-k over each query's [nprobe * maxlen] scores."""
        nq, nprobe = probes.shape
        lens = (self.list_off[1:] - self.list_off[:-1])
        maxlen = int(lens[probes.long()].max().item()) if probes.numel() else 0
        maxlen = max(maxlen, 1)
        buf = torch.empty((nq, nprobe, maxlen), dtype=torch.float32, device=self.device)
        _lib.check(_lib.lib().lzk_ivfpq_dense(self.codes.data_ptr(), self.list_off.data_ptr(), probes.data_ptr(),
                                              coarse.data_ptr(), lut.data_ptr(), nq, nprobe, self.m, maxlen,
                                              buf.data_ptr(), _lib.stream_ptr(self.device)), "lzk_ivfpq_dense")
        flat = buf.view(nq, -1)
        kk = min(k, flat.shape[1])
        s, pos = torch.topk(flat, kk, dim=1)
        p, off = pos // maxlen, pos % maxlen
        lists = torch.gather(probes.long(), 1, p)
        rows = self.list_off[lists] + off
        rows = torch.where(torch.isneginf(s), torch.full_like(rows, -1), rows)
        return s, rows

    def _scan_gpu(self, probes, coarse, lut, k):
        nq, nprobe = probes.shape
        ks = _kslot(k)
        part = nq * nprobe * ks
        ws = _ws.get(self.device, part * 8)
        ps = ws[: part * 4].view(torch.float32)
        pi = ws[part * 4: part * 8].view(torch.int32)
        st = _lib.stream_ptr(self.device)
        L = _lib.lib()
        _lib.check(L.lzk_ivfpq_scan(self.codes.data_ptr(), self.list_off.data_ptr(), probes.data_ptr(),
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
