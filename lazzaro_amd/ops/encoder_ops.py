"""Encoder ops: GEMM with fused bias/GELU/residual
epilogue, flash-style attention, LayerNorm, embedding+LayerNorm, pooling+L2.

HIP tensors -> hand-written gfx950 kernels (``csrc/kernels/encoder.hip``);
CPU tensors -> the fp32 torch reference of the same op (used as the CPU test
tier and as the numerics oracle in tests/kernels).
Activations are bf16 row-major ``[tokens, features]``; weights ``[out, in]``.
"""
from __future__ import annotations

import math

import torch
import torch.nn.functional as F

from . import _lib

_lib.register("lzk_gemm_bias_act", _lib.I, [_lib.P, _lib.L, _lib.I, _lib.P, _lib.L, _lib.I, _lib.P, _lib.P,
                                             _lib.L, _lib.P, _lib.L, _lib.I, _lib.I, _lib.P])
_lib.register("lzk_gemm_split2", _lib.I, [_lib.P, _lib.L, _lib.I, _lib.P, _lib.L, _lib.I, _lib.P, _lib.P, _lib.L,
                                           _lib.P, _lib.P, _lib.L, _lib.I, _lib.P])
_lib.register("lzk_gemm_f8", _lib.I, [_lib.P, _lib.L, _lib.I, _lib.P, _lib.P, _lib.L, _lib.I, _lib.P, _lib.P,
                                       _lib.P, _lib.L, _lib.P, _lib.L, _lib.I, _lib.I, _lib.P])
_lib.register("lzk_quant_fp8_rows", _lib.I, [_lib.P, _lib.L, _lib.I, _lib.I, _lib.P, _lib.L, _lib.P, _lib.P])
_lib.register("lzk_layernorm_q8", _lib.I, [_lib.P, _lib.L, _lib.P, _lib.L, _lib.P, _lib.P, _lib.I, _lib.I, _lib.F,
                                           _lib.P, _lib.L, _lib.P, _lib.L, _lib.P, _lib.P])
_lib.register("lzk_attention", _lib.I, [_lib.P, _lib.L, _lib.P, _lib.I, _lib.I, _lib.I, _lib.I, _lib.F,
                                         _lib.P, _lib.L, _lib.P, _lib.P])
_lib.register("lzk_layernorm", _lib.I, [_lib.P, _lib.L, _lib.P, _lib.L, _lib.P, _lib.P, _lib.I, _lib.I,
                                         _lib.F, _lib.P, _lib.L, _lib.P])
_lib.register("lzk_embed_ln", _lib.I, [_lib.P, _lib.I, _lib.I, _lib.P, _lib.P, _lib.P, _lib.P, _lib.P,
                                        _lib.I, _lib.F, _lib.P, _lib.P, _lib.P])
_lib.register("lzk_pool_norm", _lib.I, [_lib.P, _lib.P, _lib.I, _lib.I, _lib.I, _lib.I, _lib.P, _lib.P,
                                         _lib.I, _lib.P, _lib.P])


def linear(x: torch.Tensor, w: torch.Tensor, b: torch.Tensor, act: str = "none", residual=None,
           out=None) -> torch.Tensor:
    """act(x @ w.T + b) (+ residual). x [T,K] bf16, w [N,K] bf16, b [N] fp32."""
    T, K = x.shape
    N = w.shape[0]
    if not x.is_cuda:
        y = x.float() @ w.float().T + b.float()
        if act == "gelu":
            y = F.gelu(y)
        if residual is not None:
            y = y + residual.float()
        return y.to(x.dtype)
    assert x.stride(1) == 1 and w.stride(1) == 1 and K % 64 == 0 and N % 4 == 0
    y = out if out is not None else torch.empty((T, N), dtype=torch.bfloat16, device=x.device)
    rc = _lib.lib().lzk_gemm_bias_act(x.data_ptr(), x.stride(0), T, w.data_ptr(), w.stride(0), N, b.data_ptr(),
                                      _lib.ptr(residual), residual.stride(0) if residual is not None else 0,
                                      y.data_ptr(), y.stride(0), K, 1 if act == "gelu" else 0,
                                      _lib.stream_ptr(x.device))
    _lib.check(rc, "lzk_gemm_bias_act")
    return y


def linear_split2(x: torch.Tensor, w: torch.Tensor, b: torch.Tensor, residual=None):
    """Split-K pair for a following LayerNorm: (ya, yb) with ya + yb ==
    x @ w.T + b (+ residual) -- ya = first K-half + b (+ residual), yb =
    second K-half -- from ONE launch with twice the tiles of :func:`linear`
    (csrc/kernels/encoder.hip gemm256_split2_kernel). K % 128 == 0."""
    T, K = x.shape
    N = w.shape[0]
    if not x.is_cuda:
        h = K // 2
        ya = x[:, :h].float() @ w[:, :h].float().T + b.float()
        if residual is not None:
            ya = ya + residual.float()
        return ya.to(x.dtype), (x[:, h:].float() @ w[:, h:].float().T).to(x.dtype)
    assert x.stride(1) == 1 and w.stride(1) == 1 and K % 128 == 0 and N % 8 == 0
    ya = torch.empty((T, N), dtype=torch.bfloat16, device=x.device)
    yb = torch.empty((T, N), dtype=torch.bfloat16, device=x.device)
    rc = _lib.lib().lzk_gemm_split2(x.data_ptr(), x.stride(0), T, w.data_ptr(), w.stride(0), N, b.data_ptr(),
                                    _lib.ptr(residual), residual.stride(0) if residual is not None else 0,
                                    ya.data_ptr(), yb.data_ptr(), ya.stride(0), K, _lib.stream_ptr(x.device))
    _lib.check(rc, "lzk_gemm_split2")
    return ya, yb


FP8_MAX = 448.0  # OCP e4m3fn (gfx950 MFMA format, == torch.float8_e4m3fn)


def quantize_fp8_rows(x: torch.Tensor):
    """Row-wise symmetric e4m3 quantisation: (q uint8 [R, D], scale fp32 [R])
    with x ~= float(q) * scale[:, None] (scale = amax / 448)."""
    R, D = x.shape
    if not x.is_cuda:
        xf = x.float()
        amax = xf.abs().amax(dim=1)
        sc = torch.where(amax > 0, amax / FP8_MAX, torch.ones_like(amax))
        q = (xf / sc[:, None]).to(torch.float8_e4m3fn).view(torch.uint8)
        return q, sc
    assert x.dtype == torch.bfloat16 and x.stride(1) == 1 and D % 8 == 0
    q = torch.empty((R, D), dtype=torch.uint8, device=x.device)
    sc = torch.empty((R,), dtype=torch.float32, device=x.device)
    rc = _lib.lib().lzk_quant_fp8_rows(x.data_ptr(), x.stride(0), R, D, q.data_ptr(), q.stride(0), sc.data_ptr(),
                                       _lib.stream_ptr(x.device))
    _lib.check(rc, "lzk_quant_fp8_rows")
    return q, sc


def dequantize_fp8_rows(q: torch.Tensor, sc: torch.Tensor) -> torch.Tensor:
    return q.view(torch.float8_e4m3fn).float() * sc[:, None].float()


def linear_fp8(xq: torch.Tensor, sx: torch.Tensor, wq: torch.Tensor, sw: torch.Tensor, b: torch.Tensor,
               act: str = "none", residual=None, out=None) -> torch.Tensor:
    """act((xq*sx) @ (wq*sw).T + b) (+ residual) -> bf16. xq [T,K] / wq [N,K]
    e4m3 bytes (uint8) with per-row scales; K % 128 == 0 on the GPU."""
    T, K = xq.shape
    N = wq.shape[0]
    if not xq.is_cuda:
        y = dequantize_fp8_rows(xq, sx) @ dequantize_fp8_rows(wq, sw).T + b.float()
        if act == "gelu":
            y = F.gelu(y)
        if residual is not None:
            y = y + residual.float()
        return y.to(torch.bfloat16)
    assert xq.dtype == torch.uint8 and wq.dtype == torch.uint8 and K % 128 == 0 and N % 4 == 0
    y = out if out is not None else torch.empty((T, N), dtype=torch.bfloat16, device=xq.device)
    rc = _lib.lib().lzk_gemm_f8(xq.data_ptr(), xq.stride(0), T, sx.data_ptr(), wq.data_ptr(), wq.stride(0), N,
                                sw.data_ptr(), b.data_ptr(), _lib.ptr(residual),
                                residual.stride(0) if residual is not None else 0, y.data_ptr(), y.stride(0), K,
                                1 if act == "gelu" else 0, _lib.stream_ptr(xq.device))
    _lib.check(rc, "lzk_gemm_f8")
    return y


def attention(qkv: torch.Tensor, lens: torch.Tensor, B: int, S: int, nheads: int, out=None,
              cu: torch.Tensor = None) -> torch.Tensor:
    """qkv [B*S, 3H] (q|k|v), head_dim 32/64; keys >= lens[b] are masked.
    Packed ("varlen") layout when ``cu`` (int32 [B+1] row offsets) is given:
    qkv holds only the sum(lens) real tokens, S = max(lens)."""
    H = qkv.shape[1] // 3
    if cu is not None and not qkv.is_cuda:
        outs = []
        for b in range(B):
            r0, r1 = int(cu[b]), int(cu[b + 1])
            outs.append(attention(qkv[r0:r1], lens[b:b + 1], 1, r1 - r0, nheads))
        return torch.cat(outs) if outs else qkv[:, :H].clone()
    if not qkv.is_cuda:
        x = qkv.float().view(B, S, 3, nheads, H // nheads)
        q, k, v = x[:, :, 0].transpose(1, 2), x[:, :, 1].transpose(1, 2), x[:, :, 2].transpose(1, 2)
        s = (q @ k.transpose(-1, -2)) / math.sqrt(H // nheads)
        mask = torch.arange(S, device=qkv.device)[None, :] >= lens[:, None].to(qkv.device)
        s = s.masked_fill(mask[:, None, None, :], float("-inf"))
        o = torch.softmax(s, -1) @ v
        return o.transpose(1, 2).reshape(B * S, H).to(qkv.dtype)
    rows = qkv.shape[0] if cu is not None else B * S
    y = out if out is not None else torch.empty((rows, H), dtype=torch.bfloat16, device=qkv.device)
    rc = _lib.lib().lzk_attention(qkv.data_ptr(), qkv.stride(0), lens.data_ptr(), B, S, H, nheads,
                                  1.0 / math.sqrt(H // nheads), y.data_ptr(), y.stride(0), _lib.ptr(cu),
                                  _lib.stream_ptr(qkv.device))
    _lib.check(rc, "lzk_attention")
    return y


def layernorm(x: torch.Tensor, g: torch.Tensor, b: torch.Tensor, eps: float = 1e-12, residual=None,
              out=None) -> torch.Tensor:
    if not x.is_cuda:
        v = x.float() + (residual.float() if residual is not None else 0.0)
        return F.layer_norm(v, (x.shape[1],), g.float(), b.float(), eps).to(x.dtype)
    rows, H = x.shape
    y = out if out is not None else torch.empty_like(x)
    rc = _lib.lib().lzk_layernorm(x.data_ptr(), x.stride(0), _lib.ptr(residual),
                                  residual.stride(0) if residual is not None else 0, g.data_ptr(), b.data_ptr(),
                                  rows, H, float(eps), y.data_ptr(), y.stride(0), _lib.stream_ptr(x.device))
    _lib.check(rc, "lzk_layernorm")
    return y


def layernorm_q8(x: torch.Tensor, g: torch.Tensor, b: torch.Tensor, eps: float = 1e-12, residual=None):
    """:func:`layernorm` plus the output's row-wise e4m3 copy -- (y, (q, scale))
    with (q, scale) == quantize_fp8_rows(y) -- in one launch on the GPU
    (encoder.hip layernorm16_kernel Q8: H 768 / 1024); elsewhere the two ops."""
    if x.is_cuda and x.shape[1] in (768, 1024):
        rows, H = x.shape
        y = torch.empty_like(x)
        q = torch.empty((rows, H), dtype=torch.uint8, device=x.device)
        sc = torch.empty((rows,), dtype=torch.float32, device=x.device)
        rc = _lib.lib().lzk_layernorm_q8(x.data_ptr(), x.stride(0), _lib.ptr(residual),
                                         residual.stride(0) if residual is not None else 0, g.data_ptr(),
                                         b.data_ptr(), rows, H, float(eps), y.data_ptr(), y.stride(0), q.data_ptr(),
                                         q.stride(0), sc.data_ptr(), _lib.stream_ptr(x.device))
        if rc == 0:
            return y, (q, sc)
    y = layernorm(x, g, b, eps, residual=residual)
    return y, quantize_fp8_rows(y)


def embed_ln(ids: torch.Tensor, S: int, wemb, pemb, temb, g, b, eps: float = 1e-12,
             pos: torch.Tensor = None) -> torch.Tensor:
    """ids [T] int32 -> LN(word[ids] + pos_emb[p] + type[0]) bf16 [T, H] with
    p = t % S (padded batch) or the given per-token positions (packed)."""
    T = ids.numel()
    H = wemb.shape[1]
    if not ids.is_cuda:
        pos = (torch.arange(T, device=ids.device) % S) if pos is None else pos.long()
        v = wemb[ids.long()].float() + pemb[pos].float() + temb[0].float()
        return F.layer_norm(v, (H,), g.float(), b.float(), eps).to(wemb.dtype)
    y = torch.empty((T, H), dtype=torch.bfloat16, device=ids.device)
    rc = _lib.lib().lzk_embed_ln(ids.data_ptr(), T, S, wemb.data_ptr(), pemb.data_ptr(), temb.data_ptr(),
                                 g.data_ptr(), b.data_ptr(), H, float(eps), y.data_ptr(), _lib.ptr(pos),
                                 _lib.stream_ptr(ids.device))
    _lib.check(rc, "lzk_embed_ln")
    return y


def pool_norm(x: torch.Tensor, lens: torch.Tensor, B: int, S: int, mode: str = "mean", out16_width: int = 0,
              cu: torch.Tensor = None):
    """Returns (fp32 [B,H] unit rows, bf16 [B,out16_width] zero-padded copy or None).
    ``cu`` (int32 [B+1]): packed layout, sequence b = rows cu[b]:cu[b+1]."""
    H = x.shape[1]
    if cu is not None and not x.is_cuda:
        xs = torch.zeros((B, S, H), dtype=x.dtype)
        for bb in range(B):
            r0, r1 = int(cu[bb]), int(cu[bb + 1])
            xs[bb, : r1 - r0] = x[r0:r1]
        return pool_norm(xs.view(B * S, H), lens, B, S, mode, out16_width)
    if not x.is_cuda:
        v = x.float().view(B, S, H)
        if mode == "cls":
            p = v[:, 0]
        else:
            m = (torch.arange(S, device=x.device)[None, :] < lens[:, None].to(x.device)).float()
            p = (v * m[..., None]).sum(1) / m.sum(1, keepdim=True).clamp_min(1)
        p = p / p.norm(dim=1, keepdim=True).clamp_min(1e-12)
        o16 = None
        if out16_width:
            o16 = torch.zeros((B, out16_width), dtype=torch.bfloat16, device=x.device)
            o16[:, :H] = p.to(torch.bfloat16)
        return p, o16
    out32 = torch.empty((B, H), dtype=torch.float32, device=x.device)
    out16 = torch.empty((B, out16_width), dtype=torch.bfloat16, device=x.device) if out16_width else None
    rc = _lib.lib().lzk_pool_norm(x.data_ptr(), lens.data_ptr(), B, S, H, 1 if mode == "cls" else 0,
                                  out32.data_ptr(), _lib.ptr(out16), out16_width, _lib.ptr(cu),
                                  _lib.stream_ptr(x.device))
    _lib.check(rc, "lzk_pool_norm")
    return out32, out16
