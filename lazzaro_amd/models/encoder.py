"""BERT-family sentence encoders that run on-device (SURVEY.md §2.2 "vendor
embedding models -> on-device encoder", §2.4 K14).

Configs mirror the public checkpoints the north star names (all-MiniLM-L6-v2,
bge-base-en-v1.5, e5-large-v2): same widths, depths, heads, vocab, positions
and pooling. Weights are random-init (std 0.02, deterministic seed) unless a
safetensors file with HuggingFace BERT parameter names is supplied -- no
checkpoints exist offline (BASELINE.json: "random-init embedding weights").

Forward per layer (all hand-written gfx950 kernels, ``ops.encoder_ops``):
  qkv = X Wqkv^T + b          fused QKV GEMM (one launch)
  ctx = attention(qkv)        flash-style, masked, head_dim 32/64
  X   = LN(ctx Wo^T + b + X)  residual fused into the GEMM epilogue
  H   = gelu(X W1^T + b1)     GELU fused into the GEMM epilogue
  X   = LN(H W2^T + b2 + X)
then masked-mean or CLS pooling + L2 normalisation (one kernel).
"""
from __future__ import annotations

import dataclasses
import os
from dataclasses import dataclass
from typing import Dict, Optional

import numpy as np
import torch

from ..ops import encoder_ops as E


@dataclass(frozen=True)
class EncoderConfig:
    name: str
    hidden: int
    layers: int
    heads: int
    ffn: int
    vocab: int = 30522
    max_pos: int = 512
    pooling: str = "mean"  # "mean" | "cls"
    eps: float = 1e-12


CONFIGS: Dict[str, EncoderConfig] = {
    "minilm-l6": EncoderConfig("minilm-l6", 384, 6, 12, 1536, pooling="mean"),
    "bge-base": EncoderConfig("bge-base", 768, 12, 12, 3072, pooling="cls"),
    "e5-large": EncoderConfig("e5-large", 1024, 24, 16, 4096, pooling="mean"),
    "tiny": EncoderConfig("tiny", 128, 2, 2, 256, vocab=4096, max_pos=128, pooling="mean"),
}
ALIASES = {
    "all-minilm-l6-v2": "minilm-l6", "sentence-transformers/all-minilm-l6-v2": "minilm-l6",
    "bge-base-en": "bge-base", "bge-base-en-v1.5": "bge-base", "baai/bge-base-en-v1.5": "bge-base",
    "e5-large-v2": "e5-large", "intfloat/e5-large-v2": "e5-large",
}


def get_config(name: str) -> EncoderConfig:
    k = name.lower()
    k = ALIASES.get(k, k)
    if k not in CONFIGS:
        raise KeyError(f"unknown encoder {name!r}; known: {sorted(CONFIGS)}")
    return CONFIGS[k]


def _to_dev(t: torch.Tensor, device) -> torch.Tensor:
    t = t.to(torch.int32)
    if t.device.type == "cpu" and torch.device(device).type == "cuda":
        return t.contiguous().pin_memory().to(device, non_blocking=True)
    return t.to(device).contiguous()


# fp8 encoder: each LayerNorm also writes the e4m3 copy its next projection
# reads (False: a separate quantise pass per projection, A/B)
FUSED_LN_Q8 = True


class SentenceEncoder:
    """Weights + forward. ``forward(ids [B,S] int32, lens [B] int32)`` returns
    unit-norm fp32 embeddings [B, H] (and optionally a bf16 copy padded to
    ``pad_to`` columns, ready to be appended to an HBM arena)."""

    def __init__(self, config, device=None, weights: Optional[str] = None, seed: int = 0,
                 dtype=torch.bfloat16, precision: str = "bf16"):
        """precision: "bf16" (all projections on bf16 MFMA) or "fp8" (SURVEY K15 /
        BASELINE config 5: projection weights stored as OCP e4m3 with per-output-
        channel scales, activations quantised per token right before each GEMM,
        fp32 accumulate, bf16 activations everywhere else)."""
        self.cfg = get_config(config) if isinstance(config, str) else config
        self.device = torch.device(device) if device is not None else torch.device("cpu")
        self.dtype = dtype
        if precision not in ("bf16", "fp8"):
            raise ValueError("precision must be 'bf16' or 'fp8'")
        self.precision = precision
        self.q: Dict[str, tuple] = {}
        self.p = self._random_init(seed)
        if weights:
            self.load_safetensors(weights)
        self._quantize()

    _PROJ = ("wqkv", "wo", "w1", "w2")

    def _quantize(self) -> None:
        self.q = {}
        if self.precision != "fp8":
            return
        for i in range(self.cfg.layers):
            for n in self._PROJ:
                self.q[f"{i}.{n}"] = E.quantize_fp8_rows(self.p[f"{i}.{n}"].contiguous())

    # fp8: the LayerNorm that produced a projection's input also wrote its
    # e4m3 copy (E.layernorm_q8): id(bf16 tensor) -> (tensor, (q, scale)) for
    # the last few (forward_streams interleaves the sub-batches' layers)
    _q8 = None

    def _lin(self, x, i: int, w: str, b: str, act: str = "none", residual=None):
        if self.precision == "fp8":
            hit = self._q8.get(id(x)) if self._q8 is not None else None
            if hit is not None and hit[0] is x:
                xq, sx = hit[1]
            else:
                xq, sx = E.quantize_fp8_rows(x)
            wq, sw = self.q[f"{i}.{w}"]
            return E.linear_fp8(xq, sx, wq, sw, self.p[f"{i}.{b}"], act=act, residual=residual)
        return E.linear(x, self.p[f"{i}.{w}"], self.p[f"{i}.{b}"], act=act, residual=residual)

    def _lin_ln(self, x, i: int, w: str, b: str, residual, ln: str, split: bool):
        """LN(x W^T + b + residual). ``split``: the projection as a split-K
        pair (E.linear_split2, one launch with twice the tiles) whose two
        halves the LayerNorm adds -- for the hidden-width projections, whose
        few 256-wide feature tiles leave the last round of a grid mostly empty."""
        p, eps = self.p, self.cfg.eps
        if split:
            ya, yb = E.linear_split2(x, p[f"{i}.{w}"], p[f"{i}.{b}"], residual=residual)
            return E.layernorm(ya, p[f"{i}.{ln}_g"], p[f"{i}.{ln}_b"], eps, residual=yb)
        if self.precision == "fp8" and FUSED_LN_Q8:
            y, q8 = E.layernorm_q8(self._lin(x, i, w, b, residual=residual), p[f"{i}.{ln}_g"], p[f"{i}.{ln}_b"], eps)
            if self._q8 is None or len(self._q8) >= 8:
                self._q8 = {}
            self._q8[id(y)] = (y, q8)
            return y
        return E.layernorm(self._lin(x, i, w, b, residual=residual), p[f"{i}.{ln}_g"], p[f"{i}.{ln}_b"], eps)

    # split-K mode of the hidden-width projections (SPLITK: 0 off, 1 FFN2, 2 O and FFN2).
    # Off by default: in bench.py (same box, profiles/ab_splitk_r1.json) FFN2 split costs the
    # two-stream embed 5.28 -> 5.75 ms and ties on one stream (5.96 / 5.97 ms)
    SPLITK = 0

    def _split_ok(self, x, K: int) -> bool:
        # only grids that take the 256x256 pipeline anyway (>= 64 full-K tiles)
        H = self.cfg.hidden
        return (self.precision == "bf16" and x.is_cuda and K % 128 == 0 and H % 8 == 0
                and ((H + 255) // 256) * ((x.shape[0] + 255) // 256) >= 64)

    def _split_o(self, x) -> bool:
        return SentenceEncoder.SPLITK >= 2 and self._split_ok(x, self.cfg.hidden)

    def _split_ffn2(self, x) -> bool:
        return SentenceEncoder.SPLITK >= 1 and self._split_ok(x, self.cfg.ffn)

    # --------------------------------------------------------------- weights
    def _random_init(self, seed: int) -> Dict[str, torch.Tensor]:
        c, dev = self.cfg, self.device
        g = torch.Generator(device="cpu").manual_seed(seed)

        def w(*shape):
            return (torch.randn(*shape, generator=g) * 0.02).to(dev, self.dtype)

        def zeros(n):
            return torch.zeros(n, dtype=torch.float32, device=dev)

        def ones(n):
            return torch.ones(n, dtype=torch.float32, device=dev)

        H, Fh = c.hidden, c.ffn
        p = {"word": w(c.vocab, H), "pos": w(c.max_pos, H), "type": w(2, H),
             "emb_g": ones(H), "emb_b": zeros(H)}
        for i in range(c.layers):
            p[f"{i}.wqkv"] = w(3 * H, H)
            p[f"{i}.bqkv"] = zeros(3 * H)
            p[f"{i}.wo"] = w(H, H)
            p[f"{i}.bo"] = zeros(H)
            p[f"{i}.ln1_g"], p[f"{i}.ln1_b"] = ones(H), zeros(H)
            p[f"{i}.w1"] = w(Fh, H)
            p[f"{i}.b1"] = zeros(Fh)
            p[f"{i}.w2"] = w(H, Fh)
            p[f"{i}.b2"] = zeros(H)
            p[f"{i}.ln2_g"], p[f"{i}.ln2_b"] = ones(H), zeros(H)
        return p

    def load_safetensors(self, path: str) -> None:
        """Load HuggingFace BERT-layout weights (optionally ``bert.``-prefixed)."""
        from safetensors.torch import load_file

        sd = load_file(path)
        sd = {k[5:] if k.startswith("bert.") else k: v for k, v in sd.items()}
        dev, dt = self.device, self.dtype

        def get(k):
            return sd[k]

        self.p["word"] = get("embeddings.word_embeddings.weight").to(dev, dt)
        self.p["pos"] = get("embeddings.position_embeddings.weight").to(dev, dt)
        self.p["type"] = get("embeddings.token_type_embeddings.weight").to(dev, dt)
        self.p["emb_g"] = get("embeddings.LayerNorm.weight").float().to(dev)
        self.p["emb_b"] = get("embeddings.LayerNorm.bias").float().to(dev)
        for i in range(self.cfg.layers):
            pre = f"encoder.layer.{i}."
            q, k, v = (get(pre + f"attention.self.{n}.weight") for n in ("query", "key", "value"))
            qb, kb, vb = (get(pre + f"attention.self.{n}.bias") for n in ("query", "key", "value"))
            self.p[f"{i}.wqkv"] = torch.cat([q, k, v], 0).to(dev, dt).contiguous()
            self.p[f"{i}.bqkv"] = torch.cat([qb, kb, vb], 0).float().to(dev)
            self.p[f"{i}.wo"] = get(pre + "attention.output.dense.weight").to(dev, dt)
            self.p[f"{i}.bo"] = get(pre + "attention.output.dense.bias").float().to(dev)
            self.p[f"{i}.ln1_g"] = get(pre + "attention.output.LayerNorm.weight").float().to(dev)
            self.p[f"{i}.ln1_b"] = get(pre + "attention.output.LayerNorm.bias").float().to(dev)
            self.p[f"{i}.w1"] = get(pre + "intermediate.dense.weight").to(dev, dt)
            self.p[f"{i}.b1"] = get(pre + "intermediate.dense.bias").float().to(dev)
            self.p[f"{i}.w2"] = get(pre + "output.dense.weight").to(dev, dt)
            self.p[f"{i}.b2"] = get(pre + "output.dense.bias").float().to(dev)
            self.p[f"{i}.ln2_g"] = get(pre + "output.LayerNorm.weight").float().to(dev)
            self.p[f"{i}.ln2_b"] = get(pre + "output.LayerNorm.bias").float().to(dev)
        if hasattr(self, "precision"):
            self._quantize()

    def num_params(self) -> int:
        return sum(t.numel() for t in self.p.values())

    # --------------------------------------------------------------- forward
    def forward(self, ids: torch.Tensor, lens: torch.Tensor, pad_to: int = 0, packed: Optional[bool] = None):
        """ids [B, S] / lens [B] (host or device). Host inputs are staged through
        pinned memory and copied asynchronously, so enqueueing the forward never
        waits for earlier GPU work.

        ``packed`` (default: on for host inputs on a GPU): drop the padding
        tokens before the first layer ("varlen" BERT): every GEMM, LayerNorm and
        the attention run on sum(lens) tokens instead of B*S -- the padded
        positions never influence the pooled embedding (keys >= len are
        masked, pooling stops at len), so they are pure waste."""
        cls = self.cfg.pooling == "cls" and self.CLS_LAST
        x, lens_d, cu, B, S = self._layers(ids, lens, packed, cls_last=cls)
        return E.pool_norm(x, lens_d, B, S, self.cfg.pooling, pad_to, cu=cu)

    # CLS pooling reads only each sequence's first token of the last layer, so
    # that layer's attention output, O projection, FFN and LayerNorms run on
    # the B CLS rows alone (its QKV still covers every token: K and V feed the
    # CLS query). Exact -- the other rows' last-layer states are never read.
    # CLS_LAST = False computes the full last layer.
    CLS_LAST = True

    def _layers(self, ids: torch.Tensor, lens: torch.Tensor, packed: Optional[bool], cls_last: bool = False):
        """Embedding + every transformer layer. Returns (token states, lens on
        the device, cu row offsets (packed) or None, B, S). ``cls_last``: the
        last layer past its attention only for the CLS rows -- returns their
        states [B, H] with cu None and S = 1."""
        c, p = self.cfg, self.p
        B, S = ids.shape
        if packed is None:
            packed = self.device.type == "cuda" and ids.device.type == "cpu" and lens.device.type == "cpu"
        if packed:
            # host-side packing in numpy: single-threaded and ~0.5 ms for 1024 x 32
            # tokens, where torch's CPU ops fan tiny work out to the intra-op
            # thread pool (tens of ms on a shared host)
            lens_n = lens.cpu().numpy().astype(np.int64)
            ids_n = ids.cpu().numpy()
            S_eff = int(lens_n.max()) if B else 1
            mask = np.arange(S)[None, :] < lens_n[:, None]
            ids_p = _to_dev(torch.from_numpy(np.ascontiguousarray(ids_n[mask])), self.device)
            pos_p = _to_dev(torch.from_numpy(np.broadcast_to(np.arange(S, dtype=np.int32), (B, S))[mask]), self.device)
            cu_n = np.zeros(B + 1, dtype=np.int64)
            np.cumsum(lens_n, out=cu_n[1:])
            cu = _to_dev(torch.from_numpy(cu_n), self.device)
            lens = _to_dev(torch.from_numpy(lens_n), self.device)
            x = E.embed_ln(ids_p, S_eff, p["word"], p["pos"], p["type"], p["emb_g"], p["emb_b"], c.eps, pos=pos_p)
            S = S_eff
        else:
            cu = None
            ids = _to_dev(ids, self.device)
            lens = _to_dev(lens, self.device)
            x = E.embed_ln(ids.view(-1), S, p["word"], p["pos"], p["type"], p["emb_g"], p["emb_b"], c.eps)
        for i in range(c.layers):
            qkv = self._lin(x, i, "wqkv", "bqkv")
            ctx = E.attention(qkv, lens, B, S, c.heads, cu=cu)
            if cls_last and i == c.layers - 1 and B > 0:
                first = cu[:-1].long() if cu is not None else torch.arange(B, device=x.device) * S
                ctx, x = ctx.index_select(0, first), x.index_select(0, first)
                cu, S = None, 1
            x = self._lin_ln(ctx, i, "wo", "bo", x, "ln1", split=self._split_o(x))
            hdn = self._lin(x, i, "w1", "b1", act="gelu")
            x = self._lin_ln(hdn, i, "w2", "b2", x, "ln2", split=self._split_ffn2(x))
        return x, lens, cu, B, S

    def hidden_states(self, ids: torch.Tensor, lens: torch.Tensor) -> torch.Tensor:
        """Last-layer token states [B, S, H] fp32 (HF ``last_hidden_state``;
        rows past each sequence's length are zero) -- for parity checks."""
        B, S = ids.shape
        x, lens_d, cu, B, S_eff = self._layers(ids, lens, None)
        H = self.cfg.hidden
        out = torch.zeros((B, S, H), dtype=torch.float32, device=x.device)
        lh = lens.to(torch.int64).cpu().tolist()
        if cu is not None:
            off = 0
            for b, n in enumerate(lh):
                out[b, :n] = x[off: off + n].float()
                off += n
        else:
            xs = x.view(B, S_eff, H)
            for b, n in enumerate(lh):
                out[b, :n] = xs[b, :n].float()
        return out

    def forward_streams(self, ids: torch.Tensor, lens: torch.Tensor, pad_to: int = 0, parts: int = 2,
                        first_frac: float = 0.0):
        """Split the batch into ``parts`` independent sub-batches and run them on
        separate HIP streams. Every layer is a chain of dependent kernels whose
        last wave of 256x256 tiles leaves most CUs idle; kernels of the other
        sub-batch fill those CUs, so the chip stays busy through each tail.
        ``first_frac`` > 0: sub-batch 0 (on the caller's stream, which starts
        first) takes that share of the batch, the rest split evenly."""
        B = ids.shape[0]
        if parts <= 1 or self.device.type != "cuda" or B < 2 * parts:
            return self.forward(ids, lens, pad_to=pad_to)
        cur = torch.cuda.current_stream(self.device)
        if not hasattr(self, "_streams") or len(self._streams) < parts:
            self._streams = [torch.cuda.Stream(self.device) for _ in range(parts)]
        if first_frac > 0.0:
            b0 = min(B - (parts - 1), max(1, int(round(B * first_frac))))
            bounds = [0] + [b0 + (B - b0) * i // (parts - 1) for i in range(parts)]
        else:
            bounds = [B * i // parts for i in range(parts + 1)]
        if not SentenceEncoder.CALLER_STREAM:  # every sub-batch on a side stream
            outs = []
            for i in range(parts):
                st = self._streams[i]
                st.wait_stream(cur)
                with torch.cuda.stream(st):
                    outs.append(self.forward(ids[bounds[i]:bounds[i + 1]], lens[bounds[i]:bounds[i + 1]],
                                             pad_to=pad_to))
            for i in range(parts):
                cur.wait_stream(self._streams[i])
                for t in outs[i]:
                    if t is not None:
                        t.record_stream(cur)
            o32 = torch.cat([o[0] for o in outs])
            o16 = torch.cat([o[1] for o in outs]) if outs[0][1] is not None else None
            return o32, o16
        # sub-batch 0 runs on the caller's stream itself: its first kernels
        # follow the previous work on the same queue at once, while a side
        # stream's cross-queue wait resolves ~0.2 ms after that work ends
        # (rocprofv3 trace of bench.py: 0.2 ms idle per step before the embed)
        for i in range(1, parts):
            self._streams[i - 1].wait_stream(cur)
        outs = []
        for i in range(parts):
            st = cur if i == 0 else self._streams[i - 1]
            with torch.cuda.stream(st):
                o32, o16 = self.forward(ids[bounds[i]:bounds[i + 1]], lens[bounds[i]:bounds[i + 1]], pad_to=pad_to)
                outs.append((o32, o16))
        for i in range(1, parts):
            cur.wait_stream(self._streams[i - 1])
            for t in outs[i]:
                if t is not None:
                    t.record_stream(cur)
        o32 = torch.cat([o[0] for o in outs])
        o16 = torch.cat([o[1] for o in outs]) if outs[0][1] is not None else None
        return o32, o16

    # forward_streams: sub-batch 0 on the caller's stream (CALLER_STREAM = False: all on side streams)
    CALLER_STREAM = True

    def flops(self, tokens: int) -> float:
        c = self.cfg
        per_tok = 2 * (3 * c.hidden * c.hidden + c.hidden * c.hidden + 2 * c.hidden * c.ffn) * c.layers
        return float(per_tok) * tokens


class GraphedEncoder:
    """hipGraph-captured forward for one (batch, seq_len, pad_to) shape.

    Small batches (the per-turn query embed of ``chat`` / ``search_memories``)
    are launch-bound: ~7 kernels per layer, ~90 for bge-base, each a few
    microseconds of GPU work. Capturing the whole forward once and replaying it
    turns that into one graph launch. Inputs are copied into static device
    buffers (padding rows get length 1 and are sliced away); outputs are
    returned as copies so a later replay cannot overwrite them.
    """

    def __init__(self, enc: "SentenceEncoder", batch: int, seq: int, pad_to: int = 0):
        if enc.device.type != "cuda":
            raise ValueError("GraphedEncoder needs a GPU encoder")
        dev = enc.device
        self.enc, self.batch, self.seq, self.pad_to = enc, batch, seq, pad_to
        self.ids = torch.zeros((batch, seq), dtype=torch.int32, device=dev)
        self.lens = torch.ones((batch,), dtype=torch.int32, device=dev)
        side = torch.cuda.Stream(dev)
        side.wait_stream(torch.cuda.current_stream(dev))
        with torch.cuda.stream(side):
            for _ in range(2):  # first-launch work (attribute setup, workspaces) stays out of the graph
                enc.forward(self.ids, self.lens, pad_to=pad_to)
        torch.cuda.current_stream(dev).wait_stream(side)
        self.graph = torch.cuda.CUDAGraph()
        with torch.cuda.graph(self.graph):
            self.out32, self.out16 = enc.forward(self.ids, self.lens, pad_to=pad_to)

    def __call__(self, ids: torch.Tensor, lens: torch.Tensor):
        B, S = ids.shape
        if B > self.batch or S > self.seq:
            raise ValueError("input larger than the captured shape")
        dev = self.ids.device
        self.ids.zero_()
        self.lens.fill_(1)
        self.ids[:B, :S].copy_(ids.to(torch.int32).to(dev, non_blocking=True))
        self.lens[:B].copy_(lens.to(torch.int32).to(dev, non_blocking=True))
        self.graph.replay()
        o16 = self.out16[:B].clone() if self.out16 is not None else None
        return self.out32[:B].clone(), o16
