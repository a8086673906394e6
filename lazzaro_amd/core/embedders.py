"""On-device embedding provider (``EmbeddingProvider`` protocol).

Replaces the reference's remote embedders (providers.py:36-57, 101-128,
170-196): text -> native C++ tokenizer (WordPiece with vocab.txt, hashed ids
without one) -> :class:`~lazzaro_amd.models.encoder.SentenceEncoder` forward on
the GPU (hand-written MFMA kernels) -> unit-norm vectors.

Batching: ``batch_embed`` sorts texts by length and runs buckets of up to
``max_batch`` sequences so padding waste stays small.
"""
from __future__ import annotations

import os
from typing import List, Optional

import numpy as np
import torch

from ..models.encoder import GraphedEncoder, SentenceEncoder, get_config
from ..utils.device import default_device

# sub-batches (HIP streams) of a large-batch embed; bench/ab_embed_parts.py
EMBED_PARTS = max(1, int(os.environ.get("LZK_EMBED_PARTS", "2")))


class Tokenizer:
    """Thin wrapper over the native tokenizer (``_lzrt.Tokenizer``)."""

    def __init__(self, vocab_file: Optional[str] = None, vocab_size: int = 30522):
        from ..store.colstore import _rt

        self._t = _rt().Tokenizer(vocab_size, True)
        if vocab_file:
            if not self._t.load_vocab(vocab_file):
                raise FileNotFoundError(vocab_file)

    def encode(self, text: str, max_len: int = 512) -> List[int]:
        return list(self._t.encode(text, max_len))

    def encode_batch(self, texts: List[str], max_len: int = 512):
        ids, lens = self._t.encode_batch(list(texts), max_len)
        return torch.from_numpy(np.asarray(ids)), torch.from_numpy(np.asarray(lens))

    def encode_chunks(self, texts: List[str], max_len: int = 512, overlap: int = 64):
        """Overlapping windows for texts longer than ``max_len`` (owner[i] = text)."""
        ids, lens, owner = self._t.encode_chunks(list(texts), max_len, overlap)
        return (torch.from_numpy(np.asarray(ids)), torch.from_numpy(np.asarray(lens)),
                torch.from_numpy(np.asarray(owner)))


class OnDeviceEmbedder:
    def __init__(self, model: str = "bge-base", device=None, weights: Optional[str] = None,
                 vocab_file: Optional[str] = None, max_len: int = 512, max_batch: int = 1024, seed: int = 0,
                 precision: str = "bf16", graphs: bool = True):
        self.cfg = get_config(model)
        self.device = torch.device(device) if device is not None else default_device()
        self.encoder = SentenceEncoder(self.cfg, device=self.device, weights=weights, seed=seed, precision=precision)
        # small batches replay a captured hipGraph per (batch, seq) bucket
        self.graphs = graphs and self.device.type == "cuda"
        self._graphs = {}
        self.tok = Tokenizer(vocab_file, vocab_size=self.cfg.vocab)
        self.max_len = min(max_len, self.cfg.max_pos)
        self.max_batch = max_batch
        self.dim = self.cfg.hidden

    GRAPH_MAX_BATCH = 8

    def embed_tensor(self, texts: List[str], pad_to: int = 0):
        ids, lens = self.tok.encode_batch(texts, self.max_len)
        B, S = ids.shape
        if self.graphs and B <= self.GRAPH_MAX_BATCH:
            bb = 1 << max(0, (B - 1).bit_length())
            sb = min(self.max_len, max(16, 1 << max(0, (S - 1).bit_length())))
            if S <= sb:
                key = (bb, sb, pad_to)
                g = self._graphs.get(key)
                if g is None:
                    g = self._graphs[key] = GraphedEncoder(self.encoder, bb, sb, pad_to)
                return g(ids, lens)
        if B >= 512:  # large batches: sub-batches on separate streams fill each GEMM's tail
            return self.encoder.forward_streams(ids, lens, pad_to=pad_to, parts=EMBED_PARTS)
        return self.encoder.forward(ids, lens, pad_to=pad_to)

    def embed(self, text: str) -> List[float]:
        return self.batch_embed([text])[0]

    def embed_long(self, texts: List[str], overlap: int = 64) -> torch.Tensor:
        """Texts of any length: windows of the model's max length with
        ``overlap`` tokens of overlap, window embeddings averaged per text and
        re-normalised (long-context row). Returns [n, H] fp32."""
        ids, lens, owner = self.tok.encode_chunks(texts, self.max_len, overlap)
        outs = []
        for s in range(0, ids.shape[0], self.max_batch):
            v, _ = self.encoder.forward(ids[s: s + self.max_batch], lens[s: s + self.max_batch])
            outs.append(v)
        v = torch.cat(outs)
        own = owner.to(v.device).long()
        acc = torch.zeros((len(texts), v.shape[1]), dtype=v.dtype, device=v.device).index_add_(0, own, v)
        return acc / acc.norm(dim=1, keepdim=True).clamp_min(1e-30)

    def batch_embed_tensor(self, texts: List[str]) -> torch.Tensor:
        """[n, H] fp32 unit vectors on the encoder's device, in input order
        (no host round trip: the memory graph ingests / searches with it)."""
        if any(len(t) > 4 * self.max_len for t in texts):
            return torch.as_tensor(np.asarray(self.batch_embed(texts), dtype=np.float32)).to(self.device)
        if self.device.type == "cuda":
            # the GPU forward packs tokens (padding is never computed), so no
            # length sort / scatter: input order, and nothing here waits for
            # the device (host inputs go through pinned async copies)
            outs = [self.embed_tensor(texts[s: s + self.max_batch])[0] for s in range(0, len(texts), self.max_batch)]
            out = outs[0] if len(outs) == 1 else torch.cat(outs)
            return out if out.dtype == torch.float32 else out.float()
        order = sorted(range(len(texts)), key=lambda i: len(texts[i]))
        out = torch.empty((len(texts), self.dim), dtype=torch.float32, device=self.device)
        for s in range(0, len(order), self.max_batch):
            idx = order[s: s + self.max_batch]
            v32, _ = self.embed_tensor([texts[i] for i in idx])
            out[torch.as_tensor(idx, dtype=torch.long, device=self.device)] = v32.float()
        return out

    def batch_embed(self, texts: List[str]) -> List[List[float]]:
        if not texts:
            return []
        if any(len(t) > 4 * self.max_len for t in texts):
            # possibly longer than the model: chunk + average (cheap char-length screen first)
            long_ids = [i for i, t in enumerate(texts) if len(self.tok.encode(t, 1 << 30)) > self.max_len]
            if long_ids:
                out = [None] * len(texts)
                lv = self.embed_long([texts[i] for i in long_ids]).cpu().tolist()
                for i, r in zip(long_ids, lv):
                    out[i] = r
                rest = [i for i in range(len(texts)) if out[i] is None]
                for i, r in zip(rest, self.batch_embed([texts[i] for i in rest]) if rest else []):
                    out[i] = r
                return out
        order = sorted(range(len(texts)), key=lambda i: len(texts[i]))
        out: List[Optional[List[float]]] = [None] * len(texts)
        for s in range(0, len(order), self.max_batch):
            idx = order[s: s + self.max_batch]
            v32, _ = self.embed_tensor([texts[i] for i in idx])
            rows = v32.cpu().tolist()
            for i, r in zip(idx, rows):
                out[i] = r
        return out  # type: ignore[return-value]
