"""Batched cosine similarity for the orchestrator's graph maintenance.

The reference computes every similarity as a separate numpy call on Python
lists (``memory_system.py:197-203``, ~100 us/pair; linking is O(M*N) such
calls). Here every linking / hierarchy / merge step is one
batched ``[M, D] x [D, N]`` product:

* small problems: float64 numpy on cached unit rows (bit-for-bit the same
  decisions as the reference's float64 cosine);
* large problems on a GPU: the fused MFMA top-k kernel (``ops.flat_topk``) on
  bf16 rows with an fp32 re-rank, so only the top candidates ever leave HBM.

Node embeddings are Python lists at the API level; :class:`EmbeddingCache`
converts each node once (keyed by the list object's identity) instead of on
every pass.
"""
from __future__ import annotations

from typing import Dict, List, Optional, Sequence, Tuple

import numpy as np
import torch

from ..models.graph import Node

GPU_MIN_WORK = 1 << 22  # M*N above which the device kernel is used


class EmbeddingCache:
    def __init__(self):
        self._rows: Dict[str, Tuple[int, int, np.ndarray]] = {}

    def unit(self, node: Node) -> np.ndarray:
        e = node.embedding
        key = (id(e), len(e) if e is not None else 0)
        hit = self._rows.get(node.id)
        if hit is not None and hit[0] == key[0] and hit[1] == key[1]:
            return hit[2]
        v = np.asarray(e if e is not None else [], dtype=np.float64)
        n = float(np.linalg.norm(v)) if v.size else 0.0
        u = v / n if n > 0 else np.zeros_like(v)
        self._rows[node.id] = (key[0], key[1], u)
        return u

    def matrix(self, nodes: Sequence[Node], dim: Optional[int] = None) -> np.ndarray:
        if not nodes:
            return np.zeros((0, dim or 0))
        rows = [self.unit(n) for n in nodes]
        d = dim if dim is not None else max((r.size for r in rows), default=0)
        out = np.zeros((len(rows), d))
        for i, r in enumerate(rows):
            if r.size == d:
                out[i] = r
        return out

    def forget(self, node_ids) -> None:
        for i in node_ids:
            self._rows.pop(i, None)


def cosine_matrix(A: np.ndarray, B: np.ndarray) -> np.ndarray:
    """Cosine of unit rows (zeros stay zero, like the reference's norm==0 -> 0)."""
    if A.size == 0 or B.size == 0 or A.shape[1] != B.shape[1]:
        return np.zeros((A.shape[0], B.shape[0]))
    return A @ B.T


def topk_cosine(A: np.ndarray, B: np.ndarray, k: int, mask: Optional[np.ndarray] = None,
                device: Optional[torch.device] = None) -> Tuple[np.ndarray, np.ndarray]:
    """Per row of A: the k most similar rows of B (descending, ties -> lower
    index first, as Python's stable sort in the reference). ``mask[i, j]`` False
    excludes a pair. Returns (sims [M,k], idx [M,k]) with -1 for empty slots."""
    M, N = A.shape[0], B.shape[0]
    k_eff = min(k, N)
    if M == 0 or N == 0 or k_eff == 0:
        return np.full((M, k), -np.inf), np.full((M, k), -1, dtype=np.int64)
    use_gpu = (device is not None and device.type == "cuda" and mask is None and k_eff <= 16
               and M * N >= GPU_MIN_WORK)
    if use_gpu:
        from ..ops.search import flat_topk

        D = A.shape[1]
        Dp = (D + 63) // 64 * 64
        Xb = torch.zeros((N, Dp), dtype=torch.bfloat16, device=device)
        Xb[:, :D] = torch.as_tensor(B, dtype=torch.float32, device=device).to(torch.bfloat16)
        Qb = torch.zeros((M, Dp), dtype=torch.bfloat16, device=device)
        Qb[:, :D] = torch.as_tensor(A, dtype=torch.float32, device=device).to(torch.bfloat16)
        kc = min(16, max(k_eff, 4 * k_eff), N)
        _, cand = flat_topk(Xb, Qb, kc)
        cand = cand.cpu().numpy()
        sims = np.full((M, k), -np.inf)
        idx = np.full((M, k), -1, dtype=np.int64)
        for i in range(M):
            c = cand[i][cand[i] >= 0]
            s = B[c] @ A[i]
            o = sorted(range(len(c)), key=lambda j: (-s[j], c[j]))[:k_eff]
            sims[i, : len(o)] = s[o]
            idx[i, : len(o)] = c[o]
        return sims, idx
    S = cosine_matrix(A, B)
    if mask is not None:
        S = np.where(mask, S, -np.inf)
    o = np.argsort(-S, axis=1, kind="stable")[:, :k_eff]
    sims = np.take_along_axis(S, o, axis=1)
    idx = np.where(np.isneginf(sims), -1, o)
    if k_eff < k:
        sims = np.concatenate([sims, np.full((M, k - k_eff), -np.inf)], 1)
        idx = np.concatenate([idx, np.full((M, k - k_eff), -1)], 1)
    return sims, idx
