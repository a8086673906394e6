"""Interactive-path latency on one GPU (the per-turn work of ``chat`` /
``search_memories``, reference memory_system.py:262-351, 1460-1472): one
query text -> on-device embedding -> exact top-k over one user's memories.

Reports p50/p99 for: the bge-base query embed eager vs hipGraph replay, the
single-query flat scan of a 1M-row and a 10M-row arena, the end-to-end
``HBMStore.search_nodes`` call, and through ``MemorySystem`` on the GPU:
``search_memories`` and the chat retrieval (embed + retrieve + boost, LLM
excluded) over 200k- and 10M-memory tenants. Synthetic data, random-init
weights.
"""
import argparse
import json
import os
import statistics
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def pct(ts, p):
    ts = sorted(ts)
    return round(ts[min(len(ts) - 1, int(p / 100.0 * len(ts)))] * 1e3, 3)


def timed(fn, n):
    out = []
    for _ in range(n):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        fn()
        torch.cuda.synchronize()
        out.append(time.perf_counter() - t0)
    return {"p50_ms": pct(out, 50), "p99_ms": pct(out, 99), "mean_ms": round(statistics.mean(out) * 1e3, 3)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=200)
    ap.add_argument("--model", default="bge-base")
    ap.add_argument("--api-only", action="store_true", help="only the 10M-memory MemorySystem sections")
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    from lazzaro_amd.core.embedders import OnDeviceEmbedder
    from lazzaro_amd.ops.search import flat_topk

    emb = OnDeviceEmbedder(a.model, device=dev, max_len=64)
    q = "what did I say about moving to Lisbon and learning the cello?"
    ids, lens = emb.tok.encode_batch([q], emb.max_len)
    res = {"metric": "interactive search_memories latency", "model": a.model}
    if a.api_only:
        return api(a, emb, q, dev, res, (10_000_000,))
    for _ in range(5):
        emb.encoder.forward(ids, lens)
        emb.embed_tensor([q])
    res["embed_1q_eager"] = timed(lambda: emb.encoder.forward(ids, lens), a.iters)
    res["embed_1q_hipgraph"] = timed(lambda: emb.embed_tensor([q]), a.iters)
    _, q16 = emb.encoder.forward(ids, lens, pad_to=768)
    for n in (1_000_000, 10_000_000):
        X = torch.empty((n, 768), dtype=torch.bfloat16, device=dev)
        for r0 in range(0, n, 1 << 20):
            m = min(1 << 20, n - r0)
            X[r0:r0 + m] = torch.nn.functional.normalize(torch.randn(m, 768, device=dev), dim=1).to(torch.bfloat16)
        flat_topk(X, q16, 5)
        res[f"scan_1q_{n // 1_000_000}M"] = timed(lambda: flat_topk(X, q16, 5), a.iters)
        res[f"scan_1q_{n // 1_000_000}M"]["GBps_at_p50"] = round(n * 768 * 2 / (res[f"scan_1q_{n // 1_000_000}M"]["p50_ms"] / 1e3) / 1e9, 1)
        del X
        torch.cuda.empty_cache()
    # end to end through the store: one user with 200k memories
    import tempfile

    from lazzaro_amd.core.vector_store import HBMStore
    with tempfile.TemporaryDirectory() as d:
        st = HBMStore(db_dir=d, device=dev)
        n = 200_000
        rng = np.random.default_rng(0)
        vec = rng.standard_normal((n, 768)).astype(np.float32)
        vec /= np.linalg.norm(vec, axis=1, keepdims=True)
        arena = st._arena("u")
        arena.add([f"m{i}" for i in range(n)], vec)
        qv = emb.embed(q)
        st.search_nodes(qv, user_id="u", limit=5)
        res["store_search_200k"] = timed(lambda: st.search_nodes(qv, user_id="u", limit=5), a.iters // 2)
        res["embed_plus_store_search_200k"] = timed(
            lambda: st.search_nodes(emb.embed(q), user_id="u", limit=5), a.iters // 2)
    api(a, emb, q, dev, res, (200_000, 10_000_000))


def api(a, emb, q, dev, res, sizes):
    """Through the product API: MemorySystem on the GPU, the tenant graph in
    HBM (search_memories = embed + store search + Node mapping; the chat
    retrieval = embed + hierarchical/vector retrieval + neighbour boost, LLM
    excluded); plus the store search alone (the embedded query given)."""
    import tempfile

    from bench import populate
    from lazzaro_amd.core.memory_system import MemorySystem
    from lazzaro_amd.core.providers import LocalLLM
    for n in sizes:
        with tempfile.TemporaryDirectory() as d:
            ms = MemorySystem(llm_provider=LocalLLM(), embedding_provider=emb, device=dev, db_dir=d,
                              load_from_disk=False, enable_async=False, enable_caching=False,
                              max_buffer_size=2 * n)
            populate(ms, n, 768, dev, seed=1)
            ms.start_conversation()
            tag = f"{n // 1000}k" if n < 1_000_000 else f"{n // 1_000_000}M"
            ms.search_memories(q, limit=5)
            res[f"api_search_memories_{tag}"] = timed(lambda: ms.search_memories(q, limit=5), a.iters // 2)
            qe = emb.embed_tensor([q])[0]
            g = ms.graph
            g.store_search(qe, 5)
            res[f"store_search_only_{tag}"] = timed(lambda: g.store_search(qe, 5), a.iters // 2)
            res[f"embed_only_{tag}"] = timed(lambda: emb.embed_tensor([q]), a.iters // 2)
            ms._retrieve_for(q)
            res[f"api_chat_retrieval_{tag}"] = timed(lambda: ms._retrieve_for(q), a.iters // 2)
            ms.close()
            del ms
            torch.cuda.empty_cache()
    print(json.dumps(res), flush=True)
    return res


if __name__ == "__main__":
    main()
