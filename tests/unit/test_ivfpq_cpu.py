"""IVF-PQ index: CPU reference pipeline (train / add / search / rerank)."""
import torch

from lazzaro_amd.index.ivfpq import IVFPQIndex, recall_at_k


def _data(n, d, seed, clusters=32):
    g = torch.Generator().manual_seed(seed)
    c = torch.nn.functional.normalize(torch.randn(clusters, d, generator=g), dim=1)
    lab = torch.randint(0, clusters, (n,), generator=g)
    return torch.nn.functional.normalize(c[lab] + 0.3 * torch.randn(n, d, generator=g) / d ** 0.5 * 4, dim=1)


def test_ivfpq_cpu_recall_and_memory():
    d = 64
    x = _data(4000, d, 0)
    q = _data(20, d, 1)
    idx = IVFPQIndex(d, nlist=16, m=16, device="cpu", keep_vectors=True)
    idx.train(x, iters=6, pq_iters=6)
    idx.add(x)
    assert len(idx) == 4000 and idx.memory_bytes() >= 4000 * 24
    truth = torch.topk(q @ x.T, 10, dim=1).indices
    _, ids = idx.search(q, 10, nprobe=16)
    r_pq = recall_at_k(ids, truth)
    _, ids2 = idx.search(q, 10, nprobe=16, rerank=16)
    r_rr = recall_at_k(ids2, truth)
    assert r_pq > 0.4 and r_rr >= r_pq and r_rr > 0.7, (r_pq, r_rr)
    # fewer probes -> lower (or equal) recall, never errors
    _, ids3 = idx.search(q, 10, nprobe=2)
    assert ids3.shape == (20, 10)


def test_ivfpq_add_incremental_ids():
    d = 32
    x = _data(1000, d, 3, clusters=8)
    idx = IVFPQIndex(d, nlist=8, m=8, device="cpu")
    idx.train(x, iters=4, pq_iters=4)
    idx.add(x[:500])
    idx.add(x[500:], ids=torch.arange(10_000, 10_500))
    s, ids = idx.search(x[600:601], 1, nprobe=8)
    assert int(ids[0, 0]) >= 10_000 or int(ids[0, 0]) < 500
    assert sorted(idx.ids.tolist())[-1] == 10_499


def test_ivfpq_fp8_rerank_copy():
    d = 64
    x = _data(4000, d, 5)
    q = _data(20, d, 6)
    idx = IVFPQIndex(d, nlist=16, m=16, device="cpu", keep_vectors="fp8")
    idx.train(x, iters=6, pq_iters=6)
    idx.add(x)
    assert idx.vectors.dtype == torch.uint8 and idx.vscale.shape == (4000,)
    assert idx.memory_bytes() == 4000 * (16 + 4 + 8 + 8 + d + 4)  # codes, list, pos, id, fp8 row, scale
    truth = torch.topk(q @ x.T, 10, dim=1).indices
    _, ids = idx.search(q, 10, nprobe=16, rerank=32)
    assert recall_at_k(ids, truth) > 0.8


def test_store_ivfpq_tenant_matches_flat_top1(tmp_path):
    """HBMStore(index="ivfpq"): a tenant above the row threshold is served by
    IVF-PQ candidates + exact re-rank; near-duplicate queries find their row."""
    import numpy as np

    from lazzaro_amd.core.vector_store import HBMStore
    st = HBMStore(db_dir=str(tmp_path / "ivf"), device="cpu", metric="cosine", index="ivfpq",
                  nlist=32, nprobe=8, pq_m=8, ivf_min_rows=1000)
    flat = HBMStore(db_dir=str(tmp_path / "flat"), device="cpu", metric="cosine")
    x = _data(3000, 32, 9).numpy()
    rows = [{"id": f"m{i}", "content": "c", "embedding": v.tolist()} for i, v in enumerate(x)]
    st.add_nodes(rows, user_id="big")
    flat.add_nodes(rows, user_id="big")
    q = x[:40] + 0.01 * np.random.default_rng(0).standard_normal((40, 32)).astype(np.float32)
    got = [st.search_nodes(v.tolist(), user_id="big", limit=3) for v in q]
    want = [flat.search_nodes(v.tolist(), user_id="big", limit=3) for v in q]
    assert st._arena("big").ivf is not None and st._arena("big").ivf.idx is not None
    assert sum(g[0] == w[0] for g, w in zip(got, want)) >= 38
    st.delete_nodes(["m0"], user_id="big")
    assert "m0" not in st.search_nodes(q[0].tolist(), user_id="big", limit=3)


def test_ivfpq_int8_rerank_copy_beats_fp8():
    """int8 re-rank copy (per-row absmax scale): same D+4 bytes as fp8, finer
    grid -> higher recall on clustered 1024-d data (CPU reference path)."""
    g = torch.Generator().manual_seed(2)
    d, n = 1024, 6000
    c = torch.nn.functional.normalize(torch.randn(3, d, generator=g), dim=1)
    x = torch.nn.functional.normalize(c[torch.randint(0, 3, (n,), generator=g)] + 0.6 * torch.randn(n, d, generator=g)
                                      / d ** 0.5, dim=1)
    q = torch.nn.functional.normalize(c[torch.randint(0, 3, (40,), generator=g)] + 0.6 * torch.randn(40, d, generator=g)
                                      / d ** 0.5, dim=1)
    truth = torch.topk(q @ x.T, 10, dim=1).indices
    rec = {}
    for keep in ("fp8", "int8"):
        idx = IVFPQIndex(d, nlist=4, m=64, device="cpu", keep_vectors=keep)
        idx.train(x[:3000], iters=4, pq_iters=4)
        idx.add(x)
        _, ids = idx.search(q, 10, nprobe=4, rerank=n)
        rec[keep] = recall_at_k(ids, truth)
    assert rec["int8"] >= 0.93 and rec["int8"] > rec["fp8"], rec
