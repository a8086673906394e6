"""Graph kernels (csrc/kernels/graph.hip) vs their torch/host references."""
import pytest
import torch

pytestmark = pytest.mark.gpu

from lazzaro_amd.index.kmeans import kmeans  # noqa: E402
from lazzaro_amd.ops import graph_ops as G  # noqa: E402

DEV = "cuda"


def _rand_edges(n, ne, seed, dev):
    g = torch.Generator().manual_seed(seed)
    src = torch.randint(0, n, (ne,), generator=g, dtype=torch.int32)
    dst = torch.randint(0, n, (ne,), generator=g, dtype=torch.int32)
    w = torch.rand(ne, generator=g)
    e = {"src": src, "dst": dst, "w": w, "co": torch.arange(ne, dtype=torch.int32),
         "lu": torch.rand(ne, generator=g, dtype=torch.float64)}
    return {k: v.to(dev) for k, v in e.items()}


@pytest.mark.parametrize("n,ne", [(10, 5), (20000, 15000), (100000, 300000)])
def test_connected_components_gpu(n, ne):
    e = _rand_edges(n, ne, 11, "cpu")
    ref = G.connected_components(e["src"], e["dst"], n, e["w"], 0.3)
    got = G.connected_components(e["src"].to(DEV), e["dst"].to(DEV), n, e["w"].to(DEV), 0.3)
    assert torch.equal(ref.to(torch.int32), got.cpu())


def test_chain_components_gpu():
    n = 200000
    s = torch.arange(n - 1, dtype=torch.int32, device=DEV)
    lab = G.connected_components(s, s + 1, n)
    assert int(lab.max()) == 0
    # reversed and shuffled chain (worst case for index-ordered hooking)
    p = torch.randperm(n - 1, generator=torch.Generator().manual_seed(4)).to(DEV)
    lab = G.connected_components((s + 1).flip(0)[p], s.flip(0)[p], n)
    assert int(lab.max()) == 0


@pytest.mark.parametrize("method", ["uf", "hook"])
@pytest.mark.parametrize("n,ne,seed", [(2_000_000, 4_000_000, 1), (3_000_000, 1_000_000, 2), (50_000, 2, 3)])
def test_components_methods_large_gpu(method, n, ne, seed):
    """Union-find and hook/compress give the host union-find's labels
    (smallest row per component) on a giant-component graph, a graph of many
    small components and a nearly empty one."""
    e = _rand_edges(n, ne, seed, "cpu")
    ref = G.connected_components(e["src"], e["dst"], n)
    got = G.connected_components(e["src"].to(DEV), e["dst"].to(DEV), n, method=method)
    assert torch.equal(ref.to(torch.int32), got.cpu())


@pytest.mark.parametrize("plain", [True, False])
def test_union_find_load_flavours_gpu(plain, monkeypatch):
    """Cached (default) and agent-scope atomic parent loads in uf_union_kernel
    both give the host union-find's labels, staged (8 stages) and in one pass."""
    n, ne = 4_000_000, 16_000_000
    e = _rand_edges(n, ne, 7, "cpu")
    ref = G.connected_components(e["src"], e["dst"], n).to(torch.int32)
    s, d = e["src"].to(DEV), e["dst"].to(DEV)
    monkeypatch.setattr(G, "UF_PLAIN", plain)
    for stages in (0, 1):
        monkeypatch.setattr(G, "UF_STAGES", stages)
        assert torch.equal(ref, G.connected_components(s, d, n).cpu())


def test_pairs_above_gpu():
    g = torch.Generator().manual_seed(3)
    base = torch.nn.functional.normalize(torch.randn(200, 128, generator=g), dim=1)
    X = torch.cat([base, base[:50] + 0.01 * torch.randn(50, 128, generator=g)])
    X = torch.nn.functional.normalize(X, dim=1).to(torch.bfloat16)
    ref = G.pairs_above(X.float(), 0.95)
    got = G.pairs_above(X.to(DEV), 0.95).cpu()
    assert torch.equal(ref, got) and got.shape[0] >= 50


def test_centroids_gpu():
    g = torch.Generator().manual_seed(4)
    X = torch.nn.functional.normalize(torch.randn(5000, 256, generator=g), dim=1).to(torch.bfloat16)
    lab = torch.randint(-1, 37, (5000,), generator=g, dtype=torch.int32)
    c, _, cnt = G.centroids(X.float(), lab, 37)
    cg, c16, cntg = G.centroids(X.to(DEV), lab.to(DEV), 37, pad_to=256)
    assert torch.equal(cnt, cntg.cpu()) and torch.allclose(c, cg.cpu(), atol=1e-5)


@pytest.mark.parametrize("atomic", [False, True])
@pytest.mark.parametrize("D", [256, 768, 2048])
def test_seg_sum_paths_gpu(atomic, D, monkeypatch):
    """Sorted (atomic-free) and atomic segmented sums vs an fp32 reference:
    uneven clusters (one empty, one holding a third of the rows), label -1
    rows, a strided (padded-arena) view, un-normalised sums."""
    monkeypatch.setattr(G, "SEG_SUM_ATOMIC", atomic)
    g = torch.Generator().manual_seed(D)
    n, C = 7001, 53
    full = torch.randn(n, D + 64, generator=g).to(torch.bfloat16)
    X = full[:, :D]
    lab = torch.randint(-1, C, (n,), generator=g, dtype=torch.int32)
    lab[lab == 7] = 8
    lab[: n // 3] = 11
    m = lab >= 0
    ref = torch.zeros(C, D).index_add_(0, lab[m].long(), X[m].float())
    rc = torch.bincount(lab[m].long(), minlength=C).to(torch.int32)
    c32, _, cnt = G.centroids(full.to(DEV)[:, :D], lab.to(DEV), C, normalize=False)
    sums = c32.cpu() * cnt.cpu().clamp_min(1)[:, None].float()
    assert torch.equal(cnt.cpu(), rc) and int(cnt[7]) == 0
    assert torch.allclose(sums, ref, atol=2e-3, rtol=1e-4)


def test_kmeans_gpu():
    torch.manual_seed(1)
    centers = torch.nn.functional.normalize(torch.randn(16, 128), dim=1)
    X = torch.cat([torch.nn.functional.normalize(c + 0.05 * torch.randn(500, 128), dim=1) for c in centers])
    c32, c16, lab = kmeans(X.to(DEV).to(torch.bfloat16), 16, iters=6)
    lab = lab.cpu()
    for j in range(16):
        assert len(set(lab[j * 500:(j + 1) * 500].tolist())) == 1


def test_ivfpq_gpu_scan_matches_reference():
    from lazzaro_amd.index.ivfpq import IVFPQIndex, recall_at_k
    g = torch.Generator().manual_seed(0)
    d, n = 128, 20000
    c = torch.nn.functional.normalize(torch.randn(64, d, generator=g), dim=1)
    x = torch.nn.functional.normalize(c[torch.randint(0, 64, (n,), generator=g)] + 0.1 * torch.randn(n, d, generator=g), dim=1)
    q = x[:50] + 0.01 * torch.randn(50, d, generator=g)
    gi = IVFPQIndex(d, nlist=64, m=32, device=DEV, keep_vectors=True)
    gi.train(x, iters=5, pq_iters=5)
    gi.add(x)
    gi._finalize()
    ci = IVFPQIndex(d, nlist=64, m=32, device="cpu")
    ci.centroids, ci.codebooks = gi.centroids.cpu(), gi.codebooks.cpu()
    ci.codes, ci.ids, ci.list_of, ci.list_off = gi.codes.cpu(), gi.ids.cpu(), gi.list_of.cpu(), gi.list_off.cpu()
    s1, i1 = gi.search(q, 10, nprobe=8)
    s2, i2 = ci.search(q, 10, nprobe=8)
    torch.testing.assert_close(s1.cpu(), s2, atol=1e-4, rtol=1e-4)
    assert (i1.cpu() == i2).float().mean() > 0.98
    truth = torch.topk(torch.nn.functional.normalize(q, dim=1) @ x.T, 10, dim=1).indices
    _, i3 = gi.search(q, 10, nprobe=16, rerank=16)
    assert recall_at_k(i3, truth) > 0.8


def test_ivfpq_deep_rerank():
    from lazzaro_amd.index.ivfpq import IVFPQIndex, recall_at_k
    g = torch.Generator().manual_seed(1)
    d, n = 128, 30000
    c = torch.nn.functional.normalize(torch.randn(32, d, generator=g), dim=1)
    x = torch.nn.functional.normalize(c[torch.randint(0, 32, (n,), generator=g)] + 0.15 * torch.randn(n, d, generator=g), dim=1)
    q = torch.nn.functional.normalize(x[:64] + 0.02 * torch.randn(64, d, generator=g), dim=1)
    gi = IVFPQIndex(d, nlist=32, m=16, device=DEV, keep_vectors=True)
    gi.train(x, iters=5, pq_iters=5)
    gi.add(x)
    truth = torch.topk(q @ x.T, 10, dim=1).indices
    _, i_pq = gi.search(q, 10, nprobe=8)
    _, i_rr = gi.search(q, 10, nprobe=8, rerank=200)
    r_pq, r_rr = recall_at_k(i_pq, truth), recall_at_k(i_rr, truth)
    assert r_rr >= r_pq and r_rr > 0.9, (r_pq, r_rr)


def test_ivfpq_clustered_recall_int8_rerank():
    """Config-5 quality on clustered data (Gaussian mixture, d=1024): deep
    candidates (ivfpq_scan_deep_kernel) + the int8 re-rank copy reach
    recall@10 >= 0.9 against the exact fp32 inner product."""
    from lazzaro_amd.index.ivfpq import IVFPQIndex, recall_at_k
    from lazzaro_amd.ops.search import flat_topk
    g = torch.Generator(device=DEV).manual_seed(4)
    d, n, C = 1024, 400_000, 2000
    cen = torch.nn.functional.normalize(torch.randn(C, d, device=DEV, generator=g), dim=1)

    def draw(m):
        lab = torch.randint(0, C, (m,), device=DEV, generator=g)
        return torch.nn.functional.normalize(cen[lab] + torch.randn(m, d, device=DEV, generator=g) / d ** 0.5, dim=1)
    x, q = draw(n), draw(256)
    idx = IVFPQIndex(d, nlist=1024, m=64, device=DEV, keep_vectors="int8")
    idx.train(x[:100_000], iters=6, pq_iters=6)
    idx.add(x)
    # exact fp32 truth: bf16 top-64 candidates re-scored in fp32
    _, cand = flat_topk(x.to(torch.bfloat16), q.to(torch.bfloat16), 16)
    s = torch.einsum("qd,qkd->qk", q, x[cand])
    truth = torch.gather(cand, 1, torch.topk(s, 10, dim=1).indices)
    _, ids = idx.search(q, 10, nprobe=32, rerank=512)
    r = recall_at_k(ids, truth)
    assert r >= 0.9, r


def test_debug_build_catches_bad_index():
    """LZK_DEBUG build: a negative edge endpoint is reported by LZK_DCHECK
    (per-file error word) and skipped instead of being dereferenced."""
    import ctypes
    import os

    from lazzaro_amd.ops import _lib
    path = os.path.join(os.path.dirname(_lib.LIB_PATH), "liblzk_debug.so")
    if not os.path.exists(path):
        pytest.skip("debug library not built (python -m lazzaro_amd._build --debug)")
    L = ctypes.CDLL(path)
    P = ctypes.c_void_p
    L.lzk_cc_hook.argtypes = [P, P, ctypes.c_long, P, ctypes.c_float, P, P, P]
    L.lzk_graph_debug_errors.restype = ctypes.c_int
    assert L.lzk_graph_debug_errors() == 0
    src = torch.tensor([0, -1, 2], dtype=torch.int32, device="cuda")
    dst = torch.tensor([1, 2, 0], dtype=torch.int32, device="cuda")
    parent = torch.arange(3, dtype=torch.int32, device="cuda")
    changed = torch.zeros(1, dtype=torch.int32, device="cuda")
    rc = L.lzk_cc_hook(src.data_ptr(), dst.data_ptr(), 3, None, 0.0, parent.data_ptr(), changed.data_ptr(),
                       _lib.stream_ptr(src.device))
    torch.cuda.synchronize()
    assert rc == 0 and L.lzk_graph_debug_errors() > 0
    assert L.lzk_graph_debug_errors() == 0  # read-and-clear


def test_store_ivfpq_tenant_gpu(tmp_path):
    import numpy as np

    from lazzaro_amd.core.vector_store import HBMStore
    st = HBMStore(db_dir=str(tmp_path), device="cuda", metric="cosine", index="ivfpq", nlist=256, nprobe=16,
                  pq_m=32, ivf_min_rows=50_000)
    rng = np.random.default_rng(0)
    c = rng.standard_normal((500, 256)).astype(np.float32)
    x = c[rng.integers(0, 500, 120_000)] + 0.5 * rng.standard_normal((120_000, 256)).astype(np.float32) / 16
    a = st._arena("big")
    a.add([f"m{i}" for i in range(len(x))], x)
    q = x[:64] + 0.01 * rng.standard_normal((64, 256)).astype(np.float32)
    got = st.search_nodes_batch(q, user_id="big", limit=5)
    assert a.ivf.idx is not None
    assert sum(g[0] == f"m{i}" for i, g in enumerate(got)) >= 60


@pytest.mark.parametrize("keep", ["fp8", "bf16", "int8"])
def test_ivfpq_fused_rerank_matches_library_path(monkeypatch, keep):
    """rerank_kernel (ivfpq.hip) == gather + dequantise + GEMM + sort."""
    from lazzaro_amd.index.ivfpq import IVFPQIndex
    g = torch.Generator(device="cuda").manual_seed(3)
    d = 256
    x = torch.nn.functional.normalize(torch.randn(60_000, d, device="cuda", generator=g), dim=1)
    idx = IVFPQIndex(d, nlist=64, m=32, device="cuda", keep_vectors=keep)
    idx.train(x[:20_000], iters=4, pq_iters=4)
    idx.add(x)
    q = torch.nn.functional.normalize(x[:300] + 0.2 * torch.randn(300, d, device="cuda", generator=g) / d ** 0.5,
                                      dim=1)
    s1, i1 = idx.search(q, 10, nprobe=8, rerank=200)
    monkeypatch.setattr(IVFPQIndex, "_rerank_gpu_ok", lambda self, k: False)
    s2, i2 = idx.search(q, 10, nprobe=8, rerank=200)
    torch.testing.assert_close(s1, s2, atol=1e-4, rtol=1e-4)
    assert (i1 == i2).float().mean() > 0.99


@pytest.mark.parametrize("N,nq", [(37, 300), (4096, 1000), (1000, 70001)])
def test_flat_top1_gpu(N, nq):
    """256x256 argmax kernel (k-means assign) vs an fp32 reference: partial row
    and query tiles, negative best scores, exact duplicate rows (tie -> the
    smaller row)."""
    from lazzaro_amd.ops.search import flat_top1
    g = torch.Generator().manual_seed(N + nq)
    D = 192
    X = torch.randn(N, D, generator=g).to(torch.bfloat16)
    X[N // 2] = X[N // 3]  # duplicate rows: equal scores, keep the smaller index
    Q = torch.randn(nq, D, generator=g).to(torch.bfloat16)
    Q[:5] = -X[:5]  # a few queries whose best score is small
    ref = Q.float() @ X.float().T
    s, r = flat_top1(X.to(DEV), Q.to(DEV))
    s, r = s.cpu(), r.cpu().long()
    assert bool((r >= 0).all()) and bool((r < N).all())
    best = ref.max(dim=1).values
    got = ref.gather(1, r[:, None])[:, 0]
    assert torch.allclose(s, got, atol=1e-3, rtol=1e-4)
    assert bool((got >= best - 1e-3).all())
    assert int((r == N // 2).sum()) == 0  # the duplicate's larger index never wins


def test_kmeans_assign_paths_agree_gpu(monkeypatch):
    import lazzaro_amd.index.kmeans as K
    g = torch.Generator().manual_seed(5)
    X = torch.nn.functional.normalize(torch.randn(20000, 128, generator=g), dim=1).to(torch.bfloat16).to(DEV)
    C = X[:300].contiguous()
    monkeypatch.setattr(K, "ASSIGN", "lane")
    la, sa = K.assign(X, C)
    monkeypatch.setattr(K, "ASSIGN", "top1")
    lb, sb = K.assign(X, C)
    assert torch.allclose(sa, sb, atol=1e-4)
    assert float((la == lb).float().mean()) > 0.999


def test_two_level_assign_gpu_matches_full():
    """assign_two_level on the GPU (per-topic fused argmax launches) agrees
    with the full 256x256 argmax assign on well-separated topics."""
    from lazzaro_amd.index.kmeans import assign, assign_two_level
    g = torch.Generator(device="cuda").manual_seed(5)
    d, T, per = 128, 16, 32
    tops = torch.nn.functional.normalize(torch.randn(T, d, device="cuda", generator=g), dim=1)
    fine = torch.nn.functional.normalize(tops.repeat_interleave(per, 0)
                                         + 0.15 * torch.randn(T * per, d, device="cuda", generator=g), dim=1)
    top_of = torch.arange(T, device="cuda").repeat_interleave(per)
    X = torch.nn.functional.normalize(fine[torch.randint(0, T * per, (200_000,), device="cuda", generator=g)]
                                      + 0.03 * torch.randn(200_000, d, device="cuda", generator=g), dim=1)
    b = lambda t: t.to(torch.bfloat16).contiguous()  # noqa: E731
    l_full, _ = assign(b(X), b(fine))
    l_two, _ = assign_two_level(b(X), b(fine), b(tops), top_of)
    assert (l_full.long() == l_two.long()).float().mean() > 0.995


def test_device_csr_matches_host_build():
    """K13: the visible-arc CSR built on the device (one shard: every arc
    visible both ways) equals the native host build (same per-source arc
    order, self-loops once)."""
    from lazzaro_amd.ops import tenant_ops as T
    from lazzaro_amd.store.colstore import _rt

    n, ne = 3000, 20000
    e = _rand_edges(n, ne, 7, DEV)
    e["src"][:50] = e["dst"][:50]  # self-loops
    e["meta"] = torch.zeros(ne, dtype=torch.int32, device=DEV)
    off, adj, eid = T.build_visible_csr(e, torch.zeros(n, dtype=torch.int32, device=DEV), n)
    ho, ha, he = _rt().build_csr(e["src"].cpu().numpy(), e["dst"].cpu().numpy(), n, True)
    assert torch.equal(off.cpu(), torch.from_numpy(ho))
    assert torch.equal(adj.cpu(), torch.from_numpy(ha).to(adj.dtype))
    assert torch.equal(eid.cpu(), torch.from_numpy(he).to(eid.dtype))


def test_grouped_two_level_assign_matches_group_loop():
    """flat_top1_grouped_kernel (one launch, rows read by index) equals the
    gather + flat_top1 per topic group, bit for bit: labels and scores,
    including topics with > 256 fine centroids (several centroid tiles) and
    a topic with none (full-search fallback); scores match an fp32 dot."""
    import lazzaro_amd.index.kmeans as KM

    g = torch.Generator(device="cpu").manual_seed(11)
    n, d, k, t = 150_000, 768, 1100, 24
    X = torch.nn.functional.normalize(torch.randn(n, d, generator=g), dim=1).to(torch.bfloat16).to(DEV)
    C = torch.nn.functional.normalize(torch.randn(k, d, generator=g), dim=1).to(torch.bfloat16).to(DEV)
    T = torch.nn.functional.normalize(torch.randn(t, d, generator=g), dim=1).to(torch.bfloat16).to(DEV)
    top_of = torch.randint(1, t, (k,), generator=g)
    top_of[:300] = 5  # one topic with 300+ fine centroids: two centroid tiles
    top_of[top_of == 0] = 1  # topic 0 has no fine centroid
    top_of = top_of.to(DEV)
    try:
        KM.GROUPED = True
        lg, sg = KM.assign_two_level(X, C, T, top_of)
        KM.GROUPED = False
        ll, sl = KM.assign_two_level(X, C, T, top_of)
    finally:
        KM.GROUPED = True
    assert torch.equal(lg, ll)
    assert torch.equal(sg, sl)
    ref = (X.float() * C[lg.long()].float()).sum(1)
    assert torch.allclose(sg, ref, atol=1e-3)


def test_farthest_first_kernel_matches_torch_gpu():
    """The fused farthest-first seeding (kmeans.hip ff_step_kernel, one
    launch per pick enqueued from C++) picks the same rows as the torch
    GEMV + max + argmin loop (on the host) for the same subsample."""
    import time

    from lazzaro_amd.index.kmeans import _farthest_first
    gen = torch.Generator(device=DEV).manual_seed(5)
    X = torch.randn(30_000, 256, device=DEV, generator=gen)
    X = (X / X.norm(dim=1, keepdim=True)).to(torch.bfloat16)
    c_dev = _farthest_first(X, 96, seed=3)
    c_ref = _farthest_first(X.cpu(), 96, seed=3)
    assert torch.equal(c_dev.cpu(), c_ref)
    # the tenant-scale shape: 4096 picks over a 65,536-row sample of 768-d rows
    Y = torch.randn(200_000, 768, device=DEV, generator=gen)
    Y = (Y / Y.norm(dim=1, keepdim=True)).to(torch.bfloat16)
    _farthest_first(Y, 64, seed=0)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    c = _farthest_first(Y, 4096, seed=0)
    torch.cuda.synchronize()
    ms = (time.perf_counter() - t0) * 1e3
    print(f"farthest_first 4096 x 65536 x 768: {ms:.1f} ms")
    assert c.shape == (4096, 768) and ms < 400


@pytest.mark.parametrize("thr", [None, 0.45])
def test_incremental_components_match_full_recompute_gpu(thr):
    """TenantGraph.cc_begin / _cc_labels: a random tenant graph (200k rows,
    400k edges -- the full GPU digest path) goes through a batch of segments
    that decay (with or without a prune threshold the decays cross), append
    new rows with edges into the graph, evict victims (their shard's edges
    go); at every point the incremental labels equal a full union-find over
    the current edges, label for label, and so do the digests."""
    import numpy as np

    from lazzaro_amd.engine.tenant_graph import TenantGraph
    from lazzaro_amd.ops import tenant_ops as T
    n, ne, D = 200_000, 400_000, 64
    gen = torch.Generator().manual_seed(9)
    g = TenantGraph(device=DEV, dim=D)
    shards = [g.shard_id(f"s{i}") for i in range(6)]
    X = torch.randn(n, D, generator=gen)
    X = X / X.norm(dim=1, keepdim=True)
    g.add_nodes([f"n{i}" for i in range(n)], [f"c{i}" for i in range(n)], X.to(DEV),
                shard=np.asarray([shards[i % 6] for i in range(n)], np.int32), stored=True)
    src = torch.randint(0, n, (ne,), generator=gen, dtype=torch.int32)
    dst = torch.randint(0, n, (ne,), generator=gen, dtype=torch.int32)
    w = 0.44 + 0.2 * torch.rand(ne, generator=gen)  # some edges cross 0.45 within the batch's decays
    g.append_edges(src.to(DEV), dst.to(DEV), w.to(DEV), g.shard[src.to(DEV).long()], g.etype("relates_to"))
    assert not g._digest_local(3, 1)
    B, keep = 12, 0.99
    victims = torch.randperm(n, generator=gen)[:3000].numpy()
    assert g.cc_begin(victims, thr, keep, B)
    rng = np.random.default_rng(4)
    for point in range(6):
        tok = g.segment_begin(1.0 - keep, thr, 2)
        m = 40  # new rows, each linked to 3 existing rows and to each other
        n_before = g.n
        Y = torch.randn(m, D, generator=gen)
        g.add_nodes([f"p{point}_{j}" for j in range(m)], ["x"] * m, (Y / Y.norm(dim=1, keepdim=True)).to(DEV),
                    shard=np.asarray([shards[j % 6] for j in range(m)], np.int32), stored=True)
        s_new = torch.arange(n_before, n_before + m, dtype=torch.int32).repeat(3)
        d_new = torch.as_tensor(rng.integers(0, n_before, 3 * m), dtype=torch.int32)
        s_new = torch.cat([s_new, torch.arange(n_before, n_before + m - 1, dtype=torch.int32)])
        d_new = torch.cat([d_new, torch.arange(n_before + 1, n_before + m, dtype=torch.int32)])
        g.append_edges(s_new.to(DEV), d_new.to(DEV), torch.full((s_new.numel(),), 0.7, device=DEV),
                       g.shard[s_new.to(DEV).long()], g.etype("relates_to"))
        vic = victims[point * 500:(point + 1) * 500].tolist()
        g.segment_end(tok, vic, unstore=True)
        inc = g._cc_labels()
        full = T.components(g.e["src"], g.e["dst"], g.n)
        assert torch.equal(inc, full.to(torch.int32)), point
        d_inc = g.component_digest(3, 0.3, 10)
        saved, g._cc = g._cc, None
        d_full = g.component_digest(3, 0.3, 10)
        g._cc = saved
        assert len(d_inc) == len(d_full) and all(np.array_equal(a, b) for a, b in zip(d_inc, d_full)), point
    g.cc_end()
