"""CPU tier of the graph ops on the tenant engine's columns (the GPU kernels
are checked against these references in tests/kernels/test_graph_kernels_gpu.py
and tests/kernels/test_tenant_engine_gpu.py)."""
import numpy as np
import torch

from lazzaro_amd.index.kmeans import kmeans
from lazzaro_amd.ops import graph_ops as G
from lazzaro_amd.ops import tenant_ops as T


def _edges(src, dst, w, shard=0):
    n = len(src)
    return {"src": torch.tensor(src, dtype=torch.int32), "dst": torch.tensor(dst, dtype=torch.int32),
            "w": torch.tensor(w, dtype=torch.float32), "co": torch.ones(n, dtype=torch.int32),
            "lu": torch.zeros(n, dtype=torch.float64), "meta": torch.full((n,), shard, dtype=torch.int32)}


def test_decay_prune_matches_reference_arithmetic():
    e = _edges([0, 1, 2], [1, 2, 0], [0.5, 0.9, 0.6])
    sal = torch.tensor([0.9, 0.2, 0.1], dtype=torch.float32)
    kind, sup = torch.ones(3, dtype=torch.uint8), torch.zeros(3, dtype=torch.uint8)
    out, pruned, _ = T.decay_prune(e, sal, kind, sup, 0.01, 0.5)
    assert pruned == 1  # chain weight 0.5 -> 0.495 < 0.5
    assert out["src"].tolist() == [1, 2]
    # salience 0.2 + (s - 0.2) * 0.99, floor 0.2 (memory_shard.py:64-77)
    assert abs(float(sal[0]) - 0.893) < 1e-6 and abs(float(sal[2]) - 0.2) < 1e-7


def test_components_union_find():
    lab = G.connected_components(torch.tensor([0, 2, 5], dtype=torch.int32),
                                 torch.tensor([1, 3, 4], dtype=torch.int32), 7)
    assert lab.tolist() == [0, 0, 2, 2, 4, 4, 6]


def test_chain_1500_no_recursion_error():
    n = 1500
    src = torch.arange(n - 1, dtype=torch.int32)
    lab = G.connected_components(src, src + 1, n)
    assert int(lab.max()) == 0


def test_importance_excludes_super_and_ghost_rows():
    sal = torch.tensor([0.9, 0.2, 0.5, 0.2])
    acc = torch.tensor([0, 10, 0, 0], dtype=torch.int32)
    last = torch.zeros(4, dtype=torch.float64)
    kind = torch.tensor([1, 1, 1, 1], dtype=torch.uint8)
    sup = torch.tensor([0, 0, 0, 1], dtype=torch.uint8)
    s = T.importance(sal, acc, last, kind, sup, now=0.0)
    assert torch.isinf(s[3])
    # 0.5 s + 0.3 min(1, acc/10) + 0.2 / (1 + days)  (memory_system.py:545-549)
    assert torch.argsort(s, stable=True)[:2].tolist() == [2, 1]


def test_pairs_and_centroids():
    X = torch.tensor([[1, 0], [1, 0], [0, 1], [0.6, 0.8]], dtype=torch.float32)
    p = G.pairs_above(X, 0.95)
    assert p.tolist() == [[0, 1]]
    c32, _, cnt = G.centroids(X, torch.tensor([0, 0, 1, -1], dtype=torch.int32), 2)
    assert cnt.tolist() == [2, 1] and torch.allclose(c32[1], torch.tensor([0.0, 1.0]))


def test_neighbor_boost_cpu():
    e = _edges([0, 0, 1], [1, 2, 3], [0.8, 0.2, 0.9])
    shard = torch.zeros(4, dtype=torch.int32)
    csr = T.build_visible_csr(e, shard, 4)
    sal = torch.tensor([0.5, 0.5, 0.5, 0.99])
    last = torch.zeros(4, dtype=torch.float64)
    kind, sup = torch.ones(4, dtype=torch.uint8), torch.zeros(4, dtype=torch.uint8)
    dirty = torch.zeros(4, dtype=torch.uint8)
    n = T.neighbor_boost(csr, e["w"], torch.tensor([0]), kind, sup, sal, last, dirty, 5.0, T.BoostState())
    assert n == 1 and abs(float(sal[1]) - 0.52) < 1e-6 and float(sal[2]) == 0.5 and float(last[1]) == 5.0


def test_touch_counts_repeated_rows_per_occurrence():
    """update_access once per listed occurrence (buffer_graph.py:79-85)."""
    from lazzaro_amd.engine.tenant_graph import TenantGraph
    g = TenantGraph(device="cpu")
    g.add_nodes(["a", "b"], ["x", "y"], torch.eye(2, 8), shard=g.shard_id("work"), sal=0.5)
    g.touch([0, 1, 0], now=10.0)
    assert g.acc.tolist()[:2] == [2, 1]
    assert abs(float(g.sal[0]) - 0.6) < 1e-6 and abs(float(g.sal[1]) - 0.55) < 1e-6


def test_kmeans_cpu_separates_clusters():
    torch.manual_seed(1)
    centers = torch.nn.functional.normalize(torch.randn(4, 16), dim=1)
    X = torch.cat([torch.nn.functional.normalize(c + 0.05 * torch.randn(100, 16), dim=1) for c in centers])
    c32, _, lab = kmeans(X, 4, iters=8, seed=3)
    assert len(set(lab.tolist())) == 4
    for j in range(4):
        assert len(set(lab[j * 100:(j + 1) * 100].tolist())) == 1


def test_visible_csr_matches_native_build_for_one_shard():
    """With every node in one shard, the visible-arc CSR is the undirected CSR
    the native host build gives (arc order per source, self-loops once)."""
    from lazzaro_amd.store.colstore import _rt

    g = torch.Generator().manual_seed(3)
    n, ne = 500, 4000
    src = torch.randint(0, n, (ne,), generator=g, dtype=torch.int32)
    dst = torch.randint(0, n, (ne,), generator=g, dtype=torch.int32)
    src[:20] = dst[:20]
    e = {"src": src, "dst": dst, "meta": torch.zeros(ne, dtype=torch.int32)}
    off, adj, eid = T.build_visible_csr(e, torch.zeros(n, dtype=torch.int32), n)
    ho, ha, he = _rt().build_csr(src.numpy(), dst.numpy(), n, True)
    assert torch.equal(off, torch.from_numpy(ho))
    assert torch.equal(adj, torch.from_numpy(ha).to(adj.dtype))
    assert torch.equal(eid, torch.from_numpy(he).to(eid.dtype))
