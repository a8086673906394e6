"""CPU tier of the graph ops + DeviceGraph semantics (the GPU kernels are
checked against these references in tests/kernels/test_graph_kernels_gpu.py)."""
import numpy as np
import torch

from lazzaro_amd.index.device_graph import DeviceGraph
from lazzaro_amd.index.kmeans import kmeans
from lazzaro_amd.ops import graph_ops as G


def _edges(src, dst, w):
    n = len(src)
    return {"src": torch.tensor(src, dtype=torch.int32), "dst": torch.tensor(dst, dtype=torch.int32),
            "w": torch.tensor(w, dtype=torch.float32), "co": torch.ones(n, dtype=torch.int32),
            "lu": torch.zeros(n, dtype=torch.float64)}


def test_decay_prune_matches_reference_arithmetic():
    e = _edges([0, 1, 2], [1, 2, 0], [0.5, 0.9, 0.6])
    sal = torch.tensor([0.9, 0.2, 0.1], dtype=torch.float32)
    out, pruned = G.decay_prune(e, sal, torch.ones(3, dtype=torch.uint8), 0.01, 0.5)
    assert pruned == 1  # chain weight 0.5 -> 0.495 < 0.5
    assert out["src"].tolist() == [1, 2]
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


def test_importance_and_select():
    sal = torch.tensor([0.9, 0.2, 0.5, 0.2])
    acc = torch.tensor([0, 10, 0, 0], dtype=torch.int32)
    last = torch.zeros(4, dtype=torch.float64)
    prot = torch.tensor([0, 0, 0, 1], dtype=torch.uint8)
    s = G.importance(sal, acc, last, None, prot, now=0.0)
    assert torch.isinf(s[3])
    assert G.select_lowest(s, 2).tolist() == [2, 1]


def test_pairs_and_centroids():
    X = torch.tensor([[1, 0], [1, 0], [0, 1], [0.6, 0.8]], dtype=torch.float32)
    p = G.pairs_above(X, 0.95)
    assert p.tolist() == [[0, 1]]
    c32, _, cnt = G.centroids(X, torch.tensor([0, 0, 1, -1], dtype=torch.int32), 2)
    assert cnt.tolist() == [2, 1] and torch.allclose(c32[1], torch.tensor([0.0, 1.0]))


def test_neighbor_boost_cpu():
    from lazzaro_amd.store.colstore import _rt
    off, adj, eid = _rt().build_csr(np.array([0, 0, 1], np.int32), np.array([1, 2, 3], np.int32), 4, True)
    off, adj, eid = torch.from_numpy(off), torch.from_numpy(adj), torch.from_numpy(eid)
    w = torch.tensor([0.8, 0.2, 0.9])
    sal = torch.tensor([0.5, 0.5, 0.5, 0.99])
    last = torch.zeros(4, dtype=torch.float64)
    n = G.neighbor_boost(off, adj, eid, w, torch.tensor([0]), sal, last, now=5.0)
    assert n == 1 and abs(float(sal[1]) - 0.52) < 1e-6 and float(sal[2]) == 0.5 and float(last[1]) == 5.0


def test_device_graph_ingest_dedupe_link_cpu():
    torch.manual_seed(0)
    g = DeviceGraph(dim=32, device="cpu")
    base = torch.nn.functional.normalize(torch.randn(50, 32), dim=1)
    g.add_nodes(base, torch.randint(0, 4, (50,)), torch.full((50,), 0.5))
    # near-duplicate of row 3 + a fresh fact close to row 7
    q = torch.stack([base[3], torch.nn.functional.normalize(base[7] + 0.3 * torch.randn(32), dim=0)])
    out = g.ingest(q, torch.tensor([int(g.shard[3]), int(g.shard[7])]), torch.tensor([0.9, 0.6]))
    assert out["deduped"] == 1 and out["inserted"] == 1
    assert abs(float(g.sal[3]) - 0.9) < 1e-6 and int(g.acc[3]) == 1
    assert out["linked"] >= 1 and g.num_edges == out["linked"]
    assert 7 in g.edges["dst"].tolist()
    pruned = g.decay_prune(0.01, 0.5, conversations=200)
    assert g.num_edges == 0 and pruned == out["linked"]
    assert g.enforce_limit(10) == 41 and g.num_alive() == 10


def test_kmeans_cpu_separates_clusters():
    torch.manual_seed(1)
    centers = torch.nn.functional.normalize(torch.randn(4, 16), dim=1)
    X = torch.cat([torch.nn.functional.normalize(c + 0.05 * torch.randn(100, 16), dim=1) for c in centers])
    c32, _, lab = kmeans(X, 4, iters=8, seed=3)
    assert len(set(lab.tolist())) == 4
    for j in range(4):
        assert len(set(lab[j * 100:(j + 1) * 100].tolist())) == 1


def test_ingest_fixed_links_and_tombstones():
    """Sync-free batch ingest: duplicate rows are tombstoned, untaken links get
    weight -1 (pruned by the next compaction), chains skip dead facts."""
    import torch
    from lazzaro_amd.index.device_graph import DeviceGraph
    g = DeviceGraph(4, device="cpu", capacity=16)
    g.add_nodes(torch.eye(4), torch.tensor([0, 0, 1, 1]), torch.full((4,), 0.5), now=0.0)
    q = torch.nn.functional.normalize(torch.tensor([[1.0, 0.1, 0, 0], [0, 1.0, 0, 0], [1.0, 0.05, 0, 0],
                                                    [0, 0, 1.0, 0.2]]), dim=1)
    shard = torch.tensor([0, 0, 0, 1])
    dead = torch.tensor([False, True, False, False])
    # (scores, rows) per fact: in-shard top-2 and global top-2
    sw = torch.tensor([[0.99, 0.1], [0.9, 0.2], [0.98, 0.05], [0.97, 0.4]])
    rw = torch.tensor([[0, 1], [1, 0], [0, 1], [2, 3]])
    sg = torch.tensor([[0.99, 0.6], [0.9, 0.2], [0.98, 0.45], [0.97, 0.7]])
    rg = torch.tensor([[0, 2], [1, 0], [0, 3], [2, 0]])
    out = g.ingest_fixed(q, shard, torch.full((4,), 0.7), dead, (sw, rw), global_hits=(sg, rg), now=1.0,
                         link_k=2)
    assert int(out["inserted"]) == 3 and int(out["deduped"]) == 1
    assert g.n == 8 and g.alive[4:8].tolist() == [1, 0, 1, 1] and g.bias[5].item() == float("-inf")
    e = g.edges
    live = e["w"] > -1
    got = sorted(zip(e["src"][live].tolist(), e["dst"][live].tolist(), [round(w, 3) for w in e["w"][live].tolist()]))
    want = sorted([(4, 0, round(0.99 * 0.8, 3)), (6, 0, round(0.98 * 0.8, 3)), (7, 2, round(0.97 * 0.8, 3)),
                   (4, 2, round(0.6 * 0.8, 3)), (7, 0, round(0.7 * 0.8, 3)),  # global hits not linked in-shard
                   (4, 6, 0.5)])                 # chain: fact 0 -> fact 2 (fact 1 is a duplicate)
    assert got == want, got
    assert int(out["linked"]) == len(want)


def test_csr_undirected_tensor_build_matches_native():
    """The tensor-op CSR build DeviceGraph uses on the GPU equals the native
    host build (arc order, self-loops once), run here on CPU tensors."""
    import torch

    from lazzaro_amd.index.device_graph import csr_undirected
    from lazzaro_amd.store.colstore import _rt

    g = torch.Generator().manual_seed(3)
    n, ne = 500, 4000
    src = torch.randint(0, n, (ne,), generator=g, dtype=torch.int32)
    dst = torch.randint(0, n, (ne,), generator=g, dtype=torch.int32)
    src[:20] = dst[:20]
    off, adj, eid = csr_undirected(src, dst, n)
    ho, ha, he = _rt().build_csr(src.numpy(), dst.numpy(), n, True)
    assert torch.equal(off, torch.from_numpy(ho))
    assert torch.equal(adj, torch.from_numpy(ha))
    assert torch.equal(eid, torch.from_numpy(he))
