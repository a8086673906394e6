"""Row-sharded tenant on the GPU: 2 ranks (gloo for the collectives, both on
cuda:0) consolidate a 100k-row buffer whose per-rank scans take the fused
MFMA dual-scan kernel path, and end in exactly the state of a single-process
GPU ``MemorySystem`` on the union (nodes, saliences, edges, eviction victims,
per-batch counts, component digest, search results). The CPU equivalence at
1-3 ranks is tests/distributed/test_sharded_memory_gloo.py."""
import functools

import pytest
import torch

from tests.distributed.test_dist_gloo import spawn
from tests.distributed.test_sharded_memory_gloo import _sharded, check_equivalent

pytestmark = pytest.mark.gpu

GPU = {"rows": 100_000, "dim": 128, "limit": 100_050, "steps": 3, "convs": 48, "device": "cuda"}


@pytest.mark.skipif(not torch.cuda.is_available(), reason="needs a GPU")
def test_sharded_tenant_gpu_matches_single_process():
    out = spawn(2, functools.partial(_sharded, cfg=GPU))
    check_equivalent(out, 2, GPU["limit"])


@pytest.mark.skipif(not torch.cuda.is_available(), reason="needs a GPU")
def test_sharded_tenant_gpu_reference_hierarchy():
    """The reference cadence with the reference's per-shard mean super-nodes
    (collective member lists / means, super-node rows held by the rank with
    most children) on the GPU path: the single process's state, super-nodes
    and parents included."""
    cfg = dict(GPU, steps=2, convs=24, cadence="conversation", hier=True, tight=True, sthr=20)
    out = spawn(2, functools.partial(_sharded, cfg=cfg))
    check_equivalent(out, 2, cfg["limit"])
    nodes = out[0]["nodes"]
    assert any(v[4] is not None for v in nodes.values())


@pytest.mark.skipif(not torch.cuda.is_available(), reason="needs a GPU")
def test_sharded_tenant_gpu_one_rank_row_digest():
    """One GPU rank: component_digest runs the single-graph digest kernels on
    the local rows (_digest_world1); at every run_consolidation point it
    equals the replicated-edge digest, and the run is the single process's."""
    cfg = dict(GPU, steps=2, convs=24, cadence="conversation", digest_check=True)
    out = spawn(1, functools.partial(_sharded, cfg=cfg))
    check_equivalent(out, 1, cfg["limit"])
    assert out[0]["contents"]


@pytest.mark.skipif(not torch.cuda.is_available(), reason="needs a GPU")
def test_sharded_tenant_gpu_one_rank_native_vs_segments():
    """One GPU rank with and without the native segment applier: both end in
    the single process's state (nodes, edges, counts, digest, profile)."""
    for native in (True, False):
        cfg = dict(GPU, steps=3, convs=32, cadence="conversation", native_w1=native)
        out = spawn(1, functools.partial(_sharded, cfg=cfg))
        check_equivalent(out, 1, cfg["limit"])
        assert (out[0]["native"] > 0) == native, out[0]["native"]


@pytest.mark.skipif(not torch.cuda.is_available(), reason="needs a GPU")
def test_sharded_tenant_gpu_one_rank_native_persistent_graph():
    """One GPU rank, a graph that keeps its edges (prune_threshold 0, 20k
    seeded links): the native applier with the single tenant's incremental
    components (TenantGraph.cc_begin) ends in the single process's state, as
    the per-segment path does."""
    for native in (True, False):
        cfg = dict(GPU, steps=3, convs=32, cadence="conversation", native_w1=native, prune_thr=0.0,
                   seed_edges=20000)
        out = spawn(1, functools.partial(_sharded, cfg=cfg))
        check_equivalent(out, 1, cfg["limit"])
        assert (out[0]["native"] > 0) == native, out[0]["native"]


@pytest.mark.skipif(not torch.cuda.is_available(), reason="needs a GPU")
@pytest.mark.parametrize("prune_thr", [0.5, 0.0])
def test_sharded_tenant_gpu_incremental_digest(prune_thr):
    """Two GPU ranks, the incremental digest (stable base replicated and
    labelled once per batch by uf_union_sel, the volatile edges unioned on
    top, digest.hip stats): every point equals the full replicated digest and
    the run is the single process's -- decay-prune and persistent graph."""
    cfg = dict(GPU, steps=3, convs=32, cadence="conversation", dcc_min=0, dcc_check=True, prune_thr=prune_thr)
    out = spawn(2, functools.partial(_sharded, cfg=cfg))
    check_equivalent(out, 2, cfg["limit"])
    d = [out[r]["dcc"] for r in range(2)]
    assert all(x[0] > 0 for x in d), d
    if prune_thr == 0.0:  # (at 0.5 the batch's links all sit below the decayed threshold: an empty base)
        assert max(x[1] for x in d) > 0, d


@pytest.mark.skipif(not torch.cuda.is_available(), reason="needs a GPU")
@pytest.mark.parametrize("world", [1, 2])
def test_sharded_tenant_gpu_consolidate_stream(world):
    """ShardedMemorySystem.consolidate_stream on the GPU: each batch after the
    first is gathered and scanned on a side stream under the previous
    batch's apply (prefetched lists completed against the rows it left) --
    the single process's state, as the per-batch calls."""
    cfg = dict(GPU, steps=3, convs=48, cadence="conversation", stream=True)
    out = spawn(world, functools.partial(_sharded, cfg=cfg))
    check_equivalent(out, world, cfg["limit"])
    assert all(out[r]["pf_used"] == 2 for r in range(world))  # batches 2 and 3 came from the prefetch
    # one rank: the batches go through the native segment applier (csrc/kernels/apply.hip)
    assert (out[0]["native"] > 0) == (world == 1), out[0]["native"]


@pytest.mark.skipif(not torch.cuda.is_available(), reason="needs a GPU")
def test_num_rows_kernel_matches_searchsorted():
    """tenant.hip num_rows_kernel (the row-sharded tenant's number -> row
    lookup): base-then-delta binary search and the held-live filter against
    the torch searchsorted formulation, with absent numbers, a base/delta tie
    and an empty delta."""
    from lazzaro_amd.ops import tenant_ops as T
    dev = torch.device("cuda")
    g = torch.Generator().manual_seed(5)
    nb, nd = 5000, 300
    nums = torch.randperm(50_000, generator=g)[: nb + nd] * 3 + 1
    bk, bo = torch.sort(nums[:nb])
    bo = bo.clone()
    dk, do = torch.sort(nums[nb:])
    do = do + nb
    dk = torch.cat([dk, bk[:1]])  # a number in both: the base wins
    do = torch.cat([do, torch.tensor([nb + nd])])
    dk, o = torch.sort(dk)
    do = do[o]
    holder = torch.randint(0, 3, (nb + nd + 1,), generator=g)
    kind = torch.randint(0, 3, (nb + nd + 1,), generator=g).to(torch.uint8)
    q = torch.cat([nums[torch.randint(0, nb + nd, (4000,), generator=g)], torch.tensor([0, 2, 150_001, bk[0].item()])])

    def ref(q, held, empty_delta):
        out = torch.full_like(q, -1)
        pairs = [(bk, bo)] if empty_delta else [(dk, do), (bk, bo)]
        for ks, oo in pairs:
            pos = torch.searchsorted(ks, q).clamp_max(ks.numel() - 1)
            out = torch.where(ks[pos] == q, oo[pos], out)
        if held >= 0:
            rc = out.clamp_min(0)
            out = torch.where((out >= 0) & (holder[rc] == held) & (kind[rc] == 1), out, torch.full_like(out, -1))
        return out

    for empty_delta in (False, True):
        d_k = dk[:0] if empty_delta else dk
        d_o = do[:0] if empty_delta else do
        for held in (-1, 1):
            got = T.num_rows(q.to(dev) - 1, 1, bk.to(dev), bo.to(dev), d_k.to(dev), d_o.to(dev), holder.to(dev),
                             kind.to(dev), held)
            assert torch.equal(got.cpu(), ref(q, held, empty_delta))


@pytest.mark.skipif(not torch.cuda.is_available(), reason="needs a GPU")
def test_row_centroid_cos_kernel():
    """tenant.hip row_cent_cos_kernel (the cone radii of the row-sharded
    scan pruning) against the fp32 torch formula, padded row stride, rows
    without a vector."""
    from lazzaro_amd.ops import tenant_ops as T
    dev = torch.device("cuda")
    g = torch.Generator(device=dev).manual_seed(3)
    n, D, Dp, K = 5000, 760, 768, 64
    X = torch.zeros((n, Dp), device=dev)
    X[:, :D] = torch.randn((n, D), device=dev, generator=g)
    X[7] = 0.0
    sqn = (X * X).sum(1)
    C = torch.nn.functional.normalize(torch.randn((K, D), device=dev, generator=g), dim=1)
    rows = torch.randperm(n, device=dev, generator=g)[:3000]
    lab = torch.randint(0, K, (3000,), device=dev, generator=g)
    got = T.row_centroid_cos(X, D, sqn, rows, lab, C)
    nrm = sqn[rows].sqrt()
    ref = (X[rows, :D] * C[lab]).sum(1) / torch.where(nrm > 0, nrm, torch.ones_like(nrm))
    ref = torch.where(nrm > 0, ref, torch.full_like(ref, -1.0))
    assert torch.allclose(got, ref, atol=2e-6, rtol=0)
    assert float(got[(rows == 7).nonzero().flatten()].sum() if bool((rows == 7).any()) else -1.0) == -1.0
