"""The consolidation-at-scale benchmark (bench/bench_consolidate.py: one
MemorySystem tenant per rank, MemorySystem.consolidate_batch) on CPU with
gloo, and distributed k-means (C4 all-reduce) agreement across ranks."""
import os
import sys

import pytest

from tests.distributed.test_dist_gloo import spawn

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def _bench(comm):
    import torch
    sys.path.insert(0, os.path.join(ROOT, "bench"))
    sys.path.insert(0, ROOT)
    import bench_consolidate as B
    r = B.run(comm, torch.device("cpu"), nodes=3000, convs=8, facts=4, steps=3, warmup=1, encoder=None, dim=32,
              dup_rate=0.3, cluster_every=1, n_fine=16, n_top=4, cluster_iters=2, init_edges=2000)
    ps = r["per_step_rank0"]
    return (r["turns_per_s"] > 0 and ps["dup"] > 0 and ps["inserted"] > 0 and ps["evicted"] > 0
            and ps["linked"] > 0 and ps["pruned"] < ps["linked"] + 2000 and r["nodes_rank0"] == 3000
            and r["edges_rank0"] > 0)


def _kmeans_agree(comm):
    """Distributed k-means: identical centroids on every rank; every masked-in
    row labelled."""
    import torch
    from lazzaro_amd.index.kmeans import kmeans
    g = torch.Generator().manual_seed(5 + comm.rank)
    X = torch.randn(1500, 32, generator=g)
    X = X / X.norm(dim=1, keepdim=True)
    mask = torch.rand(1500, generator=g) > 0.1
    c32, _, lab = kmeans(X, 16, iters=3, comm=comm, mask=mask)
    ref = c32.clone()
    comm.broadcast(ref, src=0)
    return torch.allclose(c32, ref) and bool((lab[mask] >= 0).all()) and bool((lab[~mask] == -1).all())


@pytest.mark.parametrize("world", [1, 2])
def test_consolidation_pipeline(world):
    if world == 1:
        from lazzaro_amd.parallel import Communicator
        assert _bench(Communicator.local())
    else:
        assert all(spawn(world, _bench).values())


@pytest.mark.parametrize("world", [1, 2])
def test_distributed_kmeans(world):
    if world == 1:
        from lazzaro_amd.parallel import Communicator
        assert _kmeans_agree(Communicator.local())
    else:
        assert all(spawn(world, _kmeans_agree).values())


def _bench_rank0(comm):
    import json
    import torch
    sys.path.insert(0, os.path.join(ROOT, "bench"))
    sys.path.insert(0, ROOT)
    import bench_consolidate as B
    r = B.run(comm, torch.device("cpu"), nodes=1500, convs=4, facts=4, steps=2, warmup=1, encoder=None, dim=32,
              dup_rate=0.3, cluster_every=1, n_fine=8, n_top=2, cluster_iters=1, init_edges=500)
    return json.dumps({k: r[k] for k in ("per_step_rank0", "scan_facts_x_rows_per_rank_step", "nodes_rank0",
                                         "edges_rank0")})


def test_consolidation_weak_scales():
    """Round-1 verdict #4: per-rank scan work and rank 0's dedupe / link /
    evict decisions are the same at 1 and 8 ranks (tenant-DP: a rank only
    ever scans its own tenant's rows)."""
    import json
    from lazzaro_amd.parallel import Communicator
    one = json.loads(_bench_rank0(Communicator.local()))
    eight = spawn(8, _bench_rank0)
    assert json.loads(eight[0]) == one
    # every rank's work is its own tenant's (same size up to its dedupe rate)
    works = [json.loads(v)["scan_facts_x_rows_per_rank_step"] for v in eight.values()]
    assert max(works) / min(works) < 1.05
