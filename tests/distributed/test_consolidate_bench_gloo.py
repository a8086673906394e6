"""The consolidation-at-scale pipeline (bench/bench_consolidate.py) on CPU with
gloo: all-to-all routing, global dedupe via all-gather search, local ingest."""
import os
import sys

import pytest

from tests.distributed.test_dist_gloo import spawn

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def _bench(comm):
    import torch
    sys.path.insert(0, os.path.join(ROOT, "bench"))
    import bench_consolidate as B
    r = B.run(comm, torch.device("cpu"), nodes=3000, convs=4, facts=4, steps=2, warmup=1, encoder=None, dim=32,
              dup_rate=0.5, cluster_every=1, n_fine=16, n_top=4, cluster_iters=2)
    ps = r["per_step_rank0"]
    hc = r["hierarchical_clustering"]
    return (r["turns_per_s"] > 0 and ps["dup"] > 0 and ps["inserted"] > 0 and ps["routed"] > 0
            and hc["fine_clusters_used"] > 1)


def _cluster_agree(comm):
    """Distributed k-means leaves identical centroids on every rank, and every
    live row carries a fine and a top-level super-node label."""
    import torch
    sys.path.insert(0, os.path.join(ROOT, "bench"))
    import bench_consolidate as B
    buf = B.ShardedBuffer(comm, 32, 2000, torch.device("cpu"), seed=3)
    buf.cluster(16, 4, 3)
    c = buf.fine.clone()
    ref = c.clone()
    comm.broadcast(ref, src=0)
    n = buf.g.n
    alive = buf.g.alive[:n] > 0
    return (torch.allclose(c, ref) and bool((buf.super_fine[alive] >= 0).all())
            and bool((buf.super_top[alive] < 4).all()) and int(buf.super_top[alive].unique().numel()) > 1)


@pytest.mark.parametrize("world", [1, 2])
def test_consolidation_pipeline(world):
    if world == 1:
        import torch
        from lazzaro_amd.parallel import Communicator
        assert _bench(Communicator.local())
    else:
        assert all(spawn(world, _bench).values())


@pytest.mark.parametrize("world", [1, 2])
def test_hierarchical_clustering(world):
    if world == 1:
        from lazzaro_amd.parallel import Communicator
        assert _cluster_agree(Communicator.local())
    else:
        assert all(spawn(world, _cluster_agree).values())
