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
              dup_rate=0.5)
    ps = r["per_step_rank0"]
    return r["turns_per_s"] > 0 and ps["dup"] > 0 and ps["inserted"] > 0 and ps["routed"] > 0


@pytest.mark.parametrize("world", [1, 2])
def test_consolidation_pipeline(world):
    if world == 1:
        import torch
        from lazzaro_amd.parallel import Communicator
        assert _bench(Communicator.local())
    else:
        assert all(spawn(world, _bench).values())
