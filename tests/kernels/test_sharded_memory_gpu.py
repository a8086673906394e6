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
