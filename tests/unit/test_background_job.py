"""The worker-thread job behind TenantGraph.cluster_pass(background=True)
(engine/tenant_graph.py _BackgroundJob) and the hierarchy's join semantics,
on the CPU: a GPU tenant's background pass is covered by
tests/kernels/test_tenant_engine_gpu.py::test_consolidate_stream_matches_batches_gpu[kmeans]."""
import threading

import pytest
import torch

from lazzaro_amd.engine.tenant_graph import TenantGraph, _BackgroundJob


def test_background_job_returns_and_reraises():
    ev = threading.Event()

    def ok():
        ev.wait(5)
        return 42
    j = _BackgroundJob(ok)
    ev.set()
    assert j.result() == 42

    def bad():
        raise ValueError("boom")
    with pytest.raises(ValueError, match="boom"):
        _BackgroundJob(bad).result()


def test_hier_joins_a_pending_job_once():
    g = TenantGraph(device="cpu", dim=4)
    assert g.hier is None and not g.has_hier()
    gate = threading.Event()
    calls = []

    class _Done:  # stands in for the side stream's completion event
        pass

    class _Stream:
        def wait_event(self, ev):
            calls.append(ev)

    out = {"fine_c": torch.zeros(2, 4), "n": 0}

    def work():
        gate.wait(5)
        return out, _Done(), _Stream()
    g._hier_job = _BackgroundJob(work)
    assert g.has_hier()  # pending: has_hier does not wait
    seen = []
    readers = [threading.Thread(target=lambda: seen.append(g.hier)) for _ in range(4)]
    for t in readers:
        t.start()
    gate.set()
    for t in readers:
        t.join(5)
    assert len(seen) == 4 and all(h is out for h in seen)  # every reader sees the published pass
    assert len(calls) == 1  # joined (and the graph stream made to wait) exactly once
    assert g._hier_job is None and g.hier is out


def test_cpu_cluster_pass_ignores_background():
    g = TenantGraph(device="cpu", dim=8)
    x = torch.randn(64, 8, generator=torch.Generator().manual_seed(0))
    g.add_nodes([f"n{i}" for i in range(64)], [""] * 64, x, shard=g.shard_id("s"))
    r = g.cluster_pass(n_fine=4, n_top=2, iters=1, background=True)
    assert "background" not in r and g._hier_job is None  # on the CPU the pass runs in line
    assert g.hier is not None and g.hier["fine_c"].shape[0] == 4
