"""Deferred-prune consolidation segments (TenantGraph.segment_begin /
segment_end, csrc/kernels/tenant.hip tg_flag_remove_kernel with ``prev``
flags) on an MI355X == the CPU's sequential decay + prune, append, remove
(reference memory_shard.py:64-84, memory_system.py:558-569): same edges in
the same order, same node state, same store deletions, same pruned counts,
over several segments (appends into the spare tail of compacted buffers)."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

from lazzaro_amd.engine.tenant_graph import TenantGraph  # noqa: E402


def _graph(dev, n, ne, seed):
    g = TenantGraph(device=dev)
    gen = torch.Generator().manual_seed(seed)
    codes = [g.shard_id(f"s{i}") for i in range(5)]
    sh = torch.tensor(codes)[torch.randint(0, 5, (n,), generator=gen)].int()
    X = torch.randn(n, 32, generator=gen)
    g.add_nodes([f"n{i}" for i in range(n)], [""] * n, X, shard=sh.numpy(), sal=torch.rand(n, generator=gen),
                now=1000.0, stored=True)
    src = torch.randint(0, n, (ne,), generator=gen)
    dst = torch.randint(0, n, (ne,), generator=gen)
    w = torch.rand(ne, generator=gen) * 0.6 + 0.4
    g.append_edges(src, dst, w, sh[src], g.etype("relates_to"), now=1000.0)
    g.take_dirty_edges()  # edges now "stored": their removal must be queued for the store
    g.take_deleted()
    return g


@pytest.mark.parametrize("thr", [0.45, None])
def test_segments_match_cpu_sequence(thr):
    n, ne = 3000, 20000
    gc, gg = _graph("cpu", n, ne, 1), _graph("cuda", n, ne, 1)
    rng = np.random.default_rng(2)
    for step in range(4):
        vic = sorted(set(rng.integers(0, n, 40).tolist()))
        m = 300
        s = torch.from_numpy(rng.integers(0, n, m))
        d = torch.from_numpy(rng.integers(0, n, m))
        w = torch.from_numpy(rng.random(m).astype(np.float32))
        out = []
        for g in (gc, gg):
            tok = g.segment_begin(0.01, thr, 3)
            g.append_edges(s, d, w, g.shard[: g.n].cpu()[s].to(g.device), g.etype("relates_to"), now=2000.0 + step)
            out.append(g.segment_end(tok, vic, unstore=True))
        assert out[0] == out[1], (step, out)
        for k in gc.e:
            assert torch.equal(gc.e[k], gg.e[k].cpu()), (step, k)
        for k in ("sal", "kind", "stored"):
            assert torch.equal(getattr(gc, k)[: gc.n], getattr(gg, k)[: gg.n].cpu()), (step, k)
        assert gc.shard_count == gg.shard_count and gc.n_super == gg.n_super
        assert list(gc.deleted_ids) == list(gg.deleted_ids)
        assert set(gc.deleted_edges) == set(gg.deleted_edges) and len(gc.deleted_edges) > 0
    if thr is not None:
        assert gg.num_edges < ne  # the prune took edges


@pytest.mark.parametrize("n", [1, 1000, 8192, 78_125, 100_007])
def test_scan_blocks_matches_cumsum(n):
    """graph.hip scan_kernel: in-place exclusive prefix + total."""
    from lazzaro_amd.ops import _lib
    from lazzaro_amd.ops import tenant_ops as T
    c = torch.randint(0, 257, (n,), generator=torch.Generator().manual_seed(n), dtype=torch.int32)
    d = c.cuda()
    tot = torch.zeros(1, dtype=torch.int32, device="cuda")
    _lib.check(_lib.lib().lzk_scan_blocks(d.data_ptr(), n, tot.data_ptr(), T._st(d)), "scan")
    want = torch.cumsum(c.long(), 0) - c.long()
    assert torch.equal(d.cpu().long(), want) and int(tot) == int(c.long().sum())


@pytest.mark.parametrize("n", [1, 31, 32, 33, 1000, 10_000_001])
def test_pack_bits(n):
    from lazzaro_amd.ops import tenant_ops as T
    f = (torch.rand(n, generator=torch.Generator().manual_seed(n)) < 0.3).to(torch.uint8)
    b = T._bits(f.cuda()).cpu().numpy().view(np.uint32)
    got = np.unpackbits(b.view(np.uint8), bitorder="little")[:n]
    assert np.array_equal(got, f.numpy())
