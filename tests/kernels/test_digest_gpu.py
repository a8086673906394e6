"""digest.hip (sort-free component digest) against the sort + segmented-scan
formulation on the same device graph: a giant component, thousands of small
ones with more and fewer than ``take`` candidates, ghosts, super-nodes, four
shards and mean weights on both sides of the threshold."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


def _graph(n, ne_giant, n_small, seed):
    from lazzaro_amd.engine.tenant_graph import TenantGraph
    rng = np.random.default_rng(seed)
    g = TenantGraph(device="cuda", dim=8)
    codes = [g.shard_id(f"s{i}") for i in range(4)]
    g.add_nodes([f"node_{i}" for i in range(n)], [f"c{i}" for i in range(n)],
                rng.standard_normal((n, 8)).astype(np.float32).tolist(),
                shard=[codes[int(c)] for c in rng.integers(0, 4, n)],
                sup=(rng.random(n) < 0.02).astype(np.int64).tolist())
    # giant: random edges over the first half; small: chains of 2..30 rows in the rest
    half = n // 2
    src = [rng.integers(0, half, ne_giant)]
    dst = [rng.integers(0, half, ne_giant)]
    w = [rng.uniform(0.1, 1.0, ne_giant)]
    perm = rng.permutation(np.arange(half, n))
    at = 0
    for _ in range(n_small):
        k = int(rng.integers(2, 30))
        if at + k > perm.size:
            break
        m = perm[at:at + k]
        at += k
        src.append(m[:-1])
        dst.append(m[1:])
        w.append(np.full(k - 1, rng.choice([0.2, 0.29, 0.31, 0.6]), dtype=np.float64))
    s = torch.as_tensor(np.concatenate(src), dtype=torch.int32)
    d = torch.as_tensor(np.concatenate(dst), dtype=torch.int32)
    ww = torch.as_tensor(np.concatenate(w), dtype=torch.float32)
    meta = torch.as_tensor(np.full(s.numel(), codes[0]), dtype=torch.int32)
    g.append_edges(s.cuda(), d.cuda(), ww.cuda(), meta.cuda())
    g.remove_nodes(rng.choice(n, n // 50, replace=False).tolist())  # ghosts
    return g


@pytest.mark.parametrize("window", [1 << 16, 128])
@pytest.mark.parametrize("n,ne,n_small,seed", [(20000, 30000, 500, 1), (300000, 500000, 6000, 2),
                                                (50000, 0, 3000, 3)])
def test_digest_kernels_match_sorted(n, ne, n_small, seed, window, monkeypatch):
    """window: rows of the first selection pass (128: every large component
    continues into the second pass)."""
    from lazzaro_amd.ops import tenant_ops
    monkeypatch.setattr(tenant_ops, "DIGEST_WINDOW", window)
    g = _graph(n, ne, n_small, seed)
    for take in (10, 3):
        got = [r.tolist() for r in g.component_digest(3, 0.3, take)]
        g._digest_sorted = True
        want = [r.tolist() for r in g.component_digest(3, 0.3, take)]
        g._digest_sorted = False
        assert got == want and len(want) > 10
    torch.cuda.synchronize()


@pytest.mark.parametrize("seed", [4, 5])
def test_local_digest_matches_sorted(seed):
    """The O(edges), sync-free digest (ops.tenant_ops.component_digest_local:
    endpoint renumbering, used when the edges touch few rows) against the
    sorted formulation, and its Capture form."""
    g = _graph(200000, 600, 300, seed)  # a small "giant" + chains over a 200k-row tenant
    assert g._digest_local(3, 10)
    for take in (10, 3):
        got = [r.tolist() for r in g.component_digest(3, 0.3, take)]
        cap = [r.tolist() for r in g.digest_capture(3, 0.3, take).get()]
        g._digest_sorted = True
        want = [r.tolist() for r in g.component_digest(3, 0.3, take)]
        g._digest_sorted = False
        assert got == want == cap and len(want) > 10


def test_first_rows_kernel_matches_topk():
    """tenant.hip tg_first_rows_kernel (first shard-node rows in (shard,
    row) order from the host shard counts) against the top-k formulation on
    the CPU copy of the same tenant, after removals, with super-nodes."""
    from lazzaro_amd.engine.tenant_graph import TenantGraph
    rng = np.random.default_rng(7)
    n = 300000
    gs = []
    for dev in ("cpu", "cuda"):
        g = TenantGraph(device=dev, dim=4)
        codes = [g.shard_id(f"s{i}") for i in range(5)]
        r2 = np.random.default_rng(7)
        sh = r2.choice([codes[1], codes[3], codes[4]], n, p=[0.0001, 0.5, 0.4999]).tolist()
        g.add_nodes([f"node_{i}" for i in range(n)], [f"c{i}" for i in range(n)],
                    r2.standard_normal((n, 4)).astype(np.float32).tolist(), shard=sh,
                    sup=(r2.random(n) < 0.05).astype(np.int64).tolist())
        g.remove_nodes(np.random.default_rng(8).choice(n, 40000, replace=False).tolist())
        gs.append(g)
    cpu, gpu = gs
    cpu.FIRST_ROWS_WINDOW = 1 << 30  # the one-pass top-k
    for k in (1, 10, 40, 200):
        ref = cpu.first_node_rows_dev(k, super_=False).tolist()
        assert gpu.first_node_rows_dev(k, super_=False).tolist() == ref and len(ref) == k
        assert gpu.first_rows_capture(k).get().tolist() == ref


def test_first_rows_short_shard_returns_only_found_rows():
    """The host shard counts claim more live rows than the device columns
    hold (a shard's rows were turned into super-nodes behind the counts):
    the kernel leaves the unfilled targets at -1 and both entry points drop
    them, so every returned row is a real shard node."""
    from lazzaro_amd.engine.tenant_graph import TenantGraph, NODE
    g = TenantGraph(device="cuda", dim=4)
    a, b = g.shard_id("a"), g.shard_id("b")
    n = 64
    g.add_nodes([f"node_{i}" for i in range(n)], [f"c{i}" for i in range(n)],
                np.ones((n, 4), dtype=np.float32).tolist(), shard=[a] * 8 + [b] * (n - 8))
    g.sup[:4] = 1  # device-side: 4 of shard a's 8 rows are no longer shard nodes; host counts still say 8
    got = g.first_node_rows_dev(20, super_=False).tolist()
    cap = g.first_rows_capture(20).get().tolist()
    assert got == cap
    assert all(r >= 0 for r in got)
    kind, sup = g.kind.cpu().numpy(), g.sup.cpu().numpy()
    assert all(kind[r] == NODE and sup[r] == 0 for r in got)
    assert got[:4] == [4, 5, 6, 7]


@pytest.mark.parametrize("n,ne_giant,n_small,seed", [(5000, 300, 60, 6), (400000, 900, 40, 7), (3000, 2000, 0, 8)])
def test_small_digest_kernel_matches_sorted(n, ne_giant, n_small, seed):
    """digest.hip dg_small_kernel (one block, <= 2048 edges: sort + renumber,
    union-find, reductions, selection rounds) against the sorted formulation,
    with a giant component of more than `take` candidates, chains, ghosts and
    super-nodes."""
    from lazzaro_amd.ops import tenant_ops as T
    g = _graph(n, ne_giant, n_small, seed)
    assert 0 < g.num_edges <= T.dg_small_max_edges() and g._digest_local(3, 10)
    for take in (10, 3, 1):
        got = [r.tolist() for r in g.component_digest(3, 0.3, take)]
        cap = [r.tolist() for r in g.digest_capture(3, 0.3, take).get()]
        g._digest_sorted = True
        want = [r.tolist() for r in g.component_digest(3, 0.3, take)]
        g._digest_sorted = False
        assert got == want == cap and len(want) >= 1
