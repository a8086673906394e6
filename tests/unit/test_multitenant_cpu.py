"""Multi-tenant batched search (segment kernel path) on CPU tensors: same
results as searching each tenant separately."""
import numpy as np
import torch

from lazzaro_amd.core.vector_store import HBMStore
from lazzaro_amd.index.arena import VectorArena, multi_arena_search
from lazzaro_amd.ops.search import segment_topk


def test_segment_topk_cpu_reference():
    g = torch.Generator().manual_seed(0)
    xs = [torch.randn(n, 32, generator=g) for n in (5, 0, 40, 1)]
    Q = torch.randn(4, 32, generator=g)
    b = [torch.randn(x.shape[0], generator=g) for x in xs]
    s, i = segment_topk(xs, Q, 3, biases=b, alpha=2.0)
    for q in range(4):
        if xs[q].shape[0] == 0:
            assert (i[q] == -1).all()
            continue
        ref = 2.0 * xs[q] @ Q[q] + b[q]
        o = torch.argsort(-ref, stable=True)[:3]
        m = min(3, xs[q].shape[0])
        assert torch.equal(i[q, :m], o[:m]) and torch.allclose(s[q, :m], ref[o[:m]])


def test_multi_arena_matches_per_arena():
    rng = np.random.default_rng(1)
    arenas = []
    for t in range(5):
        a = VectorArena(dim=16, device="cpu")
        n = int(rng.integers(1, 30))
        a.add([f"t{t}_{i}" for i in range(n)], rng.standard_normal((n, 16)).astype(np.float32))
        if n > 3:
            a.delete([f"t{t}_1"])
        arenas.append(a)
    q = rng.standard_normal((7, 16)).astype(np.float32)
    owners = [arenas[i % 5] for i in range(7)]
    for metric in ("l2", "ip", "cosine"):
        s, r = multi_arena_search(owners, q, 4, metric)
        for j, a in enumerate(owners):
            rs, rr = a.search_rows(q[j:j + 1], 4, metric)
            valid = rr[0] >= 0
            assert torch.equal(r[j][valid], rr[0][valid]), metric
            assert torch.allclose(s[j][valid], rs[0][valid], atol=1e-4), metric


def test_store_search_nodes_multi(tmp_path):
    st = HBMStore(db_dir=str(tmp_path), device="cpu")
    rng = np.random.default_rng(2)
    for u in ("alice", "bob", "carol"):
        vs = rng.standard_normal((6, 8)).astype(np.float32)
        st.add_nodes([{"id": f"{u}{i}", "content": "c", "embedding": v.tolist()} for i, v in enumerate(vs)], user_id=u)
    qs = rng.standard_normal((4, 8)).astype(np.float32).tolist()
    users = ["bob", "alice", "carol", "nobody"]
    got = st.search_nodes_multi(qs, users, limit=3)
    want = [st.search_nodes(q, user_id=u, limit=3) for q, u in zip(qs, users)]
    assert got == want and got[3] == []
