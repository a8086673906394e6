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


def test_shared_store_release_keeps_other_tenants_bound(tmp_path):
    """MemorySystem.close() on a tenant whose store was passed in
    (one HBMStore shared by the service's tenants) unbinds only that tenant;
    the store itself and the other tenants' graph bindings stay."""
    from lazzaro_amd.core.memory_system import MemorySystem
    from lazzaro_amd.core.providers import HashEmbedder, LocalLLM
    from lazzaro_amd.parallel import Communicator
    from lazzaro_amd.parallel.service import DistributedMemoryService
    store = HBMStore(db_dir=str(tmp_path), device="cpu")
    emb = HashEmbedder(dim=32)

    def factory(user, load_from_disk=True):
        return MemorySystem(llm_provider=LocalLLM(), embedding_provider=emb, enable_async=False, store=store,
                            db_dir=str(tmp_path), user_id=user, device="cpu", load_from_disk=load_from_disk)
    svc = DistributedMemoryService(Communicator.local(), factory, max_resident=2)
    for u in ("a", "b", "c"):  # building c releases a (LRU)
        svc.serve([(u, "start_conversation"), (u, "chat", f"{u} works on a project with a deadline."),
                   (u, "end_conversation")])
    assert sorted(svc.systems) == ["b", "c"]
    for u in ("b", "c"):
        assert store.bound_graph(u) is svc.systems[u].graph and svc.systems[u]._store_binds_graph()
    assert store.bound_graph("a") is None
    # a comes back from the store with its memory
    got = svc.serve([("a", "search_memories", "project deadline", 2)])[0]
    assert got and all(n["id"].startswith("node_") for n in got)
    svc.close()
