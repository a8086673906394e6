"""DistributedMemoryService on one GPU: the fused multi-tenant search (one
embed + one segment_topk launch over every tenant's fp32 rows) returns what
each tenant's own MemorySystem.search_memories_batch returns."""
import hashlib

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


class RandEmbedder:
    """text -> a fixed pseudo-random unit vector (no ties between rows)."""

    def __init__(self, dim=64):
        self.dim = dim

    def _v(self, t):
        seed = int.from_bytes(hashlib.md5(t.encode()).digest()[:4], "little")
        v = np.random.default_rng(seed).standard_normal(self.dim).astype(np.float32)
        return (v / np.linalg.norm(v)).tolist()

    def embed(self, t):
        return self._v(t)

    def batch_embed(self, ts):
        return [self._v(t) for t in ts]


@pytest.mark.parametrize("comm_dev", ["cuda", None])
def test_fused_multi_tenant_search_matches_per_tenant(tmp_path, comm_dev):
    """comm_dev None: a host communicator fronting GPU tenants (the multi-
    tenant bench's setup) -- the tenant pointer table must live on the
    tenants' device, not the communicator's."""
    from lazzaro_amd.core.memory_system import MemorySystem
    from lazzaro_amd.core.providers import LocalLLM
    from lazzaro_amd.parallel import Communicator
    from lazzaro_amd.parallel.service import DistributedMemoryService
    emb = RandEmbedder()

    def factory(user, load_from_disk=True):
        return MemorySystem(llm_provider=LocalLLM(), embedding_provider=emb, enable_async=False,
                            db_dir=str(tmp_path), user_id=user, device="cuda", load_from_disk=load_from_disk,
                            max_buffer_size=10 ** 6)
    comm = Communicator.local(torch.device(comm_dev)) if comm_dev else Communicator.local()
    svc = DistributedMemoryService(comm, factory)
    users = [f"t{i}" for i in range(24)]
    rng = np.random.default_rng(0)
    for j, u in enumerate(users):
        ms = svc.system(u)
        n = 50 + 37 * j
        texts = [f"{u} memory {i}" for i in range(n)]
        V = torch.tensor(emb.batch_embed(texts), device="cuda")
        ms.graph.add_nodes([f"{u}_n{i}" for i in range(n)], texts, V, shard=ms.graph.shard_id("work"), stored=True)
    reqs = [(users[int(rng.integers(len(users)))], "search_memories", f"query {q}", 5) for q in range(200)]
    fused = svc.serve(reqs)
    for (u, _, q, k), got in zip(reqs, fused):
        ref = svc.system(u).search_memories_batch([q], limit=k)[0]
        assert [n["id"] for n in got] == [n.id for n in ref], u
    svc.close()


def test_serve_stream_equals_serve(tmp_path):
    """serve_stream (round i+1 routed and its batched search enqueued before
    round i's results are built) returns exactly what serve returns."""
    from lazzaro_amd.core.memory_system import MemorySystem
    from lazzaro_amd.core.providers import LocalLLM
    from lazzaro_amd.parallel import Communicator
    from lazzaro_amd.parallel.service import DistributedMemoryService
    emb = RandEmbedder()

    def factory(user, load_from_disk=True):
        return MemorySystem(llm_provider=LocalLLM(), embedding_provider=emb, enable_async=False,
                            db_dir=str(tmp_path), user_id=user, device="cuda", load_from_disk=load_from_disk)
    svc = DistributedMemoryService(Communicator.local(torch.device("cuda")), factory)
    users = [f"s{i}" for i in range(10)]
    for j, u in enumerate(users):
        g = svc.system(u).graph
        texts = [f"{u} fact {i}" for i in range(40 + 9 * j)]
        g.add_nodes([f"{u}_{i}" for i in range(len(texts))], texts, torch.tensor(emb.batch_embed(texts), device="cuda"),
                    shard=g.shard_id("work"), stored=True)
    rng = np.random.default_rng(1)
    rounds = [[(users[int(rng.integers(10))], "search_memories", f"r{r} q{q}", 4) for q in range(64)]
              for r in range(5)]
    want = [svc.serve(r) for r in rounds]
    got = list(svc.serve_stream(rounds))
    assert got == want
    svc.close()


def _seeded_service(tmp_path, emb, users, store=None):
    from lazzaro_amd.core.memory_system import MemorySystem
    from lazzaro_amd.core.providers import LocalLLM
    from lazzaro_amd.parallel import Communicator
    from lazzaro_amd.parallel.service import DistributedMemoryService

    def factory(user, load_from_disk=True):
        return MemorySystem(llm_provider=LocalLLM(), embedding_provider=emb, enable_async=False,
                            db_dir=str(tmp_path), user_id=user, device="cuda", load_from_disk=load_from_disk,
                            store=store, max_buffer_size=60)
    svc = DistributedMemoryService(Communicator.local(torch.device("cuda")), factory)
    for j, u in enumerate(users):
        g = svc.system(u).graph
        texts = [f"{u} fact {i}" for i in range(40 + 9 * j)]
        g.add_nodes([f"{u}_{i}" for i in range(len(texts))], texts, torch.tensor(emb.batch_embed(texts), device="cuda"),
                    shard=g.shard_id("work"), stored=True)
    return svc


def test_serve_stream_with_mutations_equals_serve(tmp_path):
    """Rounds that mix searches with mutating requests (a conversation whose
    end evicts rows past max_buffer_size) on the same tenants: serve_stream
    finishes the previous round's batched search before mutating one of its
    tenants, so every round equals serve() on an identical replica."""
    emb = RandEmbedder()
    users = [f"m{i}" for i in range(6)]
    rng = np.random.default_rng(3)
    rounds = []
    for r in range(6):
        rr = [(users[int(rng.integers(6))], "search_memories", f"r{r} q{q}", 4) for q in range(24)]
        u = users[r % 6]
        rr += [(u, "start_conversation"), (u, "chat", f"{u} round {r}: I work on a project deadline."),
               (u, "end_conversation")]
        rounds.append(rr)
    a = _seeded_service(tmp_path / "a", emb, users)
    want = [a.serve(r) for r in rounds]
    a.close()
    b = _seeded_service(tmp_path / "b", emb, users)
    got = list(b.serve_stream(rounds))
    b.close()
    def strip(v):
        """status strings carry timings, and super-node ids the creation second
        (reference ``super_{shard}_{int(time.time())}``): both are wall-clock
        dependent, so the two replicas are compared without them"""
        def norm(x):  # (search results may be lazily materialised sequences)
            if not isinstance(x, (str, bytes, dict)) and hasattr(x, "__iter__"):
                return [norm(y) for y in x]
            if isinstance(x, dict) and str(x.get("id", "")).startswith("super_"):
                return {**x, "id": x["id"].rsplit("_", 1)[0]}
            return x
        return [norm(x) for x in v if not isinstance(x, str)]
    if [strip(x) for x in got] != [strip(x) for x in want]:  # a compact account of the mismatch
        for r, (gr, wr) in enumerate(zip(got, want)):
            for q, (gq, wq) in enumerate(zip(strip(gr), strip(wr))):
                if gq != wq:
                    print("MISMATCH round", r, "req", q, rounds[r][q][:3])
                    print("  got ", [(d["id"], d["salience"], d["access_count"]) for d in gq] if isinstance(gq, list) else gq)
                    print("  want", [(d["id"], d["salience"], d["access_count"]) for d in wq] if isinstance(wq, list) else wq)
    assert [strip(x) for x in got] == [strip(x) for x in want]


def test_shared_store_survives_tenant_release(tmp_path):
    """One HBMStore shared by every tenant (the service's setup): releasing a
    tenant (LRU, max_resident) unbinds only that tenant's graph, so the fused
    multi-tenant search keeps serving the others."""
    from lazzaro_amd.core.vector_store import HBMStore
    emb = RandEmbedder()
    store = HBMStore(db_dir=str(tmp_path / "db"), device=torch.device("cuda"))
    users = [f"r{i}" for i in range(4)]
    svc = _seeded_service(tmp_path, emb, users, store=store)
    svc.max_resident = 4
    svc.system("extra")  # 5 resident > 4: releases r0 (LRU)
    assert "r0" not in svc.systems and store.bound_graph("r0") is None
    for u in users[1:]:
        assert store.bound_graph(u) is svc.systems[u].graph
        assert svc.systems[u]._store_binds_graph()
    got = svc.serve([(u, "search_memories", "fact 3", 3) for u in users[1:]])
    assert all(len(x) == 3 for x in got)
    svc.close()


def test_search_routed_matches_per_tenant_gpu(tmp_path):
    """Columnar routed search on one GPU: small tenants share one fused
    segment_topk launch (tenant table pointers), a big tenant goes through
    its store search; every query's hits equal the tenant's own
    search_memories_batch, and resolve() returns the same nodes."""
    from lazzaro_amd.parallel import routing
    emb = RandEmbedder()
    users = [f"q{i}" for i in range(12)]
    svc = _seeded_service(tmp_path, emb, users)
    svc.embedder = emb
    big = svc.system("big")
    n = routing.BIG_ROWS + 1000
    g = big.graph
    V = torch.nn.functional.normalize(torch.randn(n, 64, device="cuda"), dim=1)
    g.add_nodes([f"big_{i}" for i in range(n)], [f"big {i}" for i in range(n)], V, shard=g.shard_id("work"),
                stored=True)
    rng = np.random.default_rng(5)
    allu = users + ["big"]
    qu = [allu[int(rng.integers(len(allu)))] for _ in range(300)]
    qs = [f"query {i}" for i in range(300)]
    lim = [int(x) for x in rng.integers(1, 9, 300)]
    hits = svc.search_routed(qu, qs, lim)
    nodes = svc.resolve(hits)
    E = torch.tensor(emb.batch_embed(qs), device="cuda")
    for q in range(300):
        ms = svc.system(qu[q])
        _, rr = ms.graph.store_search(E[q:q + 1], lim[q])
        kind = ms.graph.mirror("kind")
        ref = [ms.graph.ids[int(r)] for r in rr[0].tolist() if r >= 0 and kind[int(r)] == 1]
        assert [x["id"] for x in nodes[q]] == ref, q
        assert [v.id for v in hits.local_nodes(svc, q)] == ref
    svc.close()


@pytest.mark.parametrize("overflow", [False, True])
def test_search_global_multi_tenant_pass_matches_per_tenant(tmp_path, monkeypatch, overflow):
    """search_global_batch over 40 small tenants (1..~700 rows: partial tiles,
    one-row tenants, removed rows) + one big tenant: the one-pass tile-table
    scan (csrc/kernels/mtscan.hip) returns the hits of the per-tenant store
    searches (MT_GLOBAL = False), scores to fp32 rounding. overflow=True: a
    threshold that admits every row, so every query's list overflows and is
    redone by the per-tenant path."""
    from lazzaro_amd.ops import search as S
    from lazzaro_amd.parallel import routing
    emb = RandEmbedder()
    users = [f"g{i}" for i in range(40)]
    svc = _seeded_service(tmp_path, emb, [])
    rng = np.random.default_rng(9)
    for j, u in enumerate(users):
        g = svc.system(u).graph
        n = 1 if j % 13 == 0 else int(rng.integers(2, 700))
        V = torch.nn.functional.normalize(torch.randn(n, 64, device="cuda"), dim=1)
        g.add_nodes([f"{u}_{i}" for i in range(n)], [f"{u} {i}" for i in range(n)], V, shard=g.shard_id("work"),
                    stored=True)
        if n > 20:
            g.remove_nodes([3, 7, n - 1], unstore=True)
    big = svc.system("big").graph
    n = routing.BIG_ROWS + 500
    big.add_nodes([f"big_{i}" for i in range(n)], [f"big {i}" for i in range(n)],
                  torch.nn.functional.normalize(torch.randn(n, 64, device="cuda"), dim=1), shard=big.shard_id("work"),
                  stored=True)
    Q = torch.nn.functional.normalize(torch.randn(300, 64, device="cuda"), dim=1)
    if overflow:
        monkeypatch.setattr(S, "_mt_threshold", lambda Xs, bs, Q16, *a: torch.full((Q16.shape[0],), float("-inf"),
                                                                                   device=Q16.device))
    monkeypatch.setattr(routing, "MT_GLOBAL", True)
    got = routing.search_global_batch(svc, Q, 6)
    monkeypatch.setattr(routing, "MT_GLOBAL", False)
    want = routing.search_global_batch(svc, Q, 6)
    gu, wu = got.users(svc), want.users(svc)
    _, _, grow = got.split()
    _, _, wrow = want.split()
    assert torch.allclose(got.scores, want.scores, rtol=1e-5, atol=1e-5)
    assert gu == wu
    assert torch.equal(grow, wrow)
    assert (want.keys >= 0).all()
    svc.close()
