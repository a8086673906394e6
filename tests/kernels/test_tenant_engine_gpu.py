"""The device engine under MemorySystem (engine/tenant_graph.py,
csrc/kernels/tenant.hip) on an MI355X vs the same engine on the CPU.

* kernel-level: each tenant kernel against the torch reference of tenant_ops;
* system-level: the same MemorySystem scenario (conversations, chat with
  boost/touch, dedupe, linking, decay/prune, eviction, super-nodes, deep
  consolidation, persistence reload) on cuda and on cpu must produce the same
  nodes, edges, saliences, access counts and profile; and a large-tenant
  scenario that takes the fused MFMA scan path (bf16 candidates + float64
  re-rank) must take the same decisions as the CPU's exact float64 scan.
"""
import itertools
import json
import time

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

from lazzaro_amd.core.memory_system import MemorySystem  # noqa: E402
from lazzaro_amd.core.providers import HashEmbedder, LocalLLM  # noqa: E402
from lazzaro_amd.engine.tenant_graph import NODE, TenantGraph  # noqa: E402
from lazzaro_amd.ops import tenant_ops as T  # noqa: E402

DEV = "cuda"


def _edges(n, ne, seed, dev, n_shards=4):
    g = torch.Generator().manual_seed(seed)
    e = {"src": torch.randint(0, n, (ne,), generator=g, dtype=torch.int32),
         "dst": torch.randint(0, n, (ne,), generator=g, dtype=torch.int32),
         "w": torch.rand(ne, generator=g), "co": torch.arange(ne, dtype=torch.int32),
         "lu": torch.rand(ne, generator=g, dtype=torch.float64),
         "meta": torch.randint(0, n_shards, (ne,), generator=g, dtype=torch.int32) | (1 << 24)}
    return {k: v.to(dev) for k, v in e.items()}


def _nodes(n, seed, dev, n_shards=4):
    g = torch.Generator().manual_seed(seed)
    return {"sal": torch.rand(n, generator=g), "kind": torch.randint(0, 3, (n,), generator=g).to(torch.uint8),
            "sup": (torch.rand(n, generator=g) > 0.9).to(torch.uint8),
            "shard": torch.randint(0, n_shards, (n,), generator=g, dtype=torch.int32),
            "acc": torch.randint(0, 20, (n,), generator=g, dtype=torch.int32),
            "last": torch.rand(n, generator=g, dtype=torch.float64) * 1e6,
            "dirty": torch.zeros(n, dtype=torch.uint8)}


@pytest.mark.parametrize("ne,thr", [(0, 0.5), (1, 0.5), (5000, 0.4), (400_001, 0.3), (70_000, None)])
def test_decay_prune_kernel(ne, thr):
    n = 20000
    ec, eg = _edges(n, ne, 1, "cpu"), _edges(n, ne, 1, DEV)
    nc = _nodes(n, 2, "cpu")
    ng = {k: v.to(DEV) for k, v in nc.items()}
    oc, pc, dc = T.decay_prune(ec, nc["sal"], nc["kind"], nc["sup"], 0.05, thr, True, want_dropped=True)
    og, pg, dg = T.decay_prune(eg, ng["sal"], ng["kind"], ng["sup"], 0.05, thr, True, want_dropped=True)
    assert pc == pg
    for k in oc:
        assert torch.equal(oc[k], og[k].cpu()), k
    assert torch.equal(nc["sal"], ng["sal"].cpu())
    if thr is not None and pc:
        assert torch.equal(dc[0], dg[0].cpu()) and torch.equal(dc[1], dg[1].cpu())


@pytest.mark.parametrize("ne", [1000, 300_000])
def test_remove_edges_of_kernel(ne):
    n = 10000
    ec, eg = _edges(n, ne, 3, "cpu"), _edges(n, ne, 3, DEV)
    nc = _nodes(n, 4, "cpu")
    rm = (torch.rand(n, generator=torch.Generator().manual_seed(5)) > 0.8).to(torch.uint8)
    oc, kc, _ = T.remove_edges_of(ec, rm, nc["shard"])
    og, kg, _ = T.remove_edges_of(eg, rm.to(DEV), nc["shard"].to(DEV))
    assert kc == kg and kc > 0
    for k in oc:
        assert torch.equal(oc[k], og[k].cpu()), k


def test_visible_csr_boost_touch_importance_kernels():
    n, ne = 5000, 40000
    ec, eg = _edges(n, ne, 6, "cpu"), _edges(n, ne, 6, DEV)
    nc = _nodes(n, 7, "cpu")
    ng = {k: v.to(DEV) for k, v in nc.items()}
    cc = T.build_visible_csr(ec, nc["shard"], n)
    cg = T.build_visible_csr(eg, ng["shard"], n)
    for a, b in zip(cc, cg):
        assert torch.equal(a, b.cpu())
    seeds = torch.tensor([3, 17, 999, 4000, 17], dtype=torch.int32)
    st_c, st_g = T.BoostState(), T.BoostState()
    kc = T.neighbor_boost(cc, ec["w"], seeds, nc["kind"], nc["sup"], nc["sal"], nc["last"], nc["dirty"], 5e6, st_c)
    kg = T.neighbor_boost(cg, eg["w"], seeds.to(DEV), ng["kind"], ng["sup"], ng["sal"], ng["last"], ng["dirty"], 5e6,
                          st_g)
    assert kc == kg and kc > 0
    for k in ("sal", "last", "dirty"):
        assert torch.equal(nc[k], ng[k].cpu()), k
    # a second call on the same stamp array boosts again (new epoch)
    kg2 = T.neighbor_boost(cg, eg["w"], seeds.to(DEV), ng["kind"], ng["sup"], ng["sal"], ng["last"], ng["dirty"],
                           6e6, st_g)
    kc2 = T.neighbor_boost(cc, ec["w"], seeds, nc["kind"], nc["sup"], nc["sal"], nc["last"], nc["dirty"], 6e6, st_c)
    assert kg2 == kg == kc2
    rows = torch.tensor([1, 2, 3, 4999], dtype=torch.long)
    T.touch(rows, nc["acc"], nc["last"], nc["sal"], nc["dirty"], 7e6)
    T.touch(rows.to(DEV), ng["acc"], ng["last"], ng["sal"], ng["dirty"], 7e6)
    for k in ("acc", "last", "sal", "dirty"):
        assert torch.equal(nc[k], ng[k].cpu()), k
    ic = T.importance(nc["sal"], nc["acc"], nc["last"], nc["kind"], nc["sup"], 8e6)
    ig = T.importance(ng["sal"], ng["acc"], ng["last"], ng["kind"], ng["sup"], 8e6)
    assert torch.allclose(ic, ig.cpu(), rtol=1e-12, atol=0)


# ---------------------------------------------------------------- system level
class _Clock:
    def __init__(self):
        self.t = 1.7e9

    def __call__(self):
        self.t += 1.0
        return self.t


def _snapshot(ms):
    g = ms.graph
    nodes = {}
    for nid, n in ms.buffer.nodes.items():
        nodes[nid] = (n.content, n.shard_key, n.is_super_node, round(n.salience, 5), n.access_count,
                      tuple(n.child_ids), n.parent_id)
    edges = {}
    for sk, sh in ms.shards.items():
        for key, e in sh.edges.items():
            edges[(sk,) + key] = (round(e.weight, 5), e.co_occurrence, e.edge_type)
    return nodes, edges, json.dumps(ms.profile.data, sort_keys=True), ms.get_stats()["buffer_edges"], g.num_nodes()


TURNS = ["I work on a robotics project with my colleague Ana and we have a deadline on Friday.",
         "My family lives in Lisbon and my hobby is sailing on weekends.",
         "I am learning Japanese from a book and practice every morning.",
         "I go to the gym for exercise and track my sleep and diet.",
         "I started a new project on GPU kernels for a client meeting.",
         "My friend Tom visits home every summer and we cook together.",
         "I study distributed systems in an online course.",
         "I run five kilometres for fitness and drink green tea."]


def _scenario(device, tmp_path, monkeypatch):
    monkeypatch.setattr(time, "time", _Clock())
    ms = MemorySystem(llm_provider=LocalLLM(), embedding_provider=HashEmbedder(dim=64), enable_async=False,
                      db_dir=str(tmp_path / device), device=device, max_buffer_size=14, super_node_threshold=3,
                      consolidate_every=3, prune_threshold=0.3)
    for i, t in enumerate(itertools.islice(itertools.cycle(TURNS), 14)):
        ms.start_conversation()
        ms.chat(t)
        ms.chat(TURNS[(i * 3) % len(TURNS)])
        ms.end_conversation()
    snap = _snapshot(ms)
    hits = [n.id for n in ms.search_memories("robotics project deadline", limit=5)]
    conn = {nid: sorted(x.id for x in ms.get_connected_memories(nid)) for nid in list(ms.buffer.nodes)[:6]}
    ms.close()
    ms2 = MemorySystem(llm_provider=LocalLLM(), embedding_provider=HashEmbedder(dim=64), enable_async=False,
                       db_dir=str(tmp_path / device), device=device, max_buffer_size=14, super_node_threshold=3)
    reload_snap = _snapshot(ms2)
    ms2.close()
    return snap, hits, conn, reload_snap


def test_memory_system_cuda_matches_cpu(tmp_path, monkeypatch):
    cpu = _scenario("cpu", tmp_path, monkeypatch)
    gpu = _scenario(DEV, tmp_path, monkeypatch)
    (nc, ec, pc, bc, cc), (ng, eg, pg, bg, cg) = cpu[0], gpu[0]
    assert nc.keys() == ng.keys() and cc == cg and cc > 0
    for k in nc:
        assert nc[k] == ng[k], k
    assert ec == eg and bc == bg and pc == pg and len(ec) > 0
    assert cpu[1] == gpu[1] and cpu[2] == gpu[2]
    # a reload from the incremental store reproduces the in-memory graph
    assert cpu[3][0].keys() == nc.keys() and gpu[3][0].keys() == ng.keys()
    for k in nc:
        assert cpu[3][0][k][:3] == nc[k][:3] and abs(cpu[3][0][k][3] - nc[k][3]) < 1e-4
        assert gpu[3][0][k][:3] == ng[k][:3] and abs(gpu[3][0][k][3] - ng[k][3]) < 1e-4
    assert cpu[3][1].keys() == ec.keys() and gpu[3][1].keys() == eg.keys()


def _clustered(n, d, n_clusters, seed, noise=0.35):
    g = torch.Generator().manual_seed(seed)
    C = torch.randn(n_clusters, d, generator=g)
    C = C / C.norm(dim=1, keepdim=True)
    lab = torch.randint(0, n_clusters, (n,), generator=g)
    X = C[lab] + noise * torch.randn(n, d, generator=g) / d ** 0.5
    return X / X.norm(dim=1, keepdim=True), lab


def test_consolidate_batch_int8_dual_decisions_at_scale_gpu(tmp_path, monkeypatch):
    """A 1.2M-row tenant -- past LOWP_MIN_ROWS, so consolidation's candidate
    lists come from the int8 dual scan (its default) -- consolidates a batch
    of 32 conversations (192 facts: duplicates of stored rows, related and new
    facts) at the reference cadence; the same batch on the same tenant with
    the int8 scan switched off (bf16 dual scan, itself pinned to the exact
    float64 scan) makes the same decisions: the same counts, nodes,
    saliences, access counts, edges and victims."""
    from lazzaro_amd.engine import tenant_graph as TG
    from lazzaro_amd.ops import search as S
    N, D, B, F = 1_200_000, 384, 32, 6
    X, lab = _clustered(N, D, 256, 21, noise=1.6)
    gen = torch.Generator().manual_seed(5)
    facts, vecs = [], []
    for c in range(B):
        conv = []
        for f in range(F):
            kind = (c * F + f) % 3
            if kind == 0:  # near-duplicate of a stored row
                v = X[int(torch.randint(0, N, (1,), generator=gen))] + 0.01 * torch.randn(D, generator=gen) / D ** 0.5
            elif kind == 1:  # related: a cluster centre's neighbourhood
                v = X[int(torch.randint(0, N, (1,), generator=gen))] + 0.9 * torch.randn(D, generator=gen) / D ** 0.5
            else:
                v = torch.randn(D, generator=gen)
            vecs.append(v / v.norm())
            conv.append({"content": f"fact {c}.{f}", "salience": 0.5 + 0.01 * f, "topic": f"topic{(c + f) % 8}"})
        facts.append(conv)
    V = torch.stack(vecs)
    calls = {"i8": 0}
    real = S.flat_topk_dual_i8

    def counted(*a, **k):
        calls["i8"] += 1
        return real(*a, **k)
    monkeypatch.setattr(S, "flat_topk_dual_i8", counted)
    out = {}
    for mode in ("int8", "bf16"):
        monkeypatch.setattr(TG, "DUAL_LOWP", mode == "int8")
        monkeypatch.setattr(time, "time", _Clock())
        ms = MemorySystem(llm_provider=LocalLLM(), embedding_provider=HashEmbedder(dim=D), enable_async=False,
                          db_dir=str(tmp_path / mode), device=DEV, load_from_disk=False, max_buffer_size=N + 40,
                          super_node_threshold=10 ** 9)
        g = ms.graph
        shards = [g.shard_id(f"topic{c}") for c in range(8)]
        g.add_nodes([f"node_{i + 1}" for i in range(N)], [f"m {i}" for i in range(N)], X.to(DEV),
                    shard=np.asarray([shards[int(c) % 8] for c in lab], dtype=np.int32),
                    sal=torch.rand(N, generator=torch.Generator().manual_seed(1)), stored=True)
        ms.node_counter = N
        before = calls["i8"]
        st = ms.consolidate_batch(facts, embeddings=V.to(DEV), now=1.8e9)
        used = calls["i8"] - before
        n = g.n
        live = (g.kind[:n] == NODE).cpu().numpy()
        e = {k: v.cpu() for k, v in g.e.items()}
        order = np.lexsort((e["dst"].numpy(), e["src"].numpy()))
        out[mode] = (st, used, np.nonzero(live)[0], g.sal[:n].cpu().numpy()[live], g.acc[:n].cpu().numpy()[live],
                     {k: v.numpy()[order] for k, v in e.items() if k in ("src", "dst", "w", "meta")})
        ms.close()
    a, b = out["int8"], out["bf16"]
    assert a[1] >= 1 and b[1] == 0  # the int8 dual scan made the first run's lists, not the second's
    assert a[0] == b[0]
    assert a[0]["dup"] > 0 and a[0]["linked"] > 0 and a[0]["evicted"] > 0
    assert np.array_equal(a[2], b[2]) and np.array_equal(a[3], b[3]) and np.array_equal(a[4], b[4])
    for k in a[5]:
        assert np.array_equal(a[5][k], b[5][k]), k


def test_large_tenant_kernel_path_matches_exact_cpu(tmp_path, monkeypatch):
    """60k-node tenant: dedupe + links from the fused dual MFMA scan on the
    GPU vs the exact float64 scan on the CPU; then decay/prune, eviction,
    components + profile and super-nodes. Identical decisions expected."""
    monkeypatch.setattr(time, "time", _Clock())
    N, D, M = 60000, 128, 256
    X, lab = _clustered(N + M, D, 64, 11)
    out = {}
    for dev in ("cpu", DEV):
        monkeypatch.setattr(time, "time", _Clock())  # same clock readings for both devices
        ms = MemorySystem(llm_provider=LocalLLM(), embedding_provider=HashEmbedder(dim=D), enable_async=False,
                          db_dir=str(tmp_path / dev), device=dev, load_from_disk=False, max_buffer_size=N + 64,
                          super_node_threshold=10 ** 9)
        g = ms.graph
        shards = [g.shard_id(f"topic{c % 8}") for c in range(64)]
        g.add_nodes([f"node_{i + 1}" for i in range(N)], [f"fact {i}" for i in range(N)], X[:N],
                    shard=np.asarray([shards[int(c)] for c in lab[:N]], dtype=np.int32),
                    sal=torch.rand(N, generator=torch.Generator().manual_seed(1)), stored=True)
        ms.node_counter = N
        # duplicates of existing rows + genuinely new facts
        Q = torch.cat([X[:32], X[N:N + M - 32]])
        facts = [{"content": f"new {j}", "salience": 0.9, "topic": f"topic{int(lab[j if j < 32 else N + j - 32]) % 8}"}
                 for j in range(M)]
        assert g._use_kernel(M) == (dev == DEV)
        new = ms._ingest_facts(facts, Q)
        pruned = g.decay(0.01, 0.5)
        victims = g.evict(N + 32)
        comps = g.components()
        ws, wc = g.component_edge_stats(comps)
        out[dev] = (new, pruned, victims, g.num_edges, [c.tolist() for c in comps if c.size > 1],
                    np.round(ws, 6).tolist(), wc.tolist(), g.sal[: g.n].cpu().numpy(), g.acc[: g.n].cpu().numpy(),
                    {k: v.cpu() for k, v in g.e.items()})
        ms.close()
    c, gg = out["cpu"], out[DEV]
    assert c[0] == gg[0] and len(c[0]) == M - 32
    assert c[1] == gg[1] and c[2] == gg[2] and c[3] == gg[3] and c[3] > 0
    assert c[4] == gg[4] and c[5] == gg[5] and c[6] == gg[6]
    assert np.array_equal(c[7], gg[7]) and np.array_equal(c[8], gg[8])
    for k in c[9]:
        assert torch.equal(c[9][k], gg[9][k]), k


def test_store_search_fp32_exact_recall_gpu():
    """HBM store search (bf16 MFMA candidates + fp32 re-rank) == exact fp32
    L2 top-10 over the original fp32 vectors."""
    g = TenantGraph(device=DEV)
    N, D = 300_000, 768
    gen = torch.Generator().manual_seed(3)
    X = torch.randn(N, D, generator=gen)
    X = X / X.norm(dim=1, keepdim=True)
    g.add_nodes([f"n{i}" for i in range(N)], [""] * N, X, shard=g.shard_id("work"), stored=True)
    Q = torch.randn(512, D, generator=gen)
    Q = Q / Q.norm(dim=1, keepdim=True)
    _, rows = g.store_search(Q.to(DEV), 10, "l2")
    Xg, Qg = X.to(DEV), Q.to(DEV)
    d2 = (Qg * Qg).sum(1, keepdim=True) - 2 * Qg @ Xg.T + (Xg * Xg).sum(1)[None, :]
    truth = torch.topk(-d2, 10, dim=1).indices
    hit = sum(len(set(a) & set(b)) for a, b in zip(rows.cpu().tolist(), truth.cpu().tolist()))
    assert hit / (512 * 10) == 1.0


def test_search_memories_stream_matches_batch_gpu(tmp_path):
    """Pipelined search_memories_stream == search_memories_batch per batch on
    a 200k-memory tenant (device rows -> pinned async copy -> Node views)."""
    from lazzaro_amd.core.embedders import OnDeviceEmbedder

    emb = OnDeviceEmbedder("minilm-l6", device=DEV, max_len=32)
    ms = MemorySystem(llm_provider=LocalLLM(), embedding_provider=emb, enable_async=False,
                      db_dir=str(tmp_path), device=DEV, load_from_disk=False, max_buffer_size=10 ** 7)
    g = ms.graph
    N = 200_000
    gen = torch.Generator().manual_seed(5)
    X = torch.randn(N, emb.dim, generator=gen)
    X = X / X.norm(dim=1, keepdim=True)
    g.add_nodes([f"node_{i + 1}" for i in range(N)], [f"m{i}" for i in range(N)], X, shard=g.shard_id("work"),
                stored=True)
    batches = [[f"query {b} {j} about project deadline" for j in range(300)] for b in range(3)]
    want = [[[n.id for n in r] for r in ms.search_memories_batch(qs, limit=10)] for qs in batches]
    got = [[[n.id for n in r] for r in res] for res in ms.search_memories_stream(batches, limit=10)]
    assert got == want and all(len(r) == 10 for b in got for r in b)
    ms.close()


@pytest.mark.parametrize("mode", ["i8", "fp8"])
@pytest.mark.parametrize("data", ["isotropic", "clustered"])
def test_store_search_lowp_scan_exact_recall_gpu(data, mode):
    """Large tenant (> LOWP_MIN_ROWS) + large batch: candidates from the int8
    (or fp8) MFMA scan with the error-model margin, re-scored from bf16 and
    re-ranked in fp32 == exact fp32 L2 top-10 over the original vectors."""
    from lazzaro_amd.engine import tenant_graph as TG
    saved = TG.TenantGraph.LOWP
    TG.TenantGraph.LOWP = mode
    g = TenantGraph(device=DEV)
    N, D = (1 << 20) + 4096, 768
    gen = torch.Generator(device=DEV).manual_seed(7)
    if data == "isotropic":
        X = torch.randn(N, D, device=DEV, generator=gen)
    else:
        C = torch.randn(256, D, device=DEV, generator=gen)
        X = C[torch.randint(0, 256, (N,), device=DEV, generator=gen)] + 0.5 * torch.randn(N, D, device=DEV,
                                                                                        generator=gen)
    X = X / X.norm(dim=1, keepdim=True)
    g.add_nodes([f"n{i}" for i in range(N)], [""] * N, X, shard=g.shard_id("work"), stored=True)
    assert g.emb8 is not None and g.emb8.dtype == (torch.int8 if mode == "i8" else torch.uint8)
    Q = torch.randn(512, D, device=DEV, generator=gen)
    if data == "clustered":
        Q = X[torch.randint(0, N, (512,), device=DEV, generator=gen)] + 0.3 * Q / D ** 0.5
    Q = Q / Q.norm(dim=1, keepdim=True)
    assert 512 >= TG.LOWP_MIN_Q and N >= TG.LOWP_MIN_ROWS
    _, rows = g.store_search(Q, 10, "l2")
    Xd, Qd = X.double(), Q.double()
    truth = []
    for c0 in range(0, N, 1 << 18):
        s = 2 * Qd @ Xd[c0:c0 + (1 << 18)].T - (Xd[c0:c0 + (1 << 18)] ** 2).sum(1)[None, :]
        v, i = torch.topk(s, 10, dim=1)
        truth.append((v, i + c0))
    v = torch.cat([t[0] for t in truth], 1)
    i = torch.cat([t[1] for t in truth], 1)
    top = torch.gather(i, 1, torch.topk(v, 10, dim=1).indices)
    hit = sum(len(set(a) & set(b)) for a, b in zip(rows.cpu().tolist(), top.cpu().tolist()))
    assert hit / (512 * 10) == 1.0
    # and the bf16 scan gives the same rows
    TG.TenantGraph.LOWP, g.emb8 = "off", None
    try:
        _, rows16 = g.store_search(Q, 10, "l2")
    finally:
        TG.TenantGraph.LOWP = saved
    assert torch.equal(rows16, rows)


@pytest.mark.parametrize("nq", [512, 200])
def test_flat_topk_i8_matches_bf16_gpu(nq):
    """int8 scan + error cut + bf16 re-score == the bf16 scan's top-10
    (scores equal up to accumulation order), with and without a cut; nq =
    200 leaves most of the query tile empty."""
    from lazzaro_amd.ops.search import flat_topk, flat_topk_i8, quantize_i8_rows
    gen = torch.Generator(device=DEV).manual_seed(5)
    N, D = 1_300_000, 768
    X = torch.randn(N, D, device=DEV, generator=gen)
    X = X / X.norm(dim=1, keepdim=True)
    Q = torch.randn(nq, D, device=DEV, generator=gen)
    Q = Q / Q.norm(dim=1, keepdim=True)
    X16, Q16 = X.to(torch.bfloat16), Q.to(torch.bfloat16)
    bias = -(X * X).sum(1).contiguous()
    bias[::97] = float("-inf")  # removed rows never surface
    s16, r16 = flat_topk(X16, Q16, 10, bias=bias, alpha=2.0)
    X8, rs = quantize_i8_rows(X16)
    Q8, qs = quantize_i8_rows(Q16)
    assert X8.dtype == torch.int8 and rs.shape == (N,) and float(rs.min()) > 0
    for margin in (torch.full((nq,), 0.03, device=DEV), None):
        s8, r8 = flat_topk_i8(X8, rs, Q8, qs, X16, Q16, 10, bias=bias, alpha=2.0, margin=margin)
        same = sum(len(set(a) & set(b)) for a, b in zip(r8.cpu().tolist(), r16.cpu().tolist())) / (nq * 10)
        assert same == 1.0
        assert torch.allclose(s8, s16, atol=1e-4, rtol=0)
        assert not bool((r8 % 97 == 0).any())


def test_flat_topk_fp8_matches_bf16_candidates_gpu():
    from lazzaro_amd.ops.search import flat_topk, flat_topk_fp8, quantize_e4m3
    gen = torch.Generator(device=DEV).manual_seed(3)
    N, D, nq = 1_500_000, 384, 768
    X = torch.randn(N, D, device=DEV, generator=gen)
    X = X / X.norm(dim=1, keepdim=True)
    Q = torch.randn(nq, D, device=DEV, generator=gen)
    Q = Q / Q.norm(dim=1, keepdim=True)
    X16, Q16 = X.to(torch.bfloat16), Q.to(torch.bfloat16)
    bias = -(X * X).sum(1).contiguous()
    s16, r16 = flat_topk(X16, Q16, 10, bias=bias, alpha=2.0)
    X8, Q8 = quantize_e4m3(X, 64.0), quantize_e4m3(Q, 64.0)
    margin = torch.full((nq,), 0.04, device=DEV)
    s8, r8 = flat_topk_fp8(X8, Q8, 64.0 * 64.0, X16, Q16, 10, bias=bias, alpha=2.0, margin=margin)
    same = sum(len(set(a) & set(b)) for a, b in zip(r8.cpu().tolist(), r16.cpu().tolist())) / (nq * 10)
    assert same >= 0.999 and torch.allclose(s8, s16, atol=1e-4, rtol=0)


def test_ivfpq_store_under_tenant_graph_gpu(tmp_path):
    """index="ivfpq" on the GPU: the tenant graph's store search takes IVF-PQ
    candidates (deep pool + threshold pass) re-ranked exactly in fp32."""
    import torch

    from lazzaro_amd.core.memory_system import MemorySystem
    from lazzaro_amd.core.providers import HashEmbedder, LocalLLM
    g0 = torch.Generator(device="cuda").manual_seed(0)
    C, per, d = 400, 500, 128
    cen = torch.nn.functional.normalize(torch.randn(C, d, device="cuda", generator=g0), dim=1)
    X = torch.nn.functional.normalize(cen.repeat_interleave(per, 0)
                                      + 0.5 * torch.randn(C * per, d, device="cuda", generator=g0) / d ** 0.5, dim=1)
    ms = MemorySystem(llm_provider=LocalLLM(), embedding_provider=HashEmbedder(dim=d), enable_async=False,
                      load_from_disk=False, db_dir=str(tmp_path), device="cuda", index="ivfpq",
                      index_params={"nlist": 512, "nprobe": 16, "pq_m": 32, "ivf_min_rows": 100_000})
    g = ms.graph
    g.add_nodes([f"m{i}" for i in range(len(X))], [""] * len(X), X, shard=g.shard_id("w"), stored=True)
    q = torch.nn.functional.normalize(X[:256] + 0.3 * torch.randn(256, d, device="cuda", generator=g0) / d ** 0.5,
                                      dim=1)
    _, rows = g.store_search(q, 10, "l2")
    assert g._ann is not None
    truth = torch.topk(-torch.cdist(q, X), 10, dim=1).indices
    hit = sum(len(set(a.tolist()) & set(b.tolist())) for a, b in zip(rows.cpu(), truth.cpu())) / truth.numel()
    assert hit > 0.9, hit
    ms.close()


@pytest.mark.parametrize("metric,M,C", [("l2", 300, 16), ("ip", 300, 16), ("cosine", 300, 16), ("l2", 1, 16),
                                         ("cosine", 5, 64), ("ip", 63, 40)])
def test_store_rerank_kernel_matches_torch_gpu(metric, M, C):
    """Fused fp32 re-rank (tenant.hip store_rerank_kernel; M < 64: the
    block-per-query store_rerank_block_kernel) == the torch gather / score /
    stable-sort path, with empty and masked candidates; the node-filtered
    output marks the rows whose kind is not NODE."""
    from lazzaro_amd.ops.tenant_ops import store_rerank
    gen = torch.Generator(device=DEV).manual_seed(11 + M)
    N, D, k = 5000, 384, 10
    X = torch.randn(N, D, device=DEV, generator=gen)
    sqn = (X.double() ** 2).sum(1).float()
    bias = torch.where(torch.rand(N, device=DEV, generator=gen) < 0.1, float("-inf"), 0.0)
    if metric == "l2":
        bias = bias - sqn
    Q = torch.randn(M, D, device=DEV, generator=gen)
    cand = torch.randint(0, N, (M, C), device=DEV, generator=gen)
    cand = torch.stack([torch.randperm(N, device=DEV, generator=gen)[:C] for _ in range(M)])
    cand[:, -3:] = -1
    s, r = store_rerank(Q, X, sqn, bias, cand, k, metric)
    kind = (torch.rand(N, device=DEV, generator=gen) < 0.8).to(torch.uint8)  # 1 = NODE
    s2, rn = store_rerank(Q, X, sqn, bias, cand, k, metric, kind=kind)
    assert torch.equal(s2, s)
    assert torch.equal(rn, torch.where((r >= 0) & (kind[r.clamp_min(0)] == 1), r, torch.full_like(r, -1)))
    g = TenantGraph(device=DEV)
    valid = cand >= 0
    rows = cand.clamp_min(0)
    ref = g._store_scores(Q, X[rows], sqn[rows], bias[rows], metric)
    ref = torch.where(valid, ref, torch.full_like(ref, float("-inf")))
    for q in range(M):
        pairs = sorted(((float(ref[q, c]), int(cand[q, c])) for c in range(C)
                        if cand[q, c] >= 0 and ref[q, c] != float("-inf")), key=lambda t: (-t[0], t[1]))[:k]
        got = [(float(a), int(b)) for a, b in zip(s[q].tolist(), r[q].tolist()) if b >= 0]
        assert [b for _, b in got] == [b for _, b in pairs]
        assert all(abs(a - b[0]) <= 1e-3 * (1 + abs(b[0])) for (a, _), b in zip(got, pairs))
        assert all(v == -1 for v in r[q, len(pairs):].tolist())


def test_write_emb_kernel_matches_torch_path_gpu():
    """Small inserts write every embedding column in one launch
    (tg_write_emb_kernel); the columns equal the chunked torch path's."""
    from lazzaro_amd.engine import tenant_graph as TG
    gen = torch.Generator(device=DEV).manual_seed(21)
    D = 768
    X = torch.randn(300, D, device=DEV, generator=gen) * 0.05
    X[7] = 0.0
    lists = [x.tolist() for x in X[:40].cpu()]
    lists[3] = None  # no embedding
    saved = TG.WRITE_EMB_MAX_ROWS
    gs = []
    try:
        for lim in (8192, 0):
            TG.WRITE_EMB_MAX_ROWS = lim
            g = TenantGraph(device=DEV)
            g.add_nodes([f"a{i}" for i in range(300)], [""] * 300, X, shard=g.shard_id("work"), stored=True)
            g.add_nodes([f"b{i}" for i in range(40)], [""] * 40, lists, shard=g.shard_id("work"), stored=True)
            g.add_nodes(["a5", "a9"], ["", ""], X[100:102], shard=g.shard_id("work"), stored=True)  # replace by id
            gs.append(g)
    finally:
        TG.WRITE_EMB_MAX_ROWS = saved
    k, t = gs
    n = k.n
    assert n == t.n == 340
    for col in ("emb32", "emb16", "sqn", "has_emb"):
        a, b = getattr(k, col)[:n], getattr(t, col)[:n]
        assert torch.equal(a, b), col
    # int8 copy: the same quantiser up to the last ulp of the scale
    torch.testing.assert_close(k.rs8[:n], t.rs8[:n], rtol=2e-7, atol=0)
    assert int((k.emb8[:n].int() - t.emb8[:n].int()).abs().max()) <= 1
    assert float((k.emb8[:n] != t.emb8[:n]).float().mean()) < 1e-3
    torch.testing.assert_close(k.sumsq, t.sumsq, rtol=1e-12, atol=1e-12)
    assert abs(float(k._rs8_max) - float(t._rs8_max)) <= 2e-7 * float(t._rs8_max)
    assert abs(k.max_norm_dev - t.max_norm_dev) < 1e-6


@pytest.mark.parametrize("floor", [None, 0.1])
def test_flat_topk_dual_i8_matches_bf16_dual_gpu(floor):
    """int8 dual scan (consolidation's dedupe / link candidates) == the bf16
    dual scan: same rows in both lists, scores equal to rounding."""
    from lazzaro_amd.ops.search import flat_topk_dual, flat_topk_dual_i8, quantize_i8_rows
    gen = torch.Generator(device=DEV).manual_seed(9)
    N, D, nq = 1_200_000, 768, 512
    C = torch.randn(64, D, device=DEV, generator=gen)
    X = C[torch.randint(0, 64, (N,), device=DEV, generator=gen)] + 2.0 * torch.randn(N, D, device=DEV, generator=gen)
    X = X / X.norm(dim=1, keepdim=True)
    Q = X[torch.randint(0, N, (nq,), device=DEV, generator=gen)] + 0.5 * torch.randn(nq, D, device=DEV, generator=gen) / D ** 0.5
    Q = Q / Q.norm(dim=1, keepdim=True)
    X16, Q16 = X.to(torch.bfloat16), Q.to(torch.bfloat16)
    lab = torch.randint(0, 12, (N,), device=DEV, generator=gen, dtype=torch.int32)
    ql = torch.randint(-1, 12, (nq,), device=DEV, generator=gen, dtype=torch.int32)
    bias = torch.where(torch.rand(N, device=DEV, generator=gen) < 0.05, float("-inf"), 0.0).contiguous()
    (sa, ra), (sb, rb) = flat_topk_dual(X16, Q16, 16, row_label=lab, q_label=ql, bias=bias, floor=floor)
    X8, rs = quantize_i8_rows(X16)
    Q8, qs = quantize_i8_rows(Q16)
    margin = torch.full((nq,), 0.02, device=DEV)
    (ta, ia), (tb, ib) = flat_topk_dual_i8(X8, rs, Q8, qs, X16, Q16, 16, row_label=lab, q_label=ql, bias=bias,
                                           margin=margin, floor=floor)
    for s0, r0, s1, r1 in ((sa, ra, ta, ia), (sb, rb, tb, ib)):
        assert torch.equal(r0, r1)
        fin = torch.isfinite(s0)
        assert torch.equal(fin, torch.isfinite(s1))
        assert torch.allclose(s0[fin], s1[fin], atol=1e-4, rtol=0)


def test_flat_topk_dual_i8_floor_certificate_gpu():
    """Consolidation's shape: random unit rows, a link floor far above the
    sampled k-th best, so both thresholds sit at floor - margin_rig. The
    floor certificate must fire for (almost) every query -- no exact
    fallback, no auto-mode back-off to bf16 (the relative slack
    used to push the level above the floor, so every query fell back) --
    and the lists must still equal the bf16 dual scan's for every entry
    above the floor, planted near-duplicates included."""
    from lazzaro_amd.ops.search import flat_topk_dual, flat_topk_dual_i8, quantize_i8_rows
    gen = torch.Generator(device=DEV).manual_seed(31)
    N, D, nq = 1_500_000, 768, 512
    X = torch.randn(N, D, device=DEV, generator=gen)
    X = X / X.norm(dim=1, keepdim=True)
    Q = torch.randn(nq, D, device=DEV, generator=gen)
    plant = torch.randint(0, N, (nq // 4,), device=DEV, generator=gen)  # a quarter near rows
    Q[: nq // 4] = X[plant] + 0.6 / D ** 0.5 * torch.randn(nq // 4, D, device=DEV, generator=gen)
    Q = Q / Q.norm(dim=1, keepdim=True)
    X16, Q16 = X.to(torch.bfloat16), Q.to(torch.bfloat16)
    lab = torch.randint(0, 40, (N,), device=DEV, generator=gen, dtype=torch.int32)
    ql = torch.randint(0, 40, (nq,), device=DEV, generator=gen, dtype=torch.int32)
    ql[: nq // 4] = lab[plant]
    floor = 0.5 - 0.01
    (sa, ra), (sb, rb) = flat_topk_dual(X16, Q16, 16, row_label=lab, q_label=ql, floor=floor)
    X8, rs = quantize_i8_rows(X16)
    Q8, qs = quantize_i8_rows(Q16)
    margin = torch.full((nq,), 0.02, device=DEV)
    st = []
    (ta, ia), (tb, ib) = flat_topk_dual_i8(X8, rs, Q8, qs, X16, Q16, 16, row_label=lab, q_label=ql, margin=margin,
                                           margin_rig=margin, floor=floor, floor_tol=0.005, stats=st)
    torch.cuda.synchronize()
    (oa, _), (ob, _), _cap = st
    fell_back = float(((oa != 0) | (ob != 0)).float().mean())
    assert fell_back < 0.02, fell_back
    assert int((sa[: nq // 4, 0] > 0.5).sum()) > nq // 8  # the planted rows clear the floor
    for s0, r0, s1, r1 in ((sa, ra, ta, ia), (sb, rb, tb, ib)):
        keep = s0 >= floor + 0.005
        assert torch.equal(torch.where(keep, r0, -1), torch.where(s1 >= floor + 0.005, r1, -1))
        assert torch.allclose(s0[keep], s1[keep], atol=1e-4, rtol=0)


def test_flat_topk_dual_i8_overflowing_lists_gpu():
    """Tight topics (every row of a topic at cos > 0.9 to its queries): the
    int8 dual scan's block records and per-query lists overflow, cand_select
    reads only the entries that were written, the re-score cut gathers no row
    outside the table, and the fallback returns the bf16 dual scan's lists
    for every entry above the floor (the row-sharded bench's clustered load)."""
    from lazzaro_amd.ops.search import flat_topk_dual, flat_topk_dual_i8, quantize_i8_rows
    gen = torch.Generator(device=DEV).manual_seed(23)
    N, D, nq, T_ = 2_000_000, 768, 256, 8
    C = torch.randn(T_, D, device=DEV, generator=gen)
    C = C / C.norm(dim=1, keepdim=True)
    t = torch.randint(0, T_, (N,), device=DEV, generator=gen)
    X = C[t] + 0.25 / D ** 0.5 * torch.randn(N, D, device=DEV, generator=gen)
    X = X / X.norm(dim=1, keepdim=True)
    Q = C[torch.randint(0, T_, (nq,), device=DEV, generator=gen)] + 0.25 / D ** 0.5 * torch.randn(
        nq, D, device=DEV, generator=gen)
    Q = Q / Q.norm(dim=1, keepdim=True)
    X16, Q16 = X.to(torch.bfloat16), Q.to(torch.bfloat16)
    lab = torch.randint(0, 6, (N,), device=DEV, generator=gen, dtype=torch.int32)
    ql = torch.randint(0, 6, (nq,), device=DEV, generator=gen, dtype=torch.int32)
    floor = 0.5 - 2.0 ** -7
    (sa, ra), (sb, rb) = flat_topk_dual(X16, Q16, 16, row_label=lab, q_label=ql, floor=floor)
    X8, rs = quantize_i8_rows(X16)
    Q8, qs = quantize_i8_rows(Q16)
    margin = torch.full((nq,), 0.02, device=DEV)
    st = []
    (ta, ia), (tb, ib) = flat_topk_dual_i8(X8, rs, Q8, qs, X16, Q16, 16, row_label=lab, q_label=ql, margin=margin,
                                           margin_rig=margin, floor=floor, stats=st)
    torch.cuda.synchronize()
    (oa, _), (ob, _), _cap = st
    assert bool((oa != 0).all()) and bool((ob != 0).all())  # every list overflowed: the fallback ran
    for s0, r0, s1, r1 in ((sa, ra, ta, ia), (sb, rb, tb, ib)):
        assert torch.equal(r0, r1)
        fin = torch.isfinite(s0)
        assert torch.allclose(s0[fin], s1[fin], atol=1e-4, rtol=0)


def test_zero_row_keeps_int8_error_model_gpu():
    """An embedding-less (all-zero) row quantises exactly with scale 0: the
    tenant's int8 error model (max row scale) and the scan's candidate lists
    stay as they were, and the row still surfaces where its exact score
    puts it."""
    from lazzaro_amd.engine import tenant_graph as TG
    from lazzaro_amd.ops import search as S
    saved = TG.TenantGraph.LOWP
    TG.TenantGraph.LOWP = "i8"
    try:
        g = TenantGraph(device=DEV)
        N, D = (1 << 20) + 100, 384
        gen = torch.Generator(device=DEV).manual_seed(17)
        X = torch.randn(N, D, device=DEV, generator=gen)
        X = X / X.norm(dim=1, keepdim=True)
        g.add_nodes([f"n{i}" for i in range(N)], [""] * N, X, shard=g.shard_id("work"), stored=True)
        Q = torch.randn(256, D, device=DEV, generator=gen)
        Q = Q / Q.norm(dim=1, keepdim=True)

        def cands():
            g.store_search(Q, 10, "l2")
            torch.cuda.synchronize()
            c = S._ws_cand.get(DEV, 0)[: Q.shape[0] * 4].view(torch.int32) & 0x3FFFFFFF
            return float(c.float().mean())
        smax0, c0 = float(g._rs8_max), cands()
        g.add_nodes(["zero"], [""], torch.zeros(1, D, device=DEV), shard=g.shard_id("work"), stored=True)
        r = g.row_of["zero"]
        assert float(g.rs8[r]) == 0.0 and int(g.emb8[r].abs().max()) == 0
        assert float(g._rs8_max) == smax0
        c1 = cands()
        assert c1 <= 1.2 * c0 + 2, (c0, c1)
        # L2: the zero row scores -|q|^2 = -1, above every unit row (-2 + 2<q,x> < -1 for <q,x> < 0.5)
        _, rows = g.store_search(Q, 10, "l2")
        assert bool((rows[:, 0] == r).all())
    finally:
        TG.TenantGraph.LOWP = saved


@pytest.mark.parametrize("mode,z", [("auto", 8.0), ("1", 8.0), ("1", 0.0)])
def test_store_search_i8_certificate_gpu(mode, z, monkeypatch):
    """The int8 store search in its default mode and in the exact mode
    (LOWP_EXACT=1: worst-case margin + per-query certificate) -- with z = 0
    too, where the statistical margin would keep only rows the int8 score
    alone puts above the threshold: every query's top-10 rows equal the exact
    bf16 scan's on clustered rows, for wide and narrow batches."""
    from lazzaro_amd.engine import tenant_graph as TG
    from lazzaro_amd.ops import search as S
    monkeypatch.setattr(TG.TenantGraph, "LOWP", "i8")
    monkeypatch.setattr(TG, "LOWP_MARGIN_Z", z)
    monkeypatch.setattr(TG, "LOWP_EXACT", mode)
    g = TenantGraph(device=DEV)
    N, D = (1 << 20) + 64, 256
    gen = torch.Generator(device=DEV).manual_seed(23)
    C = torch.randn(128, D, device=DEV, generator=gen)
    X = C[torch.randint(0, 128, (N,), device=DEV, generator=gen)] + 0.4 * torch.randn(N, D, device=DEV,
                                                                                     generator=gen)
    X = X / X.norm(dim=1, keepdim=True)
    g.add_nodes([f"n{i}" for i in range(N)], [""] * N, X, shard=g.shard_id("work"), stored=True)
    assert g.emb8 is not None and g.emb8.dtype == torch.int8
    for nq in (256, 5):  # the wide (speculative threshold) and the narrow int8 kernels
        Q = X[torch.randint(0, N, (nq,), device=DEV, generator=gen)] + 0.2 * torch.randn(nq, D, device=DEV,
                                                                                         generator=gen) / D ** 0.5
        Q = Q / Q.norm(dim=1, keepdim=True)
        bias = g.store_bias("l2")
        q16 = g._q16(Q)
        _, cand = g._i8_candidates(Q, q16, 16, bias, 2.0)
        _, ref = S.flat_topk(g.emb16[:g.n], q16, 16, bias=bias, alpha=2.0)
        assert torch.equal(cand[:, :10], ref[:, :10]), (nq, z)


@pytest.mark.parametrize("nq,D", [(1, 768), (7, 384), (33, 768), (127, 1024)])
def test_scan8_narrow_matches_bf16_gpu(nq, D):
    """Narrow batches (nq < 128) take the HBM-bound int8 kernel
    (scan8_narrow_kernel): the same top-10 as the bf16 scan, for one query
    and for partial 16-query tiles, with removed rows and a ragged row tail."""
    from lazzaro_amd.ops import search as S
    gen = torch.Generator(device=DEV).manual_seed(41 + nq)
    N = 1_048_583
    X = torch.randn(N, D, device=DEV, generator=gen)
    X = X / X.norm(dim=1, keepdim=True)
    Q = torch.randn(nq, D, device=DEV, generator=gen)
    Q = Q / Q.norm(dim=1, keepdim=True)
    X16, Q16 = X.to(torch.bfloat16), Q.to(torch.bfloat16)
    bias = -(X * X).sum(1).contiguous()
    bias[::101] = float("-inf")
    X8, rs = S.quantize_i8_rows(X16)
    Q8, qs = S.quantize_i8_rows(Q16)
    margin = torch.full((nq,), 0.02, device=DEV)
    s8, r8 = S.flat_topk_i8(X8, rs, Q8, qs, X16, Q16, 16, bias=bias, alpha=2.0, margin=margin)
    s16, r16 = S.flat_topk(X16, Q16, 16, bias=bias, alpha=2.0)
    assert torch.equal(r8[:, :10], r16[:, :10])
    assert torch.allclose(s8[:, :10], s16[:, :10], atol=1e-4, rtol=0)
    assert not bool((r8 % 101 == 0).any())


def test_cos_rerank64_kernel_matches_torch_gpu():
    """Consolidation's float64 candidate re-rank in one launch
    (cos_rerank64_kernel) == the torch gather / einsum / sort chain."""
    from lazzaro_amd.engine import tenant_graph as TG
    gen = torch.Generator(device=DEV).manual_seed(29)
    g = TenantGraph(device=DEV)
    N, D, M, C = 4000, 384, 300, 16
    X = torch.randn(N, D, device=DEV, generator=gen)
    g.add_nodes([f"r{i}" for i in range(N)], [""] * N, X, shard=g.shard_id("w"), stored=True)
    Q = torch.randn(M, D, device=DEV, generator=gen, dtype=torch.float64)
    Qn = Q / Q.norm(dim=1, keepdim=True)
    cand = torch.stack([torch.randperm(N, device=DEV, generator=gen)[:C] for _ in range(M)])
    cand[:, -2:] = -1
    cand[::7, 3] = cand[::7, 4]  # a duplicated row keeps both slots, in row order
    s1, r1 = g._rerank_cos(Qn, cand, 10)
    saved = TG.RERANK_KERNEL
    TG.RERANK_KERNEL = False
    try:
        s0, r0 = g._rerank_cos(Qn, cand, 10)
    finally:
        TG.RERANK_KERNEL = saved
    assert torch.equal(r1, r0)
    fin = torch.isfinite(s0)
    assert torch.equal(fin, torch.isfinite(s1))
    assert torch.allclose(s1[fin], s0[fin], atol=1e-12, rtol=0)


def test_lean_hbm_tenant_matches_full_gpu(monkeypatch):
    """LEAN_HBM: a large tenant keeps fp32 + int8 + scale only (no bf16
    copy). Store search (large and interactive batches), consolidation's dual
    and single candidate scans and the k-means pass return what the same rows
    give with the bf16 copy; the vector columns cost 4D + D + 8 bytes per row."""
    from lazzaro_amd.engine import tenant_graph as TG
    monkeypatch.setattr(TG, "LOWP_MIN_ROWS", 1 << 15)
    N, D = 70_000, 768
    gen = torch.Generator(device=DEV).manual_seed(11)
    C = torch.randn(64, D, device=DEV, generator=gen)
    X = C[torch.randint(0, 64, (N,), device=DEV, generator=gen)] + 0.7 * torch.randn(N, D, device=DEV, generator=gen)
    X = X / X.norm(dim=1, keepdim=True)
    lab = torch.randint(0, 5, (N,), device=DEV, generator=gen)

    def build():
        g = TenantGraph(device=DEV, dim=D, capacity=1 << 17)
        codes = [g.shard_id(f"s{i}") for i in range(5)]
        g.add_nodes([f"n{i}" for i in range(N)], [""] * N, X, shard=lab.cpu().int(), stored=True)
        return g, codes
    full, _ = build()
    monkeypatch.setattr(TG, "LEAN_HBM", True)
    lean, _ = build()
    assert full.emb16 is not None and not full.lean
    assert lean.emb16 is None and lean.lean and lean.emb8.dtype == torch.int8
    vec_bytes = sum(t[0].numel() * t.element_size() for t in (lean.emb32, lean.emb8, lean.rs8, lean.sqn))
    assert vec_bytes == 4 * D + D + 8
    Q = X[torch.randint(0, N, (300,), device=DEV, generator=gen)] + 0.2 * torch.randn(300, D, device=DEV,
                                                                                      generator=gen) / D ** 0.5
    Q = Q / Q.norm(dim=1, keepdim=True)
    for m in (300, 7):  # the large-batch scan and the narrow interactive one
        s1, r1 = full.store_search(Q[:m], 10)
        s2, r2 = lean.store_search(Q[:m], 10)
        assert torch.equal(r1, r2), m
        assert torch.allclose(s1, s2, atol=1e-5)
    mask = full.kind[:N] == NODE
    ql = torch.randint(0, 5, (300,), device=DEV, generator=gen)
    (a1, b1), (a2, b2) = (g.cos_topk(Q, 8, mask, dual_label=ql, min_score=0.3) for g in (full, lean))
    assert torch.equal(a1[1], a2[1]) and torch.equal(b1[1], b2[1])
    assert torch.equal(full.cos_topk(Q, 8, mask)[1], lean.cos_topk(Q, 8, mask)[1])
    hf, hl = full.cluster_pass(32, 4, 2), lean.cluster_pass(32, 4, 2)
    assert torch.equal(full.hier["fine"][:N], lean.hier["fine"][:N])
    assert lean.emb16 is None  # the pass's bf16 copy is gone


@pytest.mark.parametrize("native", [True, False])
@pytest.mark.parametrize("prune_threshold", [0.0, 0.5])
def test_consolidate_batch_incremental_components_gpu(tmp_path, monkeypatch, prune_threshold, native):
    """consolidate_batch on a tenant with many edges (the full GPU digest
    path at every run_consolidation point): the batch's incremental
    components (TenantGraph.cc_begin) give the same digest at every point,
    the same profile and the same final graph as a union-find over every
    edge at every point -- through the native segment applier
    (csrc/kernels/apply.hip: suffix-only segment ends, the incremental digest
    in C++) and through the per-segment Python path."""
    from lazzaro_amd.core import consolidation as Cn
    from lazzaro_amd.engine.tenant_graph import TenantGraph
    monkeypatch.setattr(Cn.ConsolidationMixin, "NATIVE_APPLY", native)
    nat = []
    real_run = Cn.ConsolidationMixin._native_run

    def counted(self, segs, *a, **k):
        nat.append(self.graph._cc is not None)
        return real_run(self, segs, *a, **k)
    monkeypatch.setattr(Cn.ConsolidationMixin, "_native_run", counted)
    N, D, NE, B, F = 80_000, 64, 240_000, 30, 4
    X, lab = _clustered(N, D, 64, 3, noise=1.2)
    gen = torch.Generator().manual_seed(12)
    src = torch.randint(0, N, (NE,), generator=gen, dtype=torch.int32)
    dst = torch.randint(0, N, (NE,), generator=gen, dtype=torch.int32)
    w = 0.5 + 0.5 * torch.rand(NE, generator=gen)
    facts, vecs = [], []
    for c in range(B):
        conv = []
        for f in range(F):
            v = X[int(torch.randint(0, N, (1,), generator=gen))] + 0.6 * torch.randn(D, generator=gen) / D ** 0.5
            vecs.append(v / v.norm())
            conv.append({"content": f"fact {c}.{f} about topic{(c + f) % 5}", "salience": 0.6, "topic": f"topic{f}"})
        facts.append(conv)
    V = torch.stack(vecs)
    out = {}
    real = Cn.ConsolidationMixin._rc_host
    real_begin = TenantGraph.cc_begin
    for inc in (True, False):
        digests = []

        def rec(self, cap):  # every point's digest, whichever path computed it
            digests.append([x.tolist() for x in cap["digest"].get()])
            return real(self, cap)
        monkeypatch.setattr(Cn.ConsolidationMixin, "_rc_host", rec)
        monkeypatch.setattr(TenantGraph, "CC_INCREMENTAL", inc)
        monkeypatch.setattr(time, "time", _Clock())
        ms = MemorySystem(llm_provider=LocalLLM(), embedding_provider=HashEmbedder(dim=D), enable_async=False,
                          db_dir=str(tmp_path / f"inc{int(inc)}"), device=DEV, load_from_disk=False,
                          max_buffer_size=N + 20, prune_threshold=prune_threshold, super_node_threshold=10 ** 9)
        g = ms.graph
        shards = [g.shard_id(f"topic{c}") for c in range(5)]
        g.add_nodes([f"node_{i + 1}" for i in range(N)], [f"m {i}" for i in range(N)], X.to(DEV),
                    shard=np.asarray([shards[int(c) % 5] for c in lab], dtype=np.int32),
                    sal=torch.rand(N, generator=torch.Generator().manual_seed(1)), stored=True)
        g.append_edges(src.to(DEV), dst.to(DEV), w.to(DEV), g.shard[src.to(DEV).long()], g.etype("relates_to"))
        ms.node_counter = N
        used = []
        monkeypatch.setattr(TenantGraph, "cc_begin", lambda self, *a, **k: used.append(real_begin(self, *a, **k))
                            or used[-1])
        st = ms.consolidate_batch(facts, embeddings=V.to(DEV), now=1.9e9)
        e = {k: v.cpu() for k, v in g.e.items()}
        order = np.lexsort((e["dst"].numpy(), e["src"].numpy()))
        out[inc] = (st, digests, dict(ms.profile.data), used, g.sal[: g.n].cpu().numpy(),
                    {k: v.numpy()[order] for k, v in e.items() if k in ("src", "dst", "w")})
        ms.close()
    a, b = out[True], out[False]
    assert a[3] == [True] and b[3] == [False]  # the incremental path ran (thr 0.5: the decays make many edges volatile)
    assert (True in nat) == native  # the native applier ran the partitioned batch (and only when enabled)
    assert a[0] == b[0] and a[0]["consolidations"] == B // 3 and a[0]["evicted"] > 0
    assert a[1] == b[1] and len(a[1]) == B // 3
    assert a[2] == b[2]
    assert np.array_equal(a[4], b[4])
    for k in a[5]:
        assert np.array_equal(a[5][k], b[5][k]), k


@pytest.mark.parametrize("hier", ["reference", "kmeans"])
def test_consolidate_stream_matches_batches_gpu(tmp_path, monkeypatch, hier):
    """``consolidate_stream``: batch i+1's int8 dual candidate scan runs on a
    side stream under batch i's apply and is completed against the graph
    batch i left (TenantGraph.cos_topk_finish). Three batches on a 1.2M-row
    tenant -- with facts that duplicate rows batch 1 evicts (their prefetched
    candidates are re-scanned) and facts that duplicate batch 1's own new
    facts (rows that arrived after the prefetch: re-ranked in) -- end in the
    state of three ``consolidate_batch`` calls: counts, nodes, saliences,
    access counts, edges. ``kmeans``: the k-means hierarchy re-clusters
    inside batches 1 and 2 (every 20 conversations) and batch i+1's scan
    still runs prefetched under them; the hierarchies end equal too."""
    from lazzaro_amd.engine import tenant_graph as TG
    N, D, B, F = 1_200_000, 384, 32, 6
    X, lab = _clustered(N, D, 256, 23, noise=1.6)
    sal0 = torch.rand(N, generator=torch.Generator().manual_seed(2))
    low = torch.argsort(sal0)[:64]  # the rows the first batch's eviction takes
    gen = torch.Generator().manual_seed(9)
    batches = []
    prev = []
    for b in range(3):
        facts, vecs = [], []
        for c in range(B):
            conv = []
            for f in range(F):
                kind = (c * F + f + b) % 4
                if kind == 0:
                    base = X[int(torch.randint(0, N, (1,), generator=gen))]
                elif kind == 1 and b > 0:  # a row the previous batch may have evicted
                    base = X[int(low[int(torch.randint(0, low.numel(), (1,), generator=gen))])]
                elif kind == 2 and prev:  # a fact the previous batch inserted
                    base = prev[int(torch.randint(0, len(prev), (1,), generator=gen))]
                else:
                    base = torch.randn(D, generator=gen)
                v = base + 0.01 * torch.randn(D, generator=gen) / D ** 0.5
                vecs.append(v / v.norm())
                conv.append({"content": f"fact {b}.{c}.{f}", "salience": 0.5 + 0.01 * f,
                             "topic": f"topic{(c + f) % 8}"})
            facts.append(conv)
        V = torch.stack(vecs)
        prev = list(V)
        batches.append((facts, V.to(DEV), 1.8e9 + 3600.0 * b))
    calls = {"finish": 0, "aff": 0}
    real_finish = TG.TenantGraph.cos_topk_finish
    real_cos = TG.TenantGraph._cos_topk

    def finish(self, h, k, mask):
        calls["finish"] += 1

        def cos(self_, *a, **kw):
            calls["aff"] += 1
            return real_cos(self_, *a, **kw)
        monkeypatch.setattr(TG.TenantGraph, "_cos_topk", cos)
        try:
            return real_finish(self, h, k, mask)
        finally:
            monkeypatch.setattr(TG.TenantGraph, "_cos_topk", real_cos)
    monkeypatch.setattr(TG.TenantGraph, "cos_topk_finish", finish)
    out = {}
    bg = {"n": 0}
    real_pass = TG.TenantGraph.cluster_pass

    def cluster_pass(self, *a, **kw):
        bg["n"] += bool(kw.get("background"))
        return real_pass(self, *a, **kw)
    monkeypatch.setattr(TG.TenantGraph, "cluster_pass", cluster_pass)
    # kmeans: "inline" = per-batch calls with every k-means pass in line (the
    # others run the planned batches' passes in the background)
    for mode in ("calls", "stream") + (("inline",) if hier == "kmeans" else ()):
        monkeypatch.setattr(time, "time", _Clock())
        monkeypatch.setattr(MemorySystem, "CLUSTER_BACKGROUND", mode != "inline")
        hk = {} if hier == "reference" else {"hierarchy_mode": "kmeans",
                                             "hierarchy_params": {"fine": 64, "top": 8, "every": 20, "iters": 1}}
        ms = MemorySystem(llm_provider=LocalLLM(), embedding_provider=HashEmbedder(dim=D), enable_async=False,
                          db_dir=str(tmp_path / mode), device=DEV, load_from_disk=False, max_buffer_size=N - 100,
                          super_node_threshold=10 ** 9, **hk)
        g = ms.graph
        shards = [g.shard_id(f"topic{c}") for c in range(8)]
        g.add_nodes([f"node_{i + 1}" for i in range(N)], [f"m {i}" for i in range(N)], X.to(DEV),
                    shard=np.asarray([shards[int(c) % 8] for c in lab], dtype=np.int32), sal=sal0, stored=True)
        ms.node_counter = N
        if mode in ("calls", "inline"):
            stats = [ms.consolidate_batch(f, embeddings=V, now=t) for f, V, t in batches]
        else:
            stats = list(ms.consolidate_stream(batches))
        n = g.n
        live = (g.kind[:n] == NODE).cpu().numpy()
        e = {k: v.cpu() for k, v in g.e.items()}
        order = np.lexsort((e["dst"].numpy(), e["src"].numpy()))
        out[mode] = (stats, np.nonzero(live)[0], g.sal[:n].cpu().numpy()[live], g.acc[:n].cpu().numpy()[live],
                     {k: v.numpy()[order] for k, v in e.items() if k in ("src", "dst", "w", "meta")},
                     [g.ids[r] for r in np.nonzero(live)[0][-50:]],
                     {k: v.cpu().numpy() for k, v in (getattr(g, "hier", None) or {}).items()
                      if k in ("fine", "top", "perm")})
        ms.close()
    a, b = out["calls"], out["stream"]
    assert calls["finish"] == 2  # batches 2 and 3 came from prefetched scans
    assert a[0] == b[0]
    assert sum(s["dup"] for s in a[0]) > 0 and sum(s["evicted"] for s in a[0]) > 0
    assert np.array_equal(a[1], b[1]) and np.array_equal(a[2], b[2]) and np.array_equal(a[3], b[3])
    for k in a[4]:
        assert np.array_equal(a[4][k], b[4][k]), k
    assert a[5] == b[5]
    assert a[6].keys() == b[6].keys() and all(np.array_equal(a[6][k], b[6][k]) for k in a[6])
    if hier == "kmeans":
        assert a[6], "the k-means hierarchy was built"
        assert bg["n"] >= 2, bg  # passes inside the batches ran in the background
        c = out["inline"]
        assert a[0] == c[0] and all(np.array_equal(a[i], c[i]) for i in (1, 2, 3))
        assert all(np.array_equal(a[4][k], c[4][k]) for k in a[4]) and a[5] == c[5]
        assert a[6].keys() == c[6].keys() and all(np.array_equal(a[6][k], c[6][k]) for k in a[6])
    assert calls["aff"] >= 1, calls  # some prefetched candidates lost a row to the previous batch's eviction
