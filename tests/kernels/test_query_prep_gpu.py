"""search256.hip i8_query_kernel (the int8 store search's query quantisation
+ error margin in one launch) against the torch formulation of
TenantGraph._i8_query, and the two-level partial-list merge of narrow
batches against the fp32 reference top-k."""
import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("nq", [1, 7, 300, 1024])
def test_i8_query_kernel_matches_torch(nq, monkeypatch):
    from lazzaro_amd.engine import tenant_graph as TG
    g = TG.TenantGraph(device="cuda", dim=768)
    X = torch.randn(5000, 768, device="cuda")
    X /= X.norm(dim=1, keepdim=True)
    g.add_nodes([f"n{i}" for i in range(5000)], [""] * 5000, X, shard=g.shard_id("default"), stored=True)
    if g.emb8 is None or g.emb8.dtype != torch.int8:
        pytest.skip("tenant without an int8 copy")
    Q = torch.randn(nq, 768, device="cuda")
    Q[0] = 0.0  # a zero query quantises exactly with scale 0
    q16 = g._q16(Q / Q.norm(dim=1, keepdim=True).clamp_min(1e-30))
    monkeypatch.setattr(TG, "I8_QUERY_KERNEL", True)
    monkeypatch.setattr(TG, "I8_QUERY_WIDE", True)  # (wide batches: the kernel too, not only nq < 128)
    a8, aq, am, ar = g._i8_query(q16, 2.0)
    monkeypatch.setattr(TG, "I8_QUERY_KERNEL", False)
    b8, bq, bm, br = g._i8_query(q16, 2.0)
    assert torch.equal(aq, bq) and torch.equal(a8, b8)
    assert torch.allclose(am, bm, rtol=1e-5, atol=1e-7) and float(am[0]) >= 0.0
    assert torch.allclose(ar, br, rtol=1e-5, atol=1e-7)
    assert bool((ar[1:] > am[1:]).all())  # the worst-case bound exceeds the statistical margin


@pytest.mark.parametrize("nq", [1, 3])
def test_two_level_merge_matches_one_level(nq, monkeypatch):
    """The grouped merge of a narrow batch's partial lists equals the
    single-wave merge (top-k of the union = top-k of the groups' top-k)."""
    from lazzaro_amd.ops import search as S
    torch.manual_seed(0)
    X = torch.randn(156250, 768, device="cuda").to(torch.bfloat16)
    Q = torch.randn(nq, 768, device="cuda").to(torch.bfloat16)
    nch = S._lib.lib().lzk_flat_topk_chunks(X.shape[0], nq, S.TARGET_WGS)
    assert S._merge_groups(nq, nch) > 1
    s2, i2 = S._flat_topk_lane(X, Q, 16, 16, None, None, None, 1.0, 0, None)
    monkeypatch.setattr(S, "_merge_groups", lambda nq, nch: 1)
    s1, i1 = S._flat_topk_lane(X, Q, 16, 16, None, None, None, 1.0, 0, None)
    assert torch.equal(i1, i2) and torch.equal(s1, s2)
