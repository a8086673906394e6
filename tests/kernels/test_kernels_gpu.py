"""Numerics of every HIP kernel vs a plain PyTorch fp32 reference of the same
op (the CPU path of each op). Runs on the MI355X box (`pytest -m gpu`)."""
import math

import pytest
import torch

pytestmark = pytest.mark.gpu

from lazzaro_amd.ops import _lib  # noqa: E402
from lazzaro_amd.ops import encoder_ops as E  # noqa: E402
from lazzaro_amd.ops.search import _ref_topk, flat_topk  # noqa: E402

DEV = "cuda"


def test_native_library_is_loaded():
    L = _lib.lib()
    assert L is not None and _lib.available()


@pytest.mark.parametrize("n,d,nq,k,bias,label", [
    (1000, 64, 7, 5, False, False), (5000, 768, 130, 10, True, False), (33333, 384, 257, 16, False, True),
    (20000, 1536, 64, 1, True, True), (300, 128, 1, 3, False, False), (129, 64, 129, 8, True, False),
])
def test_flat_topk_matches_reference(n, d, nq, k, bias, label):
    g = torch.Generator(device=DEV).manual_seed(n)
    X = torch.randn(n, d, device=DEV, generator=g).to(torch.bfloat16)
    Q = torch.randn(nq, d, device=DEV, generator=g).to(torch.bfloat16)
    b = torch.randn(n, device=DEV, generator=g) if bias else None
    rl = torch.randint(0, 3, (n,), device=DEV, dtype=torch.int32, generator=g) if label else None
    ql = torch.randint(-1, 3, (nq,), device=DEV, dtype=torch.int32, generator=g) if label else None
    a = 2.0 if bias else 1.0
    s, i = flat_topk(X, Q, k, bias=b, row_label=rl, q_label=ql, alpha=a)
    rs, ri = _ref_topk(X.cpu(), Q.cpu(), k, None if b is None else b.cpu(),
                       None if rl is None else rl.cpu(), None if ql is None else ql.cpu(), a)
    torch.testing.assert_close(s.cpu(), rs, atol=2e-3, rtol=1e-4)
    assert (i.cpu() == ri).float().mean() > 0.995  # ulp-level ties may swap


@pytest.mark.parametrize("n,d,nq,k,bias,label", [
    (300_001, 768, 300, 10, True, False), (200_000, 384, 513, 16, False, True), (70_000, 1024, 256, 1, True, True),
    (140_000, 64, 260, 5, False, False),
])
def test_flat_topk_candidate_path(monkeypatch, n, d, nq, k, bias, label):
    """256x256 pipeline + sampled threshold + select (search256.hip) == reference."""
    monkeypatch.setattr(__import__("lazzaro_amd.ops.search", fromlist=["x"]), "SEARCH_MODE", "cand")
    monkeypatch.setattr("lazzaro_amd.ops.search.CAND_STRIDE", 16)
    g = torch.Generator(device=DEV).manual_seed(n)
    X = torch.randn(n, d, device=DEV, generator=g).to(torch.bfloat16)
    Q = torch.randn(nq, d, device=DEV, generator=g).to(torch.bfloat16)
    b = torch.randn(n, device=DEV, generator=g) if bias else None
    rl = torch.randint(0, 3, (n,), device=DEV, dtype=torch.int32, generator=g) if label else None
    ql = torch.randint(-1, 3, (nq,), device=DEV, dtype=torch.int32, generator=g) if label else None
    a = 2.0 if bias else 1.0
    s, i = flat_topk(X, Q, k, bias=b, row_label=rl, q_label=ql, alpha=a, idx_offset=5)
    rs, ri = _ref_topk(X.cpu(), Q.cpu(), k, None if b is None else b.cpu(),
                       None if rl is None else rl.cpu(), None if ql is None else ql.cpu(), a, idx_offset=5)
    torch.testing.assert_close(s.cpu(), rs, atol=2e-3, rtol=1e-4)
    assert (i.cpu() == ri).float().mean() > 0.995


def test_flat_topk_candidate_overflow_falls_back(monkeypatch):
    """All-equal scores overflow every candidate list -> lane-kernel recompute."""
    monkeypatch.setattr(__import__("lazzaro_amd.ops.search", fromlist=["x"]), "SEARCH_MODE", "cand")
    X = torch.ones(100_000, 128, device=DEV, dtype=torch.bfloat16)
    Q = torch.ones(256, 128, device=DEV, dtype=torch.bfloat16)
    s, i = flat_topk(X, Q, 4)
    assert (i.cpu() == torch.arange(4)[None, :]).all() and (s.cpu() == 128.0).all()


def test_flat_topk_tombstones_and_chunks():
    X = torch.randn(4096, 128, device=DEV).to(torch.bfloat16)
    bias = torch.zeros(4096, device=DEV)
    bias[::2] = float("-inf")
    Q = X[:5].clone()
    s, i = flat_topk(X, Q, 4, bias=bias, n_chunks=7)
    assert (i % 2 == 1).all()


def _rel(a, b):
    return ((a.float() - b.float()).norm() / b.float().norm().clamp_min(1e-6)).item()


@pytest.mark.parametrize("T,N,K,act,res", [(300, 768, 768, "none", False), (64, 2304, 768, "none", False),
                                           (257, 3072, 768, "gelu", False), (129, 768, 3072, "none", True),
                                           (1000, 384, 384, "gelu", True),
                                           # grids of >= 64 tiles of 256x256 take the 8-wave pipeline
                                           (8200, 2304, 768, "none", False), (4100, 3072, 768, "gelu", False),
                                           (11300, 768, 768, "none", True), (11001, 768, 3072, "none", True),
                                           (6000, 768, 3072, "none", True), (5000, 768, 768, "none", True),
                                           (16385, 1024, 3072, "none", True), (21000, 1024, 768, "gelu", True),
                                           # T <= 64: skinny weight-streaming kernel
                                           (1, 768, 768, "gelu", True), (17, 3072, 768, "none", False),
                                           (40, 768, 3072, "none", True), (64, 1000, 384, "gelu", False)])
def test_linear(T, N, K, act, res):
    x = torch.randn(T, K, device=DEV).to(torch.bfloat16)
    w = (torch.randn(N, K, device=DEV) * 0.05).to(torch.bfloat16)
    b = torch.randn(N, device=DEV)
    r = torch.randn(T, N, device=DEV).to(torch.bfloat16) if res else None
    y = E.linear(x, w, b, act=act, residual=r)
    yr = E.linear(x.cpu(), w.cpu(), b.cpu(), act=act, residual=None if r is None else r.cpu())
    assert _rel(y.cpu(), yr) < 1e-2


@pytest.mark.parametrize("B,S,heads,hd", [(3, 40, 12, 64), (2, 32, 4, 64), (5, 70, 12, 32), (1, 130, 16, 64)])
def test_attention(B, S, heads, hd):
    H = heads * hd
    qkv = torch.randn(B * S, 3 * H, device=DEV).to(torch.bfloat16)
    lens = torch.randint(2, S + 1, (B,), dtype=torch.int32)
    lens[0] = S
    o = E.attention(qkv, lens.to(DEV), B, S, heads).cpu().float().view(B, S, H)
    ref = E.attention(qkv.cpu(), lens, B, S, heads).float().view(B, S, H)
    for bi in range(B):
        L = int(lens[bi])
        assert _rel(o[bi, :L], ref[bi, :L]) < 1e-2


def test_layernorm_and_embed_and_pool():
    T, H = 333, 768
    x = torch.randn(T, H, device=DEV).to(torch.bfloat16)
    r = torch.randn(T, H, device=DEV).to(torch.bfloat16)
    g = torch.rand(H, device=DEV) + 0.5
    b = torch.randn(H, device=DEV)
    y = E.layernorm(x, g, b, 1e-12, residual=r)
    yr = E.layernorm(x.cpu(), g.cpu(), b.cpu(), 1e-12, residual=r.cpu())
    assert _rel(y.cpu(), yr) < 1e-2
    V, S, B = 1000, 37, 9
    we = torch.randn(V, H, device=DEV).to(torch.bfloat16)
    pe = torch.randn(64, H, device=DEV).to(torch.bfloat16)
    te = torch.randn(2, H, device=DEV).to(torch.bfloat16)
    ids = torch.randint(0, V, (B * S,), dtype=torch.int32, device=DEV)
    e = E.embed_ln(ids, S, we, pe, te, g, b)
    er = E.embed_ln(ids.cpu(), S, we.cpu(), pe.cpu(), te.cpu(), g.cpu(), b.cpu())
    assert _rel(e.cpu(), er) < 1e-2
    lens = torch.randint(1, S + 1, (B,), dtype=torch.int32)
    for mode in ("mean", "cls"):
        p32, p16 = E.pool_norm(e, lens.to(DEV), B, S, mode, out16_width=832)
        r32, r16 = E.pool_norm(er, lens, B, S, mode, out16_width=832)
        assert _rel(p32.cpu(), r32) < 1e-3
        assert torch.allclose(p32.norm(dim=1).cpu(), torch.ones(B), atol=1e-4)
        assert (p16[:, H:] == 0).all()


@pytest.mark.parametrize("model", ["tiny", "minilm-l6", "bge-base"])
def test_encoder_forward_matches_cpu(model):
    from lazzaro_amd.models.encoder import SentenceEncoder
    gpu = SentenceEncoder(model, device=DEV, seed=3)
    cpu = SentenceEncoder(model, device="cpu", seed=3)
    B, S = 6, 24
    ids = torch.randint(1000, gpu.cfg.vocab, (B, S), dtype=torch.int32)
    lens = torch.tensor([24, 20, 3, 17, 24, 9], dtype=torch.int32)
    a, _ = gpu.forward(ids, lens)
    b, _ = cpu.forward(ids, lens)
    cos = (a.cpu() * b).sum(1)
    assert (cos > 0.99).all(), cos


@pytest.mark.parametrize("dtype,D", [(torch.bfloat16, 768), (torch.float32, 384), (torch.bfloat16, 64)])
def test_segment_topk_gpu(dtype, D):
    from lazzaro_amd.ops.search import segment_topk
    g = torch.Generator(device=DEV).manual_seed(D)
    big = torch.randn(5000, D, device=DEV, generator=g).to(dtype)
    cuts = [(0, 0), (0, 1), (10, 700), (700, 5000), (123, 124), (4000, 4033)]
    xs = [big[a:b] for a, b in cuts] * 3
    Q = torch.randn(len(xs), D, device=DEV, generator=g).to(dtype)
    bias = torch.randn(5000, device=DEV, generator=g)
    bs = [bias[a:b] if b > a else bias[:1] for a, b in cuts] * 3
    s, i = segment_topk(xs, Q, 10, biases=bs, alpha=2.0)
    rs, ri = segment_topk([x.cpu().float() for x in xs], Q.cpu().float(), 10,
                          biases=[b.cpu() for b in bs], alpha=2.0)
    torch.testing.assert_close(s.cpu(), rs, atol=2e-3, rtol=1e-4)
    assert (i.cpu() == ri).float().mean() > 0.99


def test_multi_arena_search_gpu():
    import numpy as np

    from lazzaro_amd.index.arena import VectorArena, multi_arena_search
    rng = np.random.default_rng(0)
    arenas = []
    for t in range(40):
        a = VectorArena(dim=768, device=DEV)
        n = int(rng.integers(1, 400))
        a.add([f"{t}_{i}" for i in range(n)], rng.standard_normal((n, 768)).astype(np.float32))
        arenas.append(a)
    owners = [arenas[int(j)] for j in rng.integers(0, 40, 300)]
    q = rng.standard_normal((300, 768)).astype(np.float32)
    for metric in ("l2", "cosine", "ip"):
        s, r = multi_arena_search(owners, q, 5, metric)
        for j in range(0, 300, 37):
            rs, rr = owners[j].search_rows(q[j:j + 1], 5, metric)
            assert torch.equal(r[j].cpu(), rr[0].cpu()), metric
            torch.testing.assert_close(s[j].cpu(), rs[0].cpu(), atol=1e-3, rtol=1e-4)


@pytest.mark.parametrize("H,res", [(768, False), (1024, True)])
def test_layernorm_q8_matches_layernorm_then_quantize_gpu(H, res):
    """The fp8 encoder's fused LayerNorm (layernorm16_kernel Q8): its e4m3
    copy / row scales are bit-for-bit quantize_fp8_rows of its own bf16
    output, which equals layernorm's up to one bf16 rounding (the two
    instantiations may contract the affine step differently)."""
    from lazzaro_amd.ops import encoder_ops as E
    g_ = torch.Generator().manual_seed(H)
    x = (torch.randn(333, H, generator=g_) * 3).to(torch.bfloat16).to(DEV)
    r = (torch.randn(333, H, generator=g_)).to(torch.bfloat16).to(DEV) if res else None
    gam = torch.rand(H, generator=g_).to(DEV) + 0.5
    bet = torch.randn(H, generator=g_).to(DEV) * 0.1
    y, (q, sc) = E.layernorm_q8(x, gam, bet, 1e-12, residual=r)
    y0 = E.layernorm(x, gam, bet, 1e-12, residual=r)
    q0, sc0 = E.quantize_fp8_rows(y)
    assert torch.equal(sc, sc0)
    assert torch.equal(q, q0)
    d = (y.float() - y0.float()).abs()
    assert float((d <= 2 ** -7 * y0.float().abs().clamp_min(1e-30)).float().mean()) == 1.0
    assert float((d > 0).float().mean()) < 0.01


def test_quantize_fp8_rows_gpu():
    g = torch.Generator().manual_seed(11)
    x = (torch.randn(1000, 1024, generator=g) * torch.linspace(0.01, 30, 1000)[:, None]).to(torch.bfloat16)
    q, s = E.quantize_fp8_rows(x.to(DEV))
    qr, sr = E.quantize_fp8_rows(x)
    torch.testing.assert_close(s.cpu(), sr, rtol=1e-6, atol=0)
    # RNE in both, but x * (448 / amax) is formed with a hardware reciprocal on
    # the GPU: values within an ulp of a rounding boundary may land on the
    # neighbouring e4m3 code -- never further
    qg = q.cpu()
    assert (qg == qr).float().mean() > 0.995
    dg = qg.view(torch.float8_e4m3fn).float()
    dr = qr.view(torch.float8_e4m3fn).float()
    diff = (dg - dr).abs()
    assert (diff <= torch.maximum(dr.abs(), dg.abs()) * 2.0 ** -3 + 2.0 ** -9).all()


@pytest.mark.parametrize("T,N,K,act,res", [(8200, 3072, 768, "gelu", False), (300, 1024, 4096, "none", True),
                                           (64, 256, 128, "none", False), (1000, 2304, 768, "none", True)])
def test_linear_fp8_gpu(T, N, K, act, res):
    x = torch.randn(T, K, device=DEV).to(torch.bfloat16)
    w = (torch.randn(N, K, device=DEV) * 0.05).to(torch.bfloat16)
    b = torch.randn(N, device=DEV)
    r = torch.randn(T, N, device=DEV).to(torch.bfloat16) if res else None
    xq, sx = E.quantize_fp8_rows(x)
    wq, sw = E.quantize_fp8_rows(w)
    y = E.linear_fp8(xq, sx, wq, sw, b, act=act, residual=r)
    yr = E.linear_fp8(xq.cpu(), sx.cpu(), wq.cpu(), sw.cpu(), b.cpu(), act=act,
                      residual=None if r is None else r.cpu())
    assert _rel(y.cpu(), yr) < 1e-2


def test_fp8_encoder_gpu_matches_cpu():
    from lazzaro_amd.models.encoder import SentenceEncoder
    ids = torch.randint(1000, 4000, (6, 40), dtype=torch.int32)
    lens = torch.tensor([40, 33, 17, 5, 40, 1], dtype=torch.int32)
    g = SentenceEncoder("tiny", device=DEV, seed=5, precision="fp8")
    c = SentenceEncoder("tiny", device="cpu", seed=5, precision="fp8")
    eg, _ = g.forward(ids, lens)
    ec, _ = c.forward(ids, lens)
    assert ((eg.cpu() * ec).sum(1) > 0.999).all()


def test_graphed_encoder_matches_eager():
    from lazzaro_amd.core.embedders import OnDeviceEmbedder
    emb = OnDeviceEmbedder("minilm-l6", device=DEV, max_len=64)
    texts = ["I like green tea", "my sister moved to Osaka last year and teaches math", "rust"]
    ids, lens = emb.tok.encode_batch(texts, emb.max_len)
    eager, _ = emb.encoder.forward(ids, lens)
    g1, _ = emb.embed_tensor(texts)          # captured (bucket 4 x 16)
    g2, _ = emb.embed_tensor(texts[:1])      # another bucket
    assert len(emb._graphs) == 2
    torch.testing.assert_close(g1, eager, atol=1e-5, rtol=1e-5)
    torch.testing.assert_close(g2, eager[:1], atol=1e-5, rtol=1e-5)


@pytest.mark.parametrize("n,nq,k,stride,n_labels,spec_e", [
    (300_001, 300, 3, 16, None, 16.0), (150_000, 512, 10, 16, None, 16.0),
    # speculative list-B threshold (~16 expected label rows above it), and a
    # deliberately too-high one (~1 row): underflowing queries must come back
    # exact through the select's fallback
    (300_001, 300, 3, 64, 64, 16.0), (300_001, 300, 3, 64, 64, 1.0)])
def test_flat_topk_dual_gpu(monkeypatch, n, nq, k, stride, n_labels, spec_e):
    """One fused scan == the unfiltered and the label-filtered searches."""
    from lazzaro_amd.ops.search import flat_topk_dual
    monkeypatch.setattr(__import__("lazzaro_amd.ops.search", fromlist=["x"]), "SEARCH_MODE", "cand")
    monkeypatch.setattr("lazzaro_amd.ops.search.CAND_STRIDE", stride)
    monkeypatch.setattr("lazzaro_amd.ops.search.DUAL_SPEC", n_labels is not None)
    monkeypatch.setattr("lazzaro_amd.ops.search.DUAL_SPEC_E", spec_e)
    g = torch.Generator(device=DEV).manual_seed(n)
    X = torch.randn(n, 768, device=DEV, generator=g).to(torch.bfloat16)
    Q = torch.randn(nq, 768, device=DEV, generator=g).to(torch.bfloat16)
    b = torch.where(torch.rand(n, device=DEV, generator=g) < 0.05, float("-inf"), 0.0)
    rl = torch.randint(0, 64, (n,), device=DEV, dtype=torch.int32, generator=g)
    ql = torch.randint(-1, 64, (nq,), device=DEV, dtype=torch.int32, generator=g)
    (sa, ia), (sb, ib) = flat_topk_dual(X, Q, k, bias=b, row_label=rl, q_label=ql, n_labels=n_labels)
    ra = _ref_topk(X.cpu(), Q.cpu(), k, b.cpu())
    rb = _ref_topk(X.cpu(), Q.cpu(), k, b.cpu(), rl.cpu(), ql.cpu())
    for (s, i), (rs, ri) in (((sa, ia), ra), ((sb, ib), rb)):
        torch.testing.assert_close(s.cpu(), rs, atol=2e-3, rtol=1e-4)
        assert (i.cpu() == ri).float().mean() > 0.995


def test_packed_varlen_encoder_gpu():
    from lazzaro_amd.models.encoder import SentenceEncoder
    enc = SentenceEncoder("bge-base", device=DEV, seed=1)
    ids = torch.randint(1000, 30000, (37, 40), dtype=torch.int32)
    lens = torch.randint(2, 41, (37,), dtype=torch.int32)
    lens[0] = 40
    for b in range(37):
        ids[b, lens[b]:] = 0
    a, a16 = enc.forward(ids, lens, pad_to=768, packed=False)
    b, b16 = enc.forward(ids, lens, pad_to=768, packed=True)
    assert ((a * b).sum(1) > 0.9999).all()
    assert torch.equal(a16[:, 768:], b16[:, 768:]) if a16.shape[1] > 768 else True


def test_attention_packed_gpu():
    B, heads, hd = 5, 12, 64
    H = heads * hd
    lens = torch.tensor([40, 3, 33, 64, 1], dtype=torch.int32)
    cu = torch.zeros(B + 1, dtype=torch.int32)
    cu[1:] = torch.cumsum(lens, 0)
    qkv = torch.randn(int(cu[-1]), 3 * H, device=DEV).to(torch.bfloat16)
    o = E.attention(qkv, lens.to(DEV), B, int(lens.max()), heads, cu=cu.to(DEV))
    ref = E.attention(qkv.cpu(), lens, B, int(lens.max()), heads, cu=cu)
    assert _rel(o.cpu(), ref) < 1e-2


@pytest.mark.parametrize("opt", [100, 8, 16, 24, 32, 48, 40, 56])
@pytest.mark.parametrize("n,d,nq", [(200_000, 768, 512), (150_000, 64, 300), (120_000, 192, 256),
                                    (90_001, 128, 257)])
def test_cand_schedule_variants(monkeypatch, opt, n, d, nq):
    """Every main-loop / epilogue schedule of the persistent candidate kernel
    (lzk_g256.h body / body2, cross-tile prefetch, column prefilter) returns
    the reference top-k, for even and odd K-tile counts (d=64, 192: KS odd)."""
    import ctypes
    L = _lib.lib()
    L.lzk_set_g256_opt.argtypes = [ctypes.c_int]
    L.lzk_set_cand_persist.argtypes = [ctypes.c_int]
    monkeypatch.setattr(__import__("lazzaro_amd.ops.search", fromlist=["x"]), "SEARCH_MODE", "cand")
    monkeypatch.setattr("lazzaro_amd.ops.search.CAND_STRIDE", 16)
    g = torch.Generator(device=DEV).manual_seed(n + d + opt)
    X = torch.randn(n, d, device=DEV, generator=g).to(torch.bfloat16)
    Q = torch.randn(nq, d, device=DEV, generator=g).to(torch.bfloat16)
    L.lzk_set_cand_persist(1)
    L.lzk_set_g256_opt(opt)
    try:
        s, i = flat_topk(X, Q, 10)
    finally:
        L.lzk_set_g256_opt(-1)
    rs, ri = _ref_topk(X.cpu(), Q.cpu(), 10)
    torch.testing.assert_close(s.cpu(), rs, atol=2e-3, rtol=1e-4)
    assert (i.cpu() == ri).float().mean() > 0.995


@pytest.mark.parametrize("T,H,res", [(1, 384, True), (17, 768, False), (4097, 768, True), (333, 1024, True),
                                     (70, 1000, False)])
def test_layernorm_shapes(T, H, res):
    """Rows-per-wave LayerNorm: partial last wave, every NC, with/without residual."""
    x = torch.randn(T, H, device=DEV).to(torch.bfloat16)
    r = torch.randn(T, H, device=DEV).to(torch.bfloat16) if res else None
    g = torch.rand(H, device=DEV) + 0.5
    b = torch.randn(H, device=DEV)
    y = E.layernorm(x, g, b, 1e-12, residual=r)
    yr = E.layernorm(x.cpu(), g.cpu(), b.cpu(), 1e-12, residual=None if r is None else r.cpu())
    assert _rel(y.cpu(), yr) < 1e-2


def test_concurrent_streams_do_not_share_workspaces():
    """Searches issued on two HIP streams at once (retrieval beside background
    consolidation) each get their own scratch lists."""
    g = torch.Generator(device=DEV).manual_seed(11)
    X1 = torch.randn(200_000, 256, device=DEV, generator=g).to(torch.bfloat16)
    X2 = torch.randn(150_000, 256, device=DEV, generator=g).to(torch.bfloat16)
    Q1 = torch.randn(3, 256, device=DEV, generator=g).to(torch.bfloat16)
    Q2 = torch.randn(5, 256, device=DEV, generator=g).to(torch.bfloat16)
    s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()
    torch.cuda.synchronize()
    outs = []
    for _ in range(4):
        with torch.cuda.stream(s1):
            a = flat_topk(X1, Q1, 10)
        with torch.cuda.stream(s2):
            b = flat_topk(X2, Q2, 10)
        outs.append((a, b))
    torch.cuda.synchronize()
    ra = _ref_topk(X1.cpu(), Q1.cpu(), 10)
    rb = _ref_topk(X2.cpu(), Q2.cpu(), 10)
    for (sa, ia), (sb, ib) in outs:
        torch.testing.assert_close(sa.cpu(), ra[0], atol=2e-3, rtol=1e-4)
        torch.testing.assert_close(sb.cpu(), rb[0], atol=2e-3, rtol=1e-4)
        assert (ia.cpu() == ra[1]).float().mean() > 0.99 and (ib.cpu() == rb[1]).float().mean() > 0.99


def test_forward_streams_matches_forward():
    """Two-stream sub-batch forward (the bench's embed path) == one forward,
    on a batch large enough for the 256x256 GEMM paths."""
    from lazzaro_amd.models.encoder import SentenceEncoder
    enc = SentenceEncoder("bge-base", device=DEV, seed=2)
    g = torch.Generator().manual_seed(5)
    B = 1024
    ids = torch.randint(1000, 30000, (B, 32), dtype=torch.int32, generator=g)
    lens = torch.randint(12, 27, (B,), dtype=torch.int32, generator=g)
    for b in range(B):
        ids[b, lens[b]:] = 0
    a32, a16 = enc.forward(ids, lens, pad_to=768)
    b32, b16 = enc.forward_streams(ids, lens, pad_to=768, parts=2)
    torch.cuda.synchronize()
    assert ((a32 * b32).sum(1) > 0.9999).all()
    assert torch.equal(a16, b16) or (a16.float() - b16.float()).abs().max() < 1e-2


@pytest.mark.parametrize("T", [48, 64 * 5, 6144])
def test_gelu_polynomial_extremes(T):
    """The FMA-only GELU (odd polynomial erf, exact saturation) over the whole
    fp32 range through the three GEMM paths (skinny, 128x128, 256x256 from 64
    tiles): identity weights make the GEMM exact, so the output is GELU(x)."""
    from lazzaro_amd.ops import encoder_ops as E
    g = torch.Generator().manual_seed(3)
    K = 768
    x = torch.cat([torch.linspace(-8, 8, T * K // 2), (torch.rand(T * K - T * K // 2, generator=g) - 0.5) * 600])
    x = x[torch.randperm(x.numel(), generator=g)].view(T, K).to(torch.bfloat16)
    w = torch.eye(K, dtype=torch.bfloat16)
    b = torch.zeros(K)
    y = E.linear(x.to(DEV), w.to(DEV), b.to(DEV), act="gelu").float().cpu()
    ref = torch.nn.functional.gelu(x.double()).float()
    tol = 1e-4 + ref.abs() * 2.0 ** -8
    assert ((y - ref).abs() <= tol).all(), float((y - ref).abs().max())


@pytest.mark.parametrize("T,N,K,res", [(5000, 768, 3072, True), (22585, 768, 768, True), (700, 1024, 4096, False)])
def test_linear_split2(T, N, K, res):
    """Split-K pair: ya + yb == x @ w.T + b (+ r), each half from its K range."""
    g = torch.Generator().manual_seed(T)
    x = torch.randn(T, K, generator=g).to(torch.bfloat16)
    w = (torch.randn(N, K, generator=g) * 0.05).to(torch.bfloat16)
    b = torch.randn(N, generator=g)
    r = torch.randn(T, N, generator=g).to(torch.bfloat16) if res else None
    ya, yb = E.linear_split2(x.to(DEV), w.to(DEV), b.to(DEV), residual=r.to(DEV) if res else None)
    h = K // 2
    ra = x[:, :h].float() @ w[:, :h].float().T + b
    if res:
        ra = ra + r.float()
    rb = x[:, h:].float() @ w[:, h:].float().T
    for y, ref in ((ya, ra), (yb, rb)):
        y = y.float().cpu()
        assert float((y - ref).norm() / ref.norm()) < 4e-3
    full = x.float() @ w.float().T + b + (r.float() if res else 0)
    s = ya.float().cpu() + yb.float().cpu()
    assert float((s - full).norm() / full.norm()) < 4e-3


def test_split_k_forward_matches():
    """The encoder forward with the split-K O / FFN2 projections (+ LN of the
    two halves) == the single-GEMM forward."""
    from lazzaro_amd.models.encoder import SentenceEncoder
    enc = SentenceEncoder("bge-base", device=DEV, seed=4)
    g = torch.Generator().manual_seed(9)
    B = 1024
    ids = torch.randint(1000, 30000, (B, 32), dtype=torch.int32, generator=g)
    lens = torch.randint(12, 33, (B,), dtype=torch.int32, generator=g)
    for i in range(B):
        ids[i, lens[i]:] = 0
    old = SentenceEncoder.SPLITK
    try:
        SentenceEncoder.SPLITK = 0
        a, _ = enc.forward(ids, lens, pad_to=768)
        SentenceEncoder.SPLITK = 2
        b, _ = enc.forward(ids, lens, pad_to=768)
    finally:
        SentenceEncoder.SPLITK = old
    assert ((a * b).sum(1) > 0.9995).all(), float((a * b).sum(1).min())


@pytest.mark.parametrize("k", [1, 4, 10, 16, 32])
def test_cross_rank_merge_kernel_matches_sort_merge(k):
    """K2 across ranks: topk_merge64_kernel vs the two-argsort merge on the CPU
    (64-bit global ids, tied scores, empty slots, lists from 8 'ranks')."""
    from lazzaro_amd.parallel.sharded import merge_topk

    g = torch.Generator().manual_seed(k)
    nq, world, kk = 300, 8, 32
    s = torch.randn(nq, world * kk, generator=g)
    s[:, ::7] = 0.25  # ties broken by id
    ids = torch.randperm(nq * world * kk, generator=g).view(nq, -1) * 1000003 + (1 << 33)
    empty = torch.rand(nq, world * kk, generator=g) < 0.2
    s[empty] = float("-inf")
    ids[empty] = -1
    rs, ri = merge_topk(s, ids, k)
    gs, gi = merge_topk(s.cuda(), ids.cuda(), k)
    assert torch.equal(ri, gi.cpu())
    assert torch.equal(rs, gs.cpu())
