"""Property tests (hypothesis) of the search kernels over generated shapes:
ragged row counts, query counts straddling tile edges, every supported k,
bias / tombstones / labels, and ragged tenant segments -- each case checked
against the fp32 torch reference."""
import pytest
import torch

pytestmark = pytest.mark.gpu

hyp = pytest.importorskip("hypothesis")
from hypothesis import given, settings, strategies as st  # noqa: E402

from lazzaro_amd.ops.search import _ref_topk, flat_topk, segment_topk  # noqa: E402

DEV = "cuda"


@settings(max_examples=25, deadline=None)
@given(n=st.integers(1, 3000), d=st.sampled_from([64, 128, 384, 768]), nq=st.integers(1, 300),
       k=st.sampled_from([1, 2, 3, 5, 8, 10, 16]), use_bias=st.booleans(), use_label=st.booleans(),
       seed=st.integers(0, 1 << 20))
def test_flat_topk_property(n, d, nq, k, use_bias, use_label, seed):
    g = torch.Generator(device=DEV).manual_seed(seed)
    X = torch.randn(n, d, device=DEV, generator=g).to(torch.bfloat16)
    Q = torch.randn(nq, d, device=DEV, generator=g).to(torch.bfloat16)
    b = None
    if use_bias:
        b = torch.randn(n, device=DEV, generator=g)
        b[torch.rand(n, device=DEV, generator=g) < 0.1] = float("-inf")  # tombstones
    rl = torch.randint(0, 4, (n,), device=DEV, dtype=torch.int32, generator=g) if use_label else None
    ql = torch.randint(-1, 4, (nq,), device=DEV, dtype=torch.int32, generator=g) if use_label else None
    s, i = flat_topk(X, Q, k, bias=b, row_label=rl, q_label=ql, alpha=2.0)
    rs, ri = _ref_topk(X.cpu(), Q.cpu(), k, None if b is None else b.cpu(), None if rl is None else rl.cpu(),
                       None if ql is None else ql.cpu(), 2.0)
    torch.testing.assert_close(s.cpu(), rs, atol=3e-3, rtol=1e-4)
    assert (i.cpu() == ri).float().mean() > 0.99


@settings(max_examples=20, deadline=None)
@given(sizes=st.lists(st.integers(0, 700), min_size=1, max_size=40), k=st.sampled_from([1, 4, 10, 16]),
       fp32=st.booleans(), seed=st.integers(0, 1 << 20))
def test_segment_topk_property(sizes, k, fp32, seed):
    d = 128 if fp32 else 64
    g = torch.Generator(device=DEV).manual_seed(seed)
    dt = torch.float32 if fp32 else torch.bfloat16
    big = torch.randn(sum(sizes) + 1, d, device=DEV, generator=g).to(dt)
    xs, o = [], 0
    for m in sizes:
        xs.append(big[o:o + m])
        o += m
    Q = torch.randn(len(sizes), d, device=DEV, generator=g).to(dt)
    s, i = segment_topk(xs, Q, k)
    rs, ri = segment_topk([x.cpu().float() for x in xs], Q.cpu().float(), k)
    torch.testing.assert_close(s.cpu(), rs, atol=3e-3, rtol=1e-4)
    assert (i.cpu() == ri).float().mean() > 0.99
