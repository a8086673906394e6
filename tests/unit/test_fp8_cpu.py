"""fp8 (OCP e4m3) projection path on CPU: quantisation round trip and the
fp8 encoder's agreement with the bf16 encoder."""
import torch

from lazzaro_amd.models.encoder import SentenceEncoder
from lazzaro_amd.ops import encoder_ops as E


def test_quantize_rows_roundtrip():
    x = torch.randn(37, 256) * torch.linspace(0.01, 10, 37)[:, None]
    q, s = E.quantize_fp8_rows(x.to(torch.bfloat16))
    assert q.dtype == torch.uint8 and s.shape == (37,)
    xd = E.dequantize_fp8_rows(q, s)
    rel = ((xd - x.to(torch.bfloat16).float()).norm(dim=1) / x.norm(dim=1)).max()
    assert rel < 0.05  # e4m3: 3 mantissa bits
    assert (q.view(torch.float8_e4m3fn).float().abs().amax(dim=1) <= 448).all()


def test_linear_fp8_cpu_matches_dequantised_reference():
    g = torch.Generator().manual_seed(0)
    x = torch.randn(20, 256, generator=g).to(torch.bfloat16)
    w = (torch.randn(64, 256, generator=g) * 0.05).to(torch.bfloat16)
    b = torch.randn(64, generator=g)
    xq, sx = E.quantize_fp8_rows(x)
    wq, sw = E.quantize_fp8_rows(w)
    y = E.linear_fp8(xq, sx, wq, sw, b, act="gelu")
    ref = torch.nn.functional.gelu(E.dequantize_fp8_rows(xq, sx) @ E.dequantize_fp8_rows(wq, sw).T + b)
    torch.testing.assert_close(y.float(), ref, atol=2e-2, rtol=2e-2)


def test_fp8_encoder_close_to_bf16():
    ids = torch.randint(1000, 4000, (3, 16), dtype=torch.int32)
    lens = torch.tensor([16, 9, 4], dtype=torch.int32)
    a = SentenceEncoder("tiny", seed=3)
    b = SentenceEncoder("tiny", seed=3, precision="fp8")
    ea, _ = a.forward(ids, lens)
    eb, _ = b.forward(ids, lens)
    cos = (ea * eb).sum(1)
    assert (cos > 0.98).all(), cos
