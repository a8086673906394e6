"""The certificate level of the low-precision candidate scans
(ops/search.py _cert_tau): a threshold clamped to floor - margin_rig is
certified by the floor (level exactly -inf, which the re-score kernel tests
for), anything above keeps a finite level with its relative slack (ADVICE r5:
the slack used to be added before the floor test, and nan_to_num turned -inf
into -FLT_MAX, so the floor certificate never fired)."""
import torch

from lazzaro_amd.ops.search import _cert_tau


def test_floor_clamped_threshold_is_certified():
    m = torch.full((5,), 0.02)
    floor = 0.49
    fl = torch.as_tensor(floor - m, dtype=torch.float32)
    thr = torch.maximum(torch.tensor([0.1, 0.2, 0.48, float("nan"), 0.4]), fl)
    t = _cert_tau(thr, m, floor, 0.005)
    assert torch.isneginf(t[[0, 1, 3, 4]]).all()  # (exactly -inf, not -FLT_MAX)
    assert torch.isfinite(t[2]) and float(t[2]) > 0.5  # above the floor: a real level, slack added


def test_no_floor_keeps_level_and_default_tolerance_is_rounding_only():
    m = torch.full((2,), 0.02)
    t = _cert_tau(torch.tensor([0.3, float("-inf")]), m)
    assert float(t[0]) > 0.32 and torch.isneginf(t[1])
    # floor_tol 0: a level a hair above the floor is not certified
    t = _cert_tau(torch.tensor([0.4701]), m[:1], 0.49, 0.0)
    assert torch.isfinite(t).all()
