"""Probe (diagnostic): the int8 / bf16 dual candidate scans on a tight-topic
table whose candidate lists overflow, one stage at a time with a device
synchronisation after each, so a failing stage names itself."""
import sys

import torch

from lazzaro_amd.ops import _lib
from lazzaro_amd.ops import search as S


def stage(name, fn):
    print("stage", name, flush=True)
    out = fn()
    torch.cuda.synchronize()
    print("  ok", name, flush=True)
    return out


def main():
    dev = torch.device("cuda")
    gen = torch.Generator(device=dev).manual_seed(23)
    N, D, nq, T_ = int(sys.argv[1]) if len(sys.argv) > 1 else 2_000_000, 768, 256, 8
    C = torch.randn(T_, D, device=dev, generator=gen)
    C = C / C.norm(dim=1, keepdim=True)
    t = torch.randint(0, T_, (N,), device=dev, generator=gen)
    X = C[t] + 0.25 / D ** 0.5 * torch.randn(N, D, device=dev, generator=gen)
    X = X / X.norm(dim=1, keepdim=True)
    Q = C[torch.randint(0, T_, (nq,), device=dev, generator=gen)] + 0.25 / D ** 0.5 * torch.randn(
        nq, D, device=dev, generator=gen)
    Q = Q / Q.norm(dim=1, keepdim=True)
    X16, Q16 = X.to(torch.bfloat16), Q.to(torch.bfloat16)
    del X
    lab = torch.randint(0, 6, (N,), device=dev, generator=gen, dtype=torch.int32)
    ql = torch.randint(0, 6, (nq,), device=dev, generator=gen, dtype=torch.int32)
    floor = 0.5 - 2.0 ** -7
    torch.cuda.synchronize()
    L = _lib.lib()
    k = 16
    kslot = L.lzk_flat_topk_kslot(k)
    Ss = max(1, min(S.CAND_STRIDE, N // max(16 * kslot, 1)))
    # ---- int8 dual, stage by stage (flat_topk_dual_i8)
    X8, rs = stage("quant_rows", lambda: S.quantize_i8_rows(X16))
    Q8, qs = stage("quant_q", lambda: S.quantize_i8_rows(Q16))
    margin = torch.full((nq,), 0.02, device=dev)
    thr_b = stage("thr_b", lambda: S._sample_threshold(X16, Q16, k, kslot, None, lab, ql, 1.0, Ss))
    thr_a = stage("thr_a", lambda: S._sample_threshold(X16, Q16, k, kslot, None, None, None, 1.0, Ss))
    fl = torch.as_tensor(floor - margin, device=dev)
    thr_a = torch.maximum(thr_a - margin, fl).contiguous()
    thr_b = torch.maximum(thr_b - margin, fl).contiguous()
    cap = max(2048, 16 * kslot * Ss)
    ca = S._cand_lists(dev, nq, cap, 0)
    cb = S._cand_lists(dev, nq, cap, 1)
    stage("dual_i8_scan+gather", lambda: S._dual_i8_template(X8, rs, Q8, qs.contiguous(), X16, None, 1.0, thr_a,
                                                             thr_b, lab, ql, kslot, Ss, cap, ca, cb))
    print("counts A", ca[0][:8].tolist(), "B", cb[0][:8].tolist(), "cap", cap, flush=True)
    need_a = torch.empty(nq, dtype=torch.int32, device=dev)
    need_b = torch.empty(nq, dtype=torch.int32, device=dev)
    stage("rescore_a", lambda: S._rescore_above_cut(X16, Q16, k, kslot, None, 1.0, margin, *ca, cap, floor=floor,
                                                    chk=(S._cert_tau(thr_a, margin, floor), k, cap + 1, need_a)))
    stage("rescore_b", lambda: S._rescore_above_cut(X16, Q16, k, kslot, None, 1.0, margin, *cb, cap, floor=floor,
                                                    chk=(S._cert_tau(thr_b, margin, floor), k, cap + 1, need_b)))
    stage("select_a", lambda: S._select_with_fallback(X16, Q16, k, kslot, None, None, None, 1.0, 0, *ca, cap,
                                                      need=need_a))
    stage("select_b", lambda: S._select_with_fallback(X16, Q16, k, kslot, None, lab, ql, 1.0, 0, *cb, cap,
                                                      need=need_b))
    # ---- bf16 dual (the reference of the test)
    stage("bf16_dual", lambda: S.flat_topk_dual(X16, Q16, k, row_label=lab, q_label=ql, floor=floor))
    errs = {n: getattr(L, f"lzk_{n}_debug_errors", lambda: None)() for n in ("search256", "search")}
    print("debug errors", errs, flush=True)
    print("PROBE OK", flush=True)


if __name__ == "__main__":
    main()
