"""GPU probe: flat_topk correctness vs the fp32 reference, then throughput on
N x 768 bf16 (default 10M rows) at several query batch sizes."""
import argparse
import json
import time

import torch

from lazzaro_amd.ops.search import flat_topk, _ref_topk


def check(n, d, nq, k, bias=False, label=False, seed=0):
    g = torch.Generator(device="cuda").manual_seed(seed)
    X = torch.randn(n, d, device="cuda", generator=g).to(torch.bfloat16)
    Q = torch.randn(nq, d, device="cuda", generator=g).to(torch.bfloat16)
    b = torch.randn(n, device="cuda", generator=g) if bias else None
    rl = torch.randint(0, 3, (n,), device="cuda", dtype=torch.int32, generator=g) if label else None
    ql = torch.randint(-1, 3, (nq,), device="cuda", dtype=torch.int32, generator=g) if label else None
    s, i = flat_topk(X, Q, k, bias=b, row_label=rl, q_label=ql, alpha=2.0 if bias else 1.0)
    rs, ri = _ref_topk(X, Q, k, b, rl, ql, 2.0 if bias else 1.0)
    torch.cuda.synchronize()
    ok_s = torch.allclose(s, rs, atol=1e-3, rtol=1e-4)
    match = (i == ri).float().mean().item()
    return ok_s, match


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=10_000_000)
    ap.add_argument("--d", type=int, default=768)
    ap.add_argument("--out", default="gpurun_out/probe_search.json")
    a = ap.parse_args()
    res = {"checks": [], "perf": []}
    for (n, d, nq, k, b, l) in [(1000, 64, 7, 5, False, False), (5000, 768, 130, 10, True, False),
                                (33333, 384, 257, 16, False, True), (20000, 1536, 64, 1, True, True),
                                (300, 128, 1, 3, False, False)]:
        ok, m = check(n, d, nq, k, b, l)
        res["checks"].append(dict(n=n, d=d, nq=nq, k=k, bias=b, label=l, scores_ok=ok, idx_match=m))
        print(res["checks"][-1], flush=True)
    X = torch.randn(a.n, a.d, device="cuda", dtype=torch.bfloat16)
    for nq in [1, 64, 256, 1024, 2048]:
        Q = torch.randn(nq, a.d, device="cuda", dtype=torch.bfloat16)
        flat_topk(X, Q, 10)
        torch.cuda.synchronize()
        it = 5
        t0 = time.time()
        for _ in range(it):
            flat_topk(X, Q, 10)
        torch.cuda.synchronize()
        dt = (time.time() - t0) / it
        tf = 2 * a.n * a.d * nq / dt / 1e12
        gbs = a.n * a.d * 2 / dt / 1e9
        res["perf"].append(dict(nq=nq, ms=dt * 1e3, qps=nq / dt, tflops=tf, gbps=gbs))
        print(res["perf"][-1], flush=True)
    json.dump(res, open(a.out, "w"), indent=1)


if __name__ == "__main__":
    main()
