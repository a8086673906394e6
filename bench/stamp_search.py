"""Diagnostic: per-tile phase cycles of the persistent candidate kernel from
the s_memtime stamps of the OPT-bit-8 build (search256.hip): first-wait,
K loop, epilogue+prologue issue. 10M x 768 x 1024 queries. Prints JSON."""
import ctypes
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from lazzaro_amd.ops import _lib  # noqa: E402
from lazzaro_amd.ops.search import flat_topk  # noqa: E402

L = _lib.lib()
L.lzk_set_g256_opt.argtypes = [ctypes.c_int]
L.lzk_set_stamp_buffer.argtypes = [ctypes.c_void_p]


def main():
    n, d, nq = 10_000_000, 768, 1024
    g = torch.Generator(device="cuda").manual_seed(0)
    X = torch.empty(n, d, device="cuda", dtype=torch.bfloat16)
    for r0 in range(0, n, 1 << 20):
        x = torch.randn(min(1 << 20, n - r0), d, device="cuda", generator=g)
        X[r0:r0 + x.shape[0]] = torch.nn.functional.normalize(x, dim=1).to(torch.bfloat16)
    Q = torch.nn.functional.normalize(torch.randn(nq, d, device="cuda", generator=g), dim=1).to(torch.bfloat16)
    nt = L.lzk_stamp_tiles()
    buf = torch.zeros(256 * nt * 4, dtype=torch.int64, device="cuda")
    L.lzk_set_stamp_buffer(buf.data_ptr())
    out = {}
    for opt in [int(v) for v in os.environ.get("STAMP_OPTS", "280").split(",")]:
        L.lzk_set_g256_opt(opt)
        for _ in range(3):
            flat_topk(X, Q, 10)
        torch.cuda.synchronize()
        out[opt] = phases(buf.view(256, nt, 4).cpu().numpy().astype(np.int64), d)
    L.lzk_set_g256_opt(-1)
    L.lzk_set_stamp_buffer(None)
    print(json.dumps(out), flush=True)


def phases(st, d):
    st = st[:, 2:, :]  # skip the first two tiles (pipeline start)
    wait = st[:, :, 1] - st[:, :, 0]
    loop = st[:, :, 2] - st[:, :, 1]
    epi = st[:, :, 3] - st[:, :, 2]
    tile = np.diff(st[:, :, 0], axis=1)
    q = lambda a: {"p10": int(np.percentile(a, 10)), "p50": int(np.median(a)), "p90": int(np.percentile(a, 90))}
    ideal = (d // 64) * 2 * 64 * 16  # MFMA cycles per SIMD per tile (2 waves x 64 MFMA x 16 cyc per K-tile)
    return {"unit": "s_memtime ticks", "first_wait": q(wait), "k_loop": q(loop),
            "epilogue_and_prologue_issue": q(epi), "tile_period": q(tile), "ideal_mfma_cycles_per_tile": ideal}


if __name__ == "__main__":
    main()
