"""Union-find pass A/B on the consolidation bench's graph shape (10M rows,
20M random edges): atomic (agent-scope) vs cached parent loads, and the
number of union stages. Checks every variant's labels equal the default's."""
import json
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    from lazzaro_amd.ops import graph_ops as G
    n = int(os.environ.get("NODES", 10_000_000))
    ne = int(os.environ.get("EDGES", 20_000_000))
    dev = torch.device("cuda", 0)
    gen = torch.Generator(device=dev).manual_seed(8)
    src = torch.randint(0, n, (ne,), device=dev, generator=gen).int()
    dst = torch.randint(0, n, (ne,), device=dev, generator=gen).int()
    junk = torch.empty(1 << 29, dtype=torch.float32, device=dev)

    def t(cold, reps=7):
        G.connected_components(src, dst, n)
        ts = []
        for _ in range(reps):
            if cold:
                junk.fill_(1.0)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            G.connected_components(src, dst, n)
            torch.cuda.synchronize()
            ts.append((time.perf_counter() - t0) * 1e3)
        return round(sorted(ts)[len(ts) // 2], 3)

    ref = G.connected_components(src, dst, n).clone()
    for plain in (False, True):
        for stages in (0, 1, 4, 16):
            G.UF_PLAIN, G.UF_STAGES = plain, stages
            lab = G.connected_components(src, dst, n)
            row = {"plain": plain, "stages": stages, "equal": bool(torch.equal(lab, ref)),
                   "warm_ms": t(False), "cold_ms": t(True)}
            print(json.dumps(row), flush=True)


if __name__ == "__main__":
    main()
