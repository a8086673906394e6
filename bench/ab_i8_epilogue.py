"""Interleaved A/B of the int8 scan's candidate epilogue on the headline's
store search (10M x 768 random unit rows, 1024 random unit queries, k = 10,
L2): OPT 24 (every int32 sum converted to float, then the float column
prefilter) vs the default (OPT bit 6: the prefilter on the int32 sums, a
column converted only when it survives). Also the dual (consolidation) scan
is switched by the same build. Prints one JSON line: per-round ms of each
variant and whether both return identical rows and scores."""
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    from lazzaro_amd.engine.tenant_graph import TenantGraph
    from lazzaro_amd.ops import _lib

    dev = torch.device("cuda", 0)
    N, D, nq = int(os.environ.get("AB_ROWS", 10_000_000)), 768, int(os.environ.get("AB_Q", 1024))
    g = TenantGraph(device=dev)
    g._set_dim(D)
    g.reserve(N)
    gen = torch.Generator(device=dev).manual_seed(1)
    code = g.shard_id("work")
    for r0 in range(0, N, 1 << 20):
        r1 = min(N, r0 + (1 << 20))
        v = torch.randn(r1 - r0, D, device=dev, generator=gen)
        g.add_nodes([f"n{i}" for i in range(r0, r1)], [""] * (r1 - r0), v / v.norm(dim=1, keepdim=True),
                    shard=code, stored=True)
    Q = torch.randn(nq, D, device=dev, generator=gen)
    Q = Q / Q.norm(dim=1, keepdim=True)
    L = _lib.lib()
    reps = int(os.environ.get("AB_REPS", "20"))
    out = {"rows": N, "queries": nq, "reps": reps, "rounds": []}
    res = {}
    for rnd in range(3):
        row = {}
        for name, opt in (("float_prefilter", 24), ("int_prefilter", -1)):
            L.lzk_set_i8_opt(opt)
            for _ in range(2):
                r = g.store_search(Q, 10, "l2")
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(reps):
                r = g.store_search(Q, 10, "l2")
            torch.cuda.synchronize()
            row[name] = round((time.perf_counter() - t0) / reps * 1e3, 3)
            res[name] = r
        out["rounds"].append(row)
        print(json.dumps(row), flush=True)
    L.lzk_set_i8_opt(-1)
    a, b = res["float_prefilter"], res["int_prefilter"]
    out["same_rows"] = bool(torch.equal(a[1], b[1]))
    out["same_scores"] = bool(torch.equal(a[0], b[0]))
    for k in ("float_prefilter", "int_prefilter"):
        out[k + "_ms_min"] = min(r[k] for r in out["rounds"])
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
