"""Time the native batch planner (_lzrt.plan_batch) on one batch's dumped
inputs (LZK_DUMP_PLAN=path:N on a GPU run). The planner's collective
callbacks (exact fallback, super-node means) are replaced by stubs that
record whether they were called. usage: python tools/plan_bench.py inputs.npz [reps]"""
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    from lazzaro_amd.store.colstore import _rt
    z = np.load(sys.argv[1], allow_pickle=False)
    reps = int(sys.argv[2]) if len(sys.argv) > 2 else 10
    args = {k: z[k] for k in z.files if k != "_scalars"}
    args.update(json.loads(str(z["_scalars"])))
    calls = {"fallback": 0, "super_cos": 0}
    K = args["gs"].shape[1]

    def fallback(j, evicted, same_shard):
        calls["fallback"] += 1
        return np.full(K, -np.inf), np.full(K, -1, np.int64)

    def super_cos(children, new_facts):
        calls["super_cos"] += 1
        return np.full(args["S"].shape[0], -np.inf), 1.0
    def pre_members(code):
        calls["pre_members"] = calls.get("pre_members", 0) + 1
        return np.zeros(0, np.int64)
    args.update(fallback=fallback, super_cos=super_cos, pre_members=pre_members)
    rt = _rt()
    out = rt.plan_batch(dict(args))
    ts = []
    for _ in range(reps):
        t0 = time.perf_counter()
        rt.plan_batch(dict(args))
        ts.append(time.perf_counter() - t0)
    ts.sort()
    print(json.dumps({"facts": int(args["S"].shape[0]), "rows": int(len(args["rows"])),
                      "segments": len(out["segments"]), "ms_p50": round(ts[len(ts) // 2] * 1e3, 3),
                      "ms_min": round(ts[0] * 1e3, 3), "callbacks": calls, "stats": out["stats"]}))


if __name__ == "__main__":
    main()
