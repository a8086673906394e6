"""Kernel time inside the timed window of a ``rocprofv3 --kernel-trace`` run.

usage: python tools/ktrace_window.py <run_kernel_trace.csv> <window_ms> <steps> [out.json]

The window is the last ``window_ms`` before the last kernel ends (a bench's
timed steps, ``ms_per_step * steps``). Prints the device-busy fraction of the
window (union of kernel intervals), the per-step kernel time of the top
kernels, and how much of the device time is ATen (``at::native`` /
``rocprim`` / ``Cijk_`` library kernels) vs this repo's HIP kernels.
"""
import csv
import json
import sys
from collections import defaultdict


def classify(name: str) -> str:
    if "at::native" in name or "rocprim" in name or "at::cuda" in name:
        return "aten"
    if name.startswith("Cijk_") or "Tensile" in name:
        return "library_gemm"
    if name.startswith("__amd_rocclr"):
        return "copy_fill"
    return "lzk"


def main():
    path, window_ms, steps = sys.argv[1], float(sys.argv[2]), int(sys.argv[3])
    rows = list(csv.DictReader(open(path)))
    ks = [(int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]) for r in rows]
    ks.sort()
    t1 = max(e for _, e, _ in ks)
    t0 = t1 - int(window_ms * 1e6)
    per = defaultdict(lambda: [0, 0])
    cls = defaultdict(int)
    busy, cs, ce = 0, None, None
    for s, e, n in ks:
        s, e = max(s, t0), min(e, t1)
        if e <= s:
            continue
        per[n][0] += e - s
        per[n][1] += 1
        cls[classify(n)] += e - s
        if ce is None or s > ce:
            if ce is not None:
                busy += ce - cs
            cs, ce = s, e
        else:
            ce = max(ce, e)
    busy += (ce - cs) if ce is not None else 0
    tot = sum(v[0] for v in per.values())
    top = sorted(per.items(), key=lambda kv: -kv[1][0])[:40]
    res = {
        "window_ms": window_ms, "steps": steps,
        "device_busy_ms_per_step": busy / 1e6 / steps,
        "busy_frac": busy / max(t1 - t0, 1),
        "kernel_ms_per_step": tot / 1e6 / steps,
        "launches_per_step": sum(v[1] for v in per.values()) / steps,
        "by_class_ms_per_step": {k: v / 1e6 / steps for k, v in cls.items()},
        "by_class_frac_of_device_time": {k: v / max(tot, 1) for k, v in cls.items()},
        "top": [{"ms_per_step": v[0] / 1e6 / steps, "n_per_step": v[1] / steps, "kernel": n[:160]} for n, v in top],
    }
    # the long kernels of the last step in time order (start offset in the
    # step, duration, queue): where the step's critical path goes
    t_step = t1 - int(window_ms / steps * 1e6)
    qcol = next((c for c in ("Queue_Id", "Stream_Id", "Queue_ID") if rows and c in rows[0]), None)
    tl = []
    for r in rows:
        s_, e_ = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        if e_ > t_step and (e_ - s_) >= 200_000:
            tl.append({"t_ms": round((s_ - t_step) / 1e6, 3), "dur_ms": round((e_ - s_) / 1e6, 3),
                       "q": r.get(qcol) if qcol else None, "kernel": r["Kernel_Name"][:70]})
    res["last_step_long_kernels"] = sorted(tl, key=lambda x: x["t_ms"])
    js = json.dumps(res, indent=1)
    if len(sys.argv) > 4:
        open(sys.argv[4], "w").write(js)
    print(js)


if __name__ == "__main__":
    main()
