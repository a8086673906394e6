#!/bin/bash
# consolidation steps under rocprofv3 --kernel-trace: device time vs step time (round-5 working script)
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
export PYTHONPATH=$PWD${PYTHONPATH:+:$PYTHONPATH}
OUT=${OUT:-gpurun_out/cons_kt}
mkdir -p $OUT
for cfg in default persistent; do
  A=""; [ $cfg = persistent ] && A="--prune-threshold 0"
  timeout -s KILL 400 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/ckt_$cfg -o run -- python3 bench/bench_consolidate.py --steps 4 --warmup 2 $A > $OUT/$cfg.json 2> $OUT/$cfg.err || exit 1
  cp /tmp/ckt_$cfg/run_kernel_stats.csv $OUT/${cfg}_kernel_stats.csv
  python3 - $cfg $OUT <<'PY'
import csv, sys, json
cfg, out = sys.argv[1], sys.argv[2]
res = None
for l in open(f"{out}/{cfg}.json"):
    try:
        d = json.loads(l)
    except Exception:
        continue
    if "turns_per_s" in d:
        res = d
rows = list(csv.DictReader(open(f"/tmp/ckt_{cfg}/run_kernel_trace.csv")))
ks = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"])) for r in rows)
steps = 4
t1 = max(e for _, e in ks)
t0 = t1 - int(res["ms_per_step"] * steps * 1e6)
busy, cur_s, cur_e = 0, None, None
for s, e in ks:
    s, e = max(s, t0), min(e, t1)
    if e <= s:
        continue
    if cur_e is None or s > cur_e:
        if cur_e is not None:
            busy += cur_e - cur_s
        cur_s, cur_e = s, e
    else:
        cur_e = max(cur_e, e)
busy += (cur_e - cur_s) if cur_e else 0
json.dump({"window_ms": (t1 - t0) / 1e6, "device_busy_ms_in_window": busy / 1e6,
           "busy_frac": busy / max(t1 - t0, 1), "ms_per_step": res["ms_per_step"],
           "turns_per_s": res["turns_per_s"]}, open(f"{out}/{cfg}_busy.json", "w"))
PY
done
