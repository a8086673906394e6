#!/bin/bash
# round-5 working script: kernel trace of the headline loop (one plain process)
export TMPDIR=/tmp
OUT=${OUT:-gpurun_out/prof_head}
mkdir -p $OUT
Q="--consolidate-steps 0 --sharded-steps 0 --routed-steps 0 --global-batch 0 --no-launch --steps 10 --warmup 2 --prewarm-s 1 --recall-queries 64"
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/prof_head -o run -- python3 bench.py $Q > $OUT/bench.json 2> $OUT/bench.err || exit 1
find /tmp/prof_head -name "*kernel_stats.csv" -exec cp {} $OUT/ \;
python3 - "$OUT" <<'PY'
import csv, glob, os, sys
out = sys.argv[1]
tr = glob.glob("/tmp/prof_head/**/*kernel_trace.csv", recursive=True)
rows = list(csv.DictReader(open(tr[0])))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
# the timed loop is the last ~10 steps before the recall check: keep the last 40% of kernels by time window
t0, t1 = int(rows[0]["Start_Timestamp"]), int(rows[-1]["End_Timestamp"])
with open(os.path.join(out, "trace_tail.csv"), "w") as f:
    w = csv.writer(f)
    w.writerow(["start_ns", "dur_ns", "name"])
    for r in rows[-20000:]:
        w.writerow([int(r["Start_Timestamp"]) - t0, int(r["End_Timestamp"]) - int(r["Start_Timestamp"]), r["Kernel_Name"][:160]])
PY
