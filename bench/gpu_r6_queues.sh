#!/bin/bash
# round 6: does the consolidation stream overlap depend on the HW queue count? (A/B GPU_MAX_HW_QUEUES)
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
export PYTHONPATH=$PWD${PYTHONPATH:+:$PYTHONPATH}
OUT=${OUT:-gpurun_out/r6q}
mkdir -p $OUT
for q in 4 8 4 8; do
  GPU_MAX_HW_QUEUES=$q timeout -k 10 300 python bench/bench_consolidate.py --steps 6 --warmup 2 > $OUT/q$q.json 2>> $OUT/q$q.err || exit 1
  grep turns_per_s $OUT/q$q.json | cut -c1-120 >> $OUT/summary.txt
done
timeout -s KILL 300 rocprofv3 --kernel-trace --output-format csv -d /tmp/ktq -o run -- python3 bench/bench_consolidate.py --steps 2 --warmup 1 > $OUT/kt.json 2> $OUT/kt.err || exit 1
head -1 /tmp/ktq/run_kernel_trace.csv > $OUT/kt_header.txt
python3 - <<'PY' > $OUT/kt_streams.txt
import csv
rows = list(csv.DictReader(open("/tmp/ktq/run_kernel_trace.csv")))
keys = [k for k in rows[0] if "Queue" in k or "Stream" in k or "Thread" in k or "Agent" in k]
print(keys)
seen = {}
for r in rows[-4000:]:
    n = r["Kernel_Name"][:50]
    kk = tuple(r[k] for k in keys)
    seen.setdefault((n, kk), 0)
    seen[(n, kk)] += 1
for (n, kk), c in sorted(seen.items(), key=lambda x: -x[1])[:60]:
    print(c, kk, n)
PY
