#!/bin/bash
# round 6 closing measurements: the driver's bench command (every section,
# measured HBM per section), then a kernel-trace window of the timed
# consolidation steps (default + persistent graph) summarised by
# tools/ktrace_window.py (device busy, time by kernel class)
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
export PYTHONPATH=$PWD${PYTHONPATH:+:$PYTHONPATH}
OUT=${OUT:-gpurun_out/r6fin}
mkdir -p $OUT
if [ -z "$NOBENCH" ]; then
  timeout -k 10 700 python bench.py --gpus 1 --steps 20 --warmup 5 > $OUT/bench.json 2> $OUT/bench.err || exit 1
fi
for cfg in default persistent; do
  A=""; [ $cfg = persistent ] && A="--prune-threshold 0"
  timeout -s KILL 400 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/kt_$cfg -o run -- python3 bench/bench_consolidate.py --steps 5 --warmup 2 $A > $OUT/${cfg}_kt.json 2> $OUT/${cfg}_kt.err || exit 1
  MS=$(python3 -c "
import json
r=None
for l in open('$OUT/${cfg}_kt.json'):
    try: d=json.loads(l)
    except Exception: continue
    if 'ms_per_step' in d: r=d
print(r['ms_per_step']*5)")
  python3 tools/ktrace_window.py /tmp/kt_$cfg/run_kernel_trace.csv $MS 5 $OUT/${cfg}_window.json > /dev/null || exit 1
  cp /tmp/kt_$cfg/run_kernel_stats.csv $OUT/${cfg}_kernel_stats.csv || exit 1
done
