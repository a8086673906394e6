#!/bin/bash
# round 6: consolidation benches (default + persistent), untraced then traced + kernel trace
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
export PYTHONPATH=$PWD${PYTHONPATH:+:$PYTHONPATH}
OUT=${OUT:-gpurun_out/r6cons2}
mkdir -p $OUT
if [ -n "$TESTK" ]; then
  timeout -k 10 600 python -u -m pytest tests/unit/test_consolidate_batch_exact.py tests/kernels/test_tenant_engine_gpu.py \
    -m gpu -x -v --timeout 240 --timeout-method thread -k "$TESTK" > $OUT/pytest.log 2>&1 || exit 1
fi
for cfg in ${CFGS:-default persistent}; do
  A=""; [ $cfg = persistent ] && A="--prune-threshold 0"
  timeout -k 10 400 python bench/bench_consolidate.py --steps 8 --warmup 2 $A > $OUT/${cfg}_plain.json 2> $OUT/${cfg}_plain.err || exit 1
  LZK_TRACE=1 timeout -k 10 400 python bench/bench_consolidate.py --steps 6 --warmup 2 $A > $OUT/$cfg.json 2> $OUT/$cfg.err || exit 1
  if [ -n "$KT" ]; then
    timeout -s KILL 400 rocprofv3 --kernel-trace --output-format csv -d /tmp/kt_$cfg -o run -- python3 bench/bench_consolidate.py --steps 4 --warmup 2 $A > $OUT/${cfg}_kt.json 2> $OUT/${cfg}_kt.err || exit 1
    MS=$(python3 -c "
import json
r=None
for l in open('$OUT/${cfg}_kt.json'):
    try: d=json.loads(l)
    except Exception: continue
    if 'ms_per_step' in d: r=d
print(r['ms_per_step']*4)")
    python3 tools/ktrace_window.py /tmp/kt_$cfg/run_kernel_trace.csv $MS 4 $OUT/${cfg}_window.json > /dev/null || exit 1
  fi
done
