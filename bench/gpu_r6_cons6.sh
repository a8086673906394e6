#!/bin/bash
# round 6: consolidation -- verify-kernel shortcuts + GIL-free planner: tests, plain runs, write-behind A/B
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
export PYTHONPATH=$PWD${PYTHONPATH:+:$PYTHONPATH}
OUT=${OUT:-gpurun_out/r6cons6}
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/kernels/test_eviction_pool_gpu.py tests/unit/test_consolidate_batch_exact.py -m gpu -x -v \
  --timeout 240 --timeout-method thread > $OUT/pytest.log 2>&1 || exit 1
for v in default async default2 async2 persistent; do
  A=""; case $v in async*) A="--persist-async";; persistent) A="--prune-threshold 0";; esac
  timeout -k 10 400 python bench/bench_consolidate.py --steps 10 --warmup 2 $A > $OUT/$v.json 2> $OUT/$v.err || exit 1
done
