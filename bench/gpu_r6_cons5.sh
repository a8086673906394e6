#!/bin/bash
# round 6: consolidation after the planner work -- exactness tests, plain runs (default, persistent), stage run
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
export PYTHONPATH=$PWD${PYTHONPATH:+:$PYTHONPATH}
OUT=${OUT:-gpurun_out/r6cons5}
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/unit/test_consolidate_batch_exact.py tests/kernels/test_eviction_pool_gpu.py -m gpu -x -v \
  --timeout 240 --timeout-method thread > $OUT/pytest.log 2>&1 || exit 1
for v in default persistent default2; do
  A=""; [ $v = persistent ] && A="--prune-threshold 0"
  timeout -k 10 400 python bench/bench_consolidate.py --steps 10 --warmup 2 $A > $OUT/$v.json 2> $OUT/$v.err || exit 1
done
LZK_TRACE=1 timeout -k 10 400 python bench/bench_consolidate.py --steps 8 --warmup 2 > $OUT/stages.json 2> $OUT/stages.err || exit 1
