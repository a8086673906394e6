#!/bin/bash
# consolidation: batch i+1's scan prefetched under a batch that runs a k-means
# pass -- stream-vs-calls GPU tests, then an interleaved A/B of the bench
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
export PYTHONPATH=$PWD${PYTHONPATH:+:$PYTHONPATH}
OUT=${OUT:-gpurun_out/r6pfc}
mkdir -p $OUT
timeout -k 10 500 python -u -m pytest tests/kernels/test_tenant_engine_gpu.py -m gpu -x -v --timeout 240 --timeout-method thread > $OUT/pytest.log 2>&1 || exit 1
for v in off on off2 on2; do
  A=""; case $v in off*) A="--no-prefetch-under-cluster";; esac
  timeout -k 10 400 python bench/bench_consolidate.py --steps 20 --warmup 2 $A > $OUT/$v.json 2> $OUT/$v.err || exit 1
done
timeout -k 10 400 python bench/bench_consolidate.py --steps 20 --warmup 2 --prune-threshold 0 > $OUT/persistent.json 2> $OUT/persistent.err || exit 1
