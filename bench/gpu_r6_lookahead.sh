#!/bin/bash
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
export PYTHONPATH=$PWD${PYTHONPATH:+:$PYTHONPATH}
OUT=gpurun_out/r6la
mkdir -p $OUT
timeout -k 10 500 python -u -m pytest tests/kernels/test_tenant_engine_gpu.py -m gpu -x -v --timeout 240 --timeout-method thread -k "consolidate" > $OUT/pytest.log 2>&1 || exit 1
for v in la1 la2 la1b la2b la1c la2c; do
  L=2; case $v in la1*) L=1;; esac
  timeout -k 10 400 python bench/bench_consolidate.py --steps 20 --warmup 2 --lookahead $L > $OUT/$v.json 2> $OUT/$v.err || exit 1
done
