#!/bin/bash
# GPU test tier + headline-only bench runs (round-5 working script)
export TMPDIR=/tmp
OUT=${OUT:-gpurun_out/tier}
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || exit 1
Q="--consolidate-steps 0 --sharded-steps 0 --routed-steps 0 --global-batch 0"
for i in 1 2; do
  timeout -k 10 300 python bench.py $Q > $OUT/h$i.json 2> $OUT/h$i.err || exit 1
done
