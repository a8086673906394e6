#!/bin/bash
# GPU test tier (+ FULL=1: headline-only bench runs) -- round-5 working script
export TMPDIR=/tmp
export PYTHONPATH=$PWD${PYTHONPATH:+:$PYTHONPATH}
OUT=${OUT:-gpurun_out/tier}
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || exit 1
if [ -n "$FULL" ]; then
  Q="--consolidate-steps 0 --sharded-steps 0 --routed-steps 0 --global-batch 0"
  for i in 1 2; do
    timeout -k 10 300 python bench.py $Q > $OUT/h$i.json 2> $OUT/h$i.err || exit 1
  done
fi
