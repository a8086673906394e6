#!/bin/bash
# headline-only bench runs + one full default bench (round-5 working script)
export TMPDIR=/tmp
export PYTHONPATH=$PWD${PYTHONPATH:+:$PYTHONPATH}
OUT=${OUT:-gpurun_out/head}
mkdir -p $OUT
Q="--consolidate-steps 0 --sharded-steps 0 --routed-steps 0 --global-batch 0"
for i in 1 2; do
  timeout -k 10 300 python bench.py $Q > $OUT/h$i.json 2> $OUT/h$i.err || exit 1
done
if [ -n "$FULL" ]; then
  timeout -k 10 600 python bench.py > $OUT/full.json 2> $OUT/full.err || exit 1
fi
