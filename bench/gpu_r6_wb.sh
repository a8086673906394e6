#!/bin/bash
# write-behind persistence A/B on the current tree (interleaved x3)
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
export PYTHONPATH=$PWD${PYTHONPATH:+:$PYTHONPATH}
OUT=${OUT:-gpurun_out/r6wb}
mkdir -p $OUT
for v in sync1 async1 sync2 async2 sync3 async3; do
  A=""; case $v in async*) A="--persist-async";; esac
  timeout -k 10 400 python bench/bench_consolidate.py --steps 20 --warmup 2 $A > $OUT/$v.json 2> $OUT/$v.err || exit 1
done
