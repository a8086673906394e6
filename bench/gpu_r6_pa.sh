#!/bin/bash
# round 6: consolidation A/B -- synchronous commit vs write-behind (persist_async), plain runs
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
export PYTHONPATH=$PWD${PYTHONPATH:+:$PYTHONPATH}
OUT=${OUT:-gpurun_out/r6pa}
mkdir -p $OUT
for v in sync async sync2 async2; do
  A=""; case $v in async*) A="--persist-async";; esac
  timeout -k 10 400 python bench/bench_consolidate.py --steps 10 --warmup 2 $A > $OUT/$v.json 2> $OUT/$v.err || exit 1
done
