#!/bin/bash
# round 6: consolidation A/B, interleaved x3: synchronous commit vs write-behind (persist_async)
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
export PYTHONPATH=$PWD${PYTHONPATH:+:$PYTHONPATH}
OUT=${OUT:-gpurun_out/r6pa3}
mkdir -p $OUT
for v in warm sync1 async1 sync2 async2 sync3 async3; do
  A=""; case $v in async*) A="--persist-async";; esac
  S=10; [ $v = warm ] && S=3
  timeout -k 10 400 python bench/bench_consolidate.py --steps $S --warmup 2 $A > $OUT/$v.json 2> $OUT/$v.err || exit 1
done
