#!/bin/bash
# round 6: ATen ops per Python call site in the default consolidation's timed steps
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
export PYTHONPATH=$PWD${PYTHONPATH:+:$PYTHONPATH}
OUT=${OUT:-gpurun_out/r6ops}
mkdir -p $OUT
LZK_PROF_OPS=1 timeout -k 10 500 python bench/bench_consolidate.py --steps 5 --warmup 2 $EXTRA > $OUT/ops.json 2> $OUT/ops.txt || exit 1
