#!/bin/bash
# round 6: host profile (cProfile) of the default consolidation's timed steps
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
export PYTHONPATH=$PWD${PYTHONPATH:+:$PYTHONPATH}
OUT=${OUT:-gpurun_out/r6hprof}
mkdir -p $OUT
LZK_PROF_HOST=1 timeout -k 10 400 python bench/bench_consolidate.py --steps 8 --warmup 2 $EXTRA > $OUT/default.json 2> $OUT/default_prof.txt || exit 1
