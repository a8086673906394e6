#!/bin/bash
# single-tenant consolidation: host profile (round-5 working script)
export TMPDIR=/tmp
export PYTHONPATH=$PWD${PYTHONPATH:+:$PYTHONPATH}
OUT=${OUT:-gpurun_out/cons_prof}
mkdir -p $OUT
LZK_PROF_HOST=1 timeout -k 10 400 python bench/bench_consolidate.py --steps 4 --warmup 2 > $OUT/default_prof.json 2> $OUT/default_prof.err || exit 1
