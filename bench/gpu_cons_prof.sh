#!/bin/bash
# single-tenant consolidation: traced stages + host profile (round-5 working script)
export TMPDIR=/tmp
export PYTHONPATH=$PWD${PYTHONPATH:+:$PYTHONPATH}
OUT=${OUT:-gpurun_out/cons_prof}
mkdir -p $OUT
LZK_TRACE=1 timeout -k 10 400 python bench/bench_consolidate.py --steps 5 --warmup 2 > $OUT/default.json 2> $OUT/default.err || exit 1
LZK_PROF_HOST=1 timeout -k 10 400 python bench/bench_consolidate.py --steps 3 --warmup 2 > $OUT/default_prof.json 2> $OUT/default_prof.err || exit 1
