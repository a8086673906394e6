#!/bin/bash
# round-5 working script: traced stage breakdowns of the consolidation benches
export TMPDIR=/tmp
export PYTHONPATH=$PWD${PYTHONPATH:+:$PYTHONPATH}
OUT=${OUT:-gpurun_out/cons_stages}
mkdir -p $OUT
LZK_TRACE=1 timeout -k 10 400 python bench/bench_consolidate.py --steps 5 --warmup 2 > $OUT/default.json 2> $OUT/default.err || exit 1
LZK_TRACE=1 timeout -k 10 400 python bench/bench_consolidate.py --steps 5 --warmup 2 --prune-threshold 0 > $OUT/persistent.json 2> $OUT/persistent.err || exit 1
LZK_TRACE=1 timeout -k 10 400 python bench/bench_consolidate.py --steps 3 --warmup 1 --sharded --clustered > $OUT/sharded.json 2> $OUT/sharded.err || exit 1
