#!/bin/bash
# consolidate_stream vs per-batch calls inside bench.py, same box (round-5 working script)
export TMPDIR=/tmp
export PYTHONPATH=$PWD${PYTHONPATH:+:$PYTHONPATH}
OUT=${OUT:-gpurun_out/cons_ab}
mkdir -p $OUT
A="--steps 2 --warmup 1 --routed-steps 0 --global-batch 0 --sharded-steps 0"
LZK_TRACE=1 timeout -k 10 500 python bench.py $A > $OUT/stream.json 2> $OUT/stream.err || exit 1
LZK_TRACE=1 timeout -k 10 500 python bench.py $A --consolidate-calls > $OUT/calls.json 2> $OUT/calls.err || exit 1
