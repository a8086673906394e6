#!/bin/bash
# round 6: one steady-state batch's planner inputs (LZK_DUMP_PLAN) for CPU-side planner profiling
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
export PYTHONPATH=$PWD${PYTHONPATH:+:$PYTHONPATH}
OUT=${OUT:-gpurun_out/r6dump}
mkdir -p $OUT
rm -f $OUT/plan_inputs.npz
# the dump is written by the first planner call after warmup starts: run 3 batches, keep the file of batch 3
LZK_DUMP_PLAN=/tmp/p1.npz:3 timeout -k 10 400 python bench/bench_consolidate.py --steps 1 --warmup 2 > $OUT/b.json 2> $OUT/b.err || exit 1
cp /tmp/p1.npz $OUT/plan_inputs.npz
