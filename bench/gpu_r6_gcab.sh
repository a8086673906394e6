#!/bin/bash
# headline only: default (no gc.freeze) vs --gc-freeze, interleaved x2, then
# the exact int8 mode (LZK_LOWP_EXACT=1: worst-case margin on wide batches too)
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
export PYTHONPATH=$PWD${PYTHONPATH:+:$PYTHONPATH}
OUT=${OUT:-gpurun_out/r6gcab}
mkdir -p $OUT
H="python bench.py --gpus 1 --steps 20 --warmup 5 --consolidate-steps 0 --sharded-steps 0 --sharded-persistent-steps 0 --no-persistent-graph"
for v in nofreeze freeze nofreeze2 freeze2; do
  A=""; case $v in freeze*) A="--gc-freeze";; esac
  timeout -k 10 400 $H $A > $OUT/$v.json 2> $OUT/$v.err || exit 1
done
LZK_LOWP_EXACT=1 timeout -k 10 400 $H > $OUT/exact.json 2> $OUT/exact.err || exit 1
