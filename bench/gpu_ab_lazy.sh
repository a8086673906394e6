#!/bin/bash
# round-5 working script: headline under torchrun (lazy RCCL) vs one plain process, then a full default bench
export TMPDIR=/tmp
OUT=${OUT:-gpurun_out/ab_lazy}
mkdir -p $OUT
Q="--consolidate-steps 0 --sharded-steps 0 --routed-steps 0 --global-batch 0"
timeout -k 10 300 python bench.py $Q > $OUT/head_1.json 2> $OUT/head_1.err || exit 1
timeout -k 10 300 python bench.py $Q --no-launch > $OUT/nolaunch_1.json 2> $OUT/nolaunch_1.err || exit 1
timeout -k 10 300 python bench.py $Q > $OUT/head_2.json 2> $OUT/head_2.err || exit 1
timeout -k 10 900 python bench.py > $OUT/full.json 2> $OUT/full.err || exit 1
