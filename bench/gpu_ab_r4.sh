#!/bin/bash
# round-5 working script: headline A/B of the round-4 tree against HEAD on one box
export TMPDIR=/tmp
OUT=${OUT:-gpurun_out/ab_r4}
mkdir -p $OUT
Q="--consolidate-steps 0 --sharded-steps 0 --routed-steps 0 --global-batch 0"
ROOT=$PWD
for i in 1 2; do
  (cd r4tree && timeout -k 10 300 python bench.py $Q > $ROOT/$OUT/r4_$i.json 2> $ROOT/$OUT/r4_$i.err) || exit 1
  timeout -k 10 300 python bench.py $Q > $OUT/head_$i.json 2> $OUT/head_$i.err || exit 1
done
timeout -k 10 300 python bench.py $Q --no-launch > $OUT/head_nolaunch.json 2> $OUT/head_nolaunch.err || exit 1
PYTHONPATH=$ROOT timeout -k 10 200 python bench/probe_gemm_lib.py > $OUT/gemm_lib.json 2> $OUT/gemm_lib.err || exit 1
