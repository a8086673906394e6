#!/bin/bash
# round-5 working script: encoder A/B (hidden-width projections in the library GEMM)
export TMPDIR=/tmp
OUT=${OUT:-gpurun_out/ab_enc}
mkdir -p $OUT
Q="--consolidate-steps 0 --sharded-steps 0 --routed-steps 0 --global-batch 0 --no-launch"
for i in 1 2; do
  LZK_ENC_LIB_GEMM=0 timeout -k 10 300 python bench.py $Q > $OUT/own_$i.json 2> $OUT/own_$i.err || exit 1
  LZK_ENC_LIB_GEMM=1 timeout -k 10 300 python bench.py $Q > $OUT/lib_$i.json 2> $OUT/lib_$i.err || exit 1
done
