#!/bin/bash
# persistent graph: edge partition A/B on one box (round-5 working script)
export TMPDIR=/tmp
export PYTHONPATH=$PWD${PYTHONPATH:+:$PYTHONPATH}
OUT=${OUT:-gpurun_out/ab_part}
mkdir -p $OUT
for v in 1 0; do
  timeout -k 10 300 python bench/ab_partition.py $v >> $OUT/ab.jsonl 2>> $OUT/ab.err || exit 1
done
