#!/bin/bash
# the driver's default bench run (round-5 working script)
export TMPDIR=/tmp
export PYTHONPATH=$PWD${PYTHONPATH:+:$PYTHONPATH}
OUT=${OUT:-gpurun_out/full}
mkdir -p $OUT
timeout -k 10 1000 python bench.py > $OUT/full.json 2> $OUT/full.err || exit 1
