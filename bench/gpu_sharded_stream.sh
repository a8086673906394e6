#!/bin/bash
# row-sharded consolidate_stream: GPU tests + A/B inside bench.py (round-5 working script)
export TMPDIR=/tmp
export PYTHONPATH=$PWD${PYTHONPATH:+:$PYTHONPATH}
OUT=${OUT:-gpurun_out/sharded_stream}
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/kernels/test_sharded_memory_gpu.py -x -v --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1 || exit 1
A="--steps 2 --warmup 1 --consolidate-steps 0 --routed-steps 0 --global-batch 0 --sharded-steps 5"
LZK_TRACE=1 timeout -k 10 500 python bench.py $A > $OUT/stream.json 2> $OUT/stream.err || exit 1
LZK_TRACE=1 timeout -k 10 500 python bench.py $A --consolidate-calls > $OUT/calls.json 2> $OUT/calls.err || exit 1
