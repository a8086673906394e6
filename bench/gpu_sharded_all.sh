#!/bin/bash
# row-sharded consolidation: GPU tests, plain traced run, the 1-rank torchrun bench (round-5 working script)
export TMPDIR=/tmp
export PYTHONPATH=$PWD${PYTHONPATH:+:$PYTHONPATH}
OUT=${OUT:-gpurun_out/sharded_all}
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/kernels/test_sharded_memory_gpu.py -x -v --timeout 240 --timeout-method thread > $OUT/pytest.log 2>&1 || exit 1
LZK_TRACE=1 timeout -k 10 400 python bench/bench_consolidate.py --steps 5 --warmup 1 --sharded --clustered > $OUT/sharded.json 2> $OUT/sharded.err || exit 1
LZK_TRACE=1 timeout -k 10 600 python bench.py --steps 2 --warmup 1 --consolidate-steps 0 --routed-steps 0 --global-batch 0 --sharded-steps 5 > $OUT/bench.json 2> $OUT/bench.err || exit 1
