#!/bin/bash
# consolidate_stream: GPU exactness tests + A/B against per-batch calls (round-5 working script)
export TMPDIR=/tmp
export PYTHONPATH=$PWD${PYTHONPATH:+:$PYTHONPATH}
OUT=${OUT:-gpurun_out/stream}
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/kernels/test_tenant_engine_gpu.py -x -v --timeout 300 --timeout-method thread -k "stream or at_scale or incremental" > $OUT/pytest.log 2>&1 || exit 1
LZK_TRACE=1 timeout -k 10 400 python bench/bench_consolidate.py --steps 5 --warmup 2 > $OUT/stream.json 2> $OUT/stream.err || exit 1
LZK_TRACE=1 timeout -k 10 400 python bench/bench_consolidate.py --steps 5 --warmup 2 --no-stream > $OUT/calls.json 2> $OUT/calls.err || exit 1
