#!/bin/bash
# row-sharded consolidation: GPU tests + traced stages (round-5 working script)
export TMPDIR=/tmp
export PYTHONPATH=$PWD${PYTHONPATH:+:$PYTHONPATH}
OUT=${OUT:-gpurun_out/sharded}
mkdir -p $OUT
[ -n "$NOTEST" ] || timeout -k 10 300 python -u -m pytest tests/kernels/test_sharded_memory_gpu.py -x -v --timeout 240 --timeout-method thread > $OUT/pytest.log 2>&1 || exit 1
LZK_TRACE=1 timeout -k 10 400 python bench/bench_consolidate.py --steps 3 --warmup 1 --sharded --clustered > $OUT/sharded.json 2> $OUT/sharded.err || exit 1
LZK_PROF_HOST=1 timeout -k 10 400 python bench/bench_consolidate.py --steps 2 --warmup 1 --sharded --clustered > $OUT/sharded_prof.json 2> $OUT/sharded_prof.err || exit 1
