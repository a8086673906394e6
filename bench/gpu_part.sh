#!/bin/bash
# stable/volatile edge partition within a batch: GPU tests + consolidation sections of bench.py (round-5 working script)
export TMPDIR=/tmp
export PYTHONPATH=$PWD${PYTHONPATH:+:$PYTHONPATH}
OUT=${OUT:-gpurun_out/part}
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/kernels/test_tenant_engine_gpu.py tests/kernels/test_graph_kernels_gpu.py tests/unit/test_consolidate_batch_exact.py -x -v --timeout 300 --timeout-method thread -m gpu > $OUT/pytest.log 2>&1 || exit 1
A="--steps 2 --warmup 1 --routed-steps 0 --global-batch 0 --sharded-steps 0"
LZK_TRACE=1 timeout -k 10 500 python bench.py $A > $OUT/bench.json 2> $OUT/bench.err || exit 1
