#!/bin/bash
# round-5 working script: overflow-path probe, its tests, the row-sharded bench section
export TMPDIR=/tmp
export PYTHONPATH=$PWD${PYTHONPATH:+:$PYTHONPATH}
OUT=${OUT:-gpurun_out/r5k}
mkdir -p $OUT
timeout -k 10 180 python -u bench/probe_dual_ovf.py > $OUT/probe.log 2>&1 || exit 1
timeout -k 10 400 python -u -m pytest -x -v --timeout 240 --timeout-method thread tests/kernels/test_tenant_engine_gpu.py -m gpu -k "dual_i8 or int8_dual_decisions" > $OUT/pytest.log 2>&1 || exit 1
timeout -k 10 600 python bench.py --steps 5 --warmup 2 --consolidate-steps 0 --routed-steps 0 --global-batch 0 > $OUT/sharded.json 2> $OUT/sharded.err || exit 1
