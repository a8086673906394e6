#!/bin/bash
# eviction verification shortcut for rows under the salience floor: GPU tests,
# then the verify kernel's time in a kernel trace of the consolidation bench
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
export PYTHONPATH=$PWD${PYTHONPATH:+:$PYTHONPATH}
OUT=${OUT:-gpurun_out/r6verify}
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/kernels/test_eviction_pool_gpu.py tests/unit/test_consolidate_batch_exact.py tests/kernels/test_tenant_engine_gpu.py -m gpu -x -v --timeout 240 --timeout-method thread -k "evict or verify or pool or consolidate" > $OUT/pytest.log 2>&1 || exit 1
timeout -s KILL 400 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/kt_v -o run -- python3 bench/bench_consolidate.py --steps 5 --warmup 2 > $OUT/kt.json 2> $OUT/kt.err || exit 1
cp /tmp/kt_v/run_kernel_stats.csv $OUT/kernel_stats.csv || exit 1
timeout -k 10 400 python bench/bench_consolidate.py --steps 20 --warmup 2 > $OUT/plain.json 2> $OUT/plain.err || exit 1
