#!/bin/bash
# first-rows kernel with four barriers per chunk: GPU tests, then its time in a
# kernel trace of the consolidation bench, then the plain bench
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
export PYTHONPATH=$PWD${PYTHONPATH:+:$PYTHONPATH}
OUT=${OUT:-gpurun_out/r6fr}
mkdir -p $OUT
timeout -k 10 700 python -u -m pytest tests/kernels/test_digest_gpu.py tests/kernels/test_tenant_engine_gpu.py tests/unit/test_consolidate_batch_exact.py tests/kernels/test_sharded_memory_gpu.py -m gpu -x -v --timeout 240 --timeout-method thread > $OUT/pytest.log 2>&1 || exit 1
timeout -s KILL 400 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/kt_fr -o run -- python3 bench/bench_consolidate.py --steps 5 --warmup 2 > $OUT/kt.json 2> $OUT/kt.err || exit 1
cp /tmp/kt_fr/run_kernel_stats.csv $OUT/kernel_stats.csv || exit 1
for v in a b; do
  timeout -k 10 400 python bench/bench_consolidate.py --steps 20 --warmup 2 > $OUT/$v.json 2> $OUT/$v.err || exit 1
done
