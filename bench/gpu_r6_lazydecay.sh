#!/bin/bash
# lazy node decay in the native applier: bit-exactness GPU tests (batched vs
# sequential, stream vs calls, one-rank sharded), then an interleaved A/B
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
export PYTHONPATH=$PWD${PYTHONPATH:+:$PYTHONPATH}
OUT=${OUT:-gpurun_out/r6lazy}
mkdir -p $OUT
timeout -k 10 800 python -u -m pytest tests/unit/test_consolidate_batch_exact.py tests/kernels/test_tenant_engine_gpu.py tests/kernels/test_sharded_memory_gpu.py tests/kernels/test_eviction_pool_gpu.py tests/kernels/test_digest_gpu.py -m gpu -x -v --timeout 240 --timeout-method thread > $OUT/pytest.log 2>&1 || exit 1
for v in eager lazy eager2 lazy2; do
  A=""; case $v in eager*) A="--eager-node-decay";; esac
  timeout -k 10 400 python bench/bench_consolidate.py --steps 20 --warmup 2 $A > $OUT/$v.json 2> $OUT/$v.err || exit 1
done
timeout -k 10 400 python bench/bench_consolidate.py --steps 20 --warmup 2 --prune-threshold 0 > $OUT/persistent.json 2> $OUT/persistent.err || exit 1
