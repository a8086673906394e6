#!/bin/bash
# incremental digest: the selected count and pairs read back in one wait --
# GPU tests of the native applier's incremental path, then the persistent bench
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
export PYTHONPATH=$PWD${PYTHONPATH:+:$PYTHONPATH}
OUT=${OUT:-gpurun_out/r6ccsync}
mkdir -p $OUT
timeout -k 10 700 python -u -m pytest tests/kernels/test_tenant_engine_gpu.py tests/kernels/test_sharded_memory_gpu.py tests/unit/test_consolidate_batch_exact.py -m gpu -x -v --timeout 240 --timeout-method thread > $OUT/pytest.log 2>&1 || exit 1
for v in p1 p2; do
  timeout -k 10 400 python bench/bench_consolidate.py --steps 20 --warmup 2 --prune-threshold 0 > $OUT/$v.json 2> $OUT/$v.err || exit 1
done
