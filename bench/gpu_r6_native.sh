#!/bin/bash
# round 6: native segment applier -- exactness tests first, then the bench with stages and a kernel trace
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
export PYTHONPATH=$PWD${PYTHONPATH:+:$PYTHONPATH}
OUT=${OUT:-gpurun_out/r6native}
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/unit/test_consolidate_batch_exact.py tests/kernels/test_tenant_engine_gpu.py \
  -m gpu -x -v --timeout 240 --timeout-method thread -k "${TESTK:-sequential_gpu or consolidat}" > $OUT/pytest.log 2>&1 || exit 1
OUT=$OUT KT=1 NOTEST=1 bash bench/gpu_r6_cons.sh || exit 1
