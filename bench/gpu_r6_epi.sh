#!/bin/bash
# int8 scan epilogue: integer-domain column prefilter -- GPU tests of the
# int8 / dual scans, then the interleaved A/B on the headline store search
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
export PYTHONPATH=$PWD${PYTHONPATH:+:$PYTHONPATH}
OUT=${OUT:-gpurun_out/r6epi}
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/kernels/test_tenant_engine_gpu.py tests/kernels/test_query_prep_gpu.py tests/kernels/test_segment_gpu.py -m gpu -x -v --timeout 200 --timeout-method thread > $OUT/pytest.log 2>&1 || exit 1
timeout -k 10 300 python -u bench/ab_i8_epilogue.py > $OUT/ab.json 2> $OUT/ab.err || exit 1
