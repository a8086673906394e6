#!/bin/bash
# consolidation: k-means passes in the background -- GPU tests (stream vs
# calls vs in-line passes), then an interleaved A/B of the bench
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
export PYTHONPATH=$PWD${PYTHONPATH:+:$PYTHONPATH}
OUT=${OUT:-gpurun_out/r6clbg}
mkdir -p $OUT
timeout -k 10 500 python -u -m pytest tests/kernels/test_tenant_engine_gpu.py -m gpu -x -v --timeout 240 --timeout-method thread -k "consolidate or cluster or hier" > $OUT/pytest.log 2>&1 || exit 1
for v in inline bg inline2 bg2 inline3 bg3; do
  A=""; case $v in inline*) A="--cluster-inline";; esac
  timeout -k 10 400 python bench/bench_consolidate.py --steps 20 --warmup 2 $A > $OUT/$v.json 2> $OUT/$v.err || exit 1
done
timeout -k 10 400 python bench/bench_consolidate.py --steps 20 --warmup 2 --prune-threshold 0 > $OUT/persistent.json 2> $OUT/persistent.err || exit 1
