#!/bin/bash
# round 6: i8 query kernel on wide batches (LZK_I8_QUERY_WIDE) -- test, then interleaved headline A/B
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
export PYTHONPATH=$PWD${PYTHONPATH:+:$PYTHONPATH}
OUT=${OUT:-gpurun_out/r6i8q}
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/kernels/test_query_prep_gpu.py -m gpu -x -v --timeout 240 --timeout-method thread > $OUT/pytest.log 2>&1 || exit 1
H="python bench.py --gpus 1 --steps 20 --warmup 5 --consolidate-steps 0 --sharded-steps 0 --sharded-persistent-steps 0 --no-persistent-graph --routed-steps 0 --global-batch 0"
for v in base wide base2 wide2; do
  W=0; case $v in wide*) W=1;; esac
  LZK_I8_QUERY_WIDE=$W timeout -k 10 400 $H > $OUT/$v.json 2> $OUT/$v.err || exit 1
done
