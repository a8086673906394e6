#!/bin/bash
# round 6: incremental sharded digest -- GPU tests, then the row-sharded
# buffer (one rank) with prune_threshold 0 (incremental digest on / off) and 0.5
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
export PYTHONPATH=$PWD${PYTHONPATH:+:$PYTHONPATH}
OUT=${OUT:-gpurun_out/r6shpg}
mkdir -p $OUT
if [ -z "$NOTEST" ]; then
  timeout -k 10 600 python -u -m pytest tests/kernels/test_sharded_memory_gpu.py -m gpu -x -v --timeout 240 \
    --timeout-method thread -k "${TESTK:-incremental or one_rank}" > $OUT/pytest.log 2>&1 || exit 1
fi
B="python bench/bench_consolidate.py --sharded --clustered --no-stream --steps ${STEPS:-3} --warmup 1"
LZK_TRACE=1 timeout -k 10 400 $B --prune-threshold 0 > $OUT/pg_inc.json 2> $OUT/pg_inc.err || exit 1
LZK_TRACE=1 timeout -k 10 400 $B --prune-threshold 0 --no-incremental-digest > $OUT/pg_full.json 2> $OUT/pg_full.err || exit 1
LZK_TRACE=1 timeout -k 10 400 $B > $OUT/default.json 2> $OUT/default.err || exit 1
