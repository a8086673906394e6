#!/bin/bash
# round 6: one-rank sharded buffer on a persistent graph through the native applier + incremental components
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
export PYTHONPATH=$PWD${PYTHONPATH:+:$PYTHONPATH}
OUT=${OUT:-gpurun_out/r6sharded}
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/kernels/test_sharded_memory_gpu.py -m gpu -x -v --timeout 240 \
  --timeout-method thread -k "one_rank or incremental" > $OUT/pytest.log 2>&1 || exit 1
B="python bench/bench_consolidate.py --sharded --clustered --no-stream --steps 5 --warmup 1"
timeout -k 10 400 $B --prune-threshold 0 > $OUT/pg.json 2> $OUT/pg.err || exit 1
timeout -k 10 400 $B > $OUT/default.json 2> $OUT/default.err || exit 1
