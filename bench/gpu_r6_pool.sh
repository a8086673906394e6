#!/bin/bash
# round 6: tie-aware sampled eviction pool -- tests, then the default consolidation bench (plain + stages)
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
export PYTHONPATH=$PWD${PYTHONPATH:+:$PYTHONPATH}
OUT=${OUT:-gpurun_out/r6pool}
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/kernels/test_eviction_pool_gpu.py tests/unit/test_consolidate_batch_exact.py -m gpu -x -v \
  --timeout 240 --timeout-method thread > $OUT/pytest.log 2>&1 || exit 1
timeout -k 10 400 python bench/bench_consolidate.py --steps 10 --warmup 2 > $OUT/plain.json 2> $OUT/plain.err || exit 1
timeout -k 10 400 python bench/bench_consolidate.py --steps 10 --warmup 2 --prune-threshold 0 > $OUT/persistent.json 2> $OUT/persistent.err || exit 1
LZK_PROF_HOST=1 timeout -k 10 400 python bench/bench_consolidate.py --steps 8 --warmup 2 > $OUT/prof.json 2> $OUT/prof.txt || exit 1
