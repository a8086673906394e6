#!/bin/bash
# round 6: headline + serving sections only (consolidation sections skipped)
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
export PYTHONPATH=$PWD${PYTHONPATH:+:$PYTHONPATH}
OUT=${OUT:-gpurun_out/r6head}
mkdir -p $OUT
for r in ${RUNS:-1}; do
  timeout -k 10 500 python bench.py --gpus 1 --steps 20 --warmup 5 --consolidate-steps 0 --sharded-steps 0 \
    --sharded-persistent-steps 0 --no-persistent-graph $BENCH_ARGS > $OUT/head_$r.json 2> $OUT/head_$r.err || exit 1
done
