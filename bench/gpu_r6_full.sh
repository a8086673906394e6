#!/bin/bash
# round 6: the GPU test tier, smoke(), then the full default bench (the driver's command)
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
export PYTHONPATH=$PWD${PYTHONPATH:+:$PYTHONPATH}
OUT=${OUT:-gpurun_out/r6full}
mkdir -p $OUT
if [ -z "$NOTEST" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || exit 1
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || exit 1
fi
if [ -z "$NOBENCH" ]; then
  timeout -k 10 700 python bench.py --gpus 1 --steps 20 --warmup 5 ${BENCH_ARGS} > $OUT/bench.json 2> $OUT/bench.err || exit 1
fi
