#!/bin/bash
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
export PYTHONPATH=$PWD${PYTHONPATH:+:$PYTHONPATH}
OUT=${OUT:-gpurun_out/r6probe}
mkdir -p $OUT
timeout -k 10 400 python tools/narrow_margins.py > $OUT/margins.json 2> $OUT/margins.err || exit 1
