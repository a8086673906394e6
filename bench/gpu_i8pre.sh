#!/bin/bash
# int8 scan: integer-max column prefilter -- tests, scan probe, headline (round-5 working script)
export TMPDIR=/tmp
export PYTHONPATH=$PWD${PYTHONPATH:+:$PYTHONPATH}
OUT=${OUT:-gpurun_out/i8pre}
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread > $OUT/pytest.log 2>&1 || exit 1
timeout -k 10 300 python bench/probe_i8_scan.py > $OUT/probe.json 2> $OUT/probe.err || exit 1
Q="--consolidate-steps 0 --sharded-steps 0 --routed-steps 0 --global-batch 0"
for i in 1 2; do
  timeout -k 10 300 python bench.py $Q > $OUT/h$i.json 2> $OUT/h$i.err || exit 1
done
