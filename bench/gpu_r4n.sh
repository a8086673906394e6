# headline: default (narrow-only query kernel) and the wide kernel with fallback stats
set -o pipefail
export PYTHONPATH=$PWD
mkdir -p gpurun_out
H="--consolidate-steps 0 --sharded-steps 0 --no-persistent-graph --routed-steps 0 --global-batch 0 --recall-queries 256"
timeout -k 10 300 python -u bench.py $H --json-out gpurun_out/hb_default.json > gpurun_out/hb_default.log 2>&1 || exit 1
LZK_I8_QUERY_WIDE=1 LZK_SPEC_STATS=1 timeout -k 10 300 python -u bench.py $H --json-out gpurun_out/hb_wide.json > gpurun_out/hb_wide.log 2>&1 || exit 2
LZK_SPEC_STATS=1 timeout -k 10 300 python -u bench.py $H --json-out gpurun_out/hb_stats.json > gpurun_out/hb_stats.log 2>&1 || exit 3
