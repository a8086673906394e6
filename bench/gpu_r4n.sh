# headline bisect: pipelined search_memories_stream QPS under toggles
set -o pipefail
export PYTHONPATH=$PWD
mkdir -p gpurun_out
H="--consolidate-steps 0 --sharded-steps 0 --no-persistent-graph --routed-steps 0 --global-batch 0 --recall-queries 256"
timeout -k 10 300 python -u bench.py $H --json-out gpurun_out/hb_default.json > gpurun_out/hb_default.log 2>&1 || exit 1
LZK_I8_QUERY=0 timeout -k 10 300 python -u bench.py $H --json-out gpurun_out/hb_noq.json > gpurun_out/hb_noq.log 2>&1 || exit 2
LZK_SPEC_CHECK_KERNEL=0 timeout -k 10 300 python -u bench.py $H --json-out gpurun_out/hb_nochk.json > gpurun_out/hb_nochk.log 2>&1 || exit 3
