# headline with blocking result events (x2) vs spinning (x1), host profile on one
set -o pipefail
export PYTHONPATH=$PWD
mkdir -p gpurun_out
H="--consolidate-steps 0 --sharded-steps 0 --no-persistent-graph --routed-steps 0 --global-batch 0 --recall-queries 256 --steps 30"
for v in a b; do timeout -k 10 300 python -u bench.py $H --json-out gpurun_out/hq_blk_$v.json > gpurun_out/hq_blk_$v.log 2>&1 || exit 1; done
LZK_PROF_HEADLINE=1 timeout -k 10 300 python -u bench.py $H --json-out gpurun_out/hq_blk_p.json > gpurun_out/hq_blk_p.log 2> gpurun_out/hq_blk_p.err || exit 2
LZK_BLOCKING_EVENTS=0 timeout -k 10 300 python -u bench.py $H --json-out gpurun_out/hq_spin.json > gpurun_out/hq_spin.log 2>&1 || exit 3
