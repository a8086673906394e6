# headline stability: repeated runs, side-stream priority, no overlap
set -o pipefail
export PYTHONPATH=$PWD
mkdir -p gpurun_out
H="--consolidate-steps 0 --sharded-steps 0 --no-persistent-graph --routed-steps 0 --global-batch 0 --recall-queries 256 --steps 30"
for v in a b; do timeout -k 10 300 python -u bench.py $H --json-out gpurun_out/hs_def_$v.json > gpurun_out/hs_def_$v.log 2>&1 || exit 1; done
for v in a b; do LZK_SIDE_PRIO=-1 timeout -k 10 300 python -u bench.py $H --json-out gpurun_out/hs_hi_$v.json > gpurun_out/hs_hi_$v.log 2>&1 || exit 2; done
LZK_SEARCH_OVERLAP=0 timeout -k 10 300 python -u bench.py $H --json-out gpurun_out/hs_noov.json > gpurun_out/hs_noov.log 2>&1 || exit 3
