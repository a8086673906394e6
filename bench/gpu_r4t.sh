set -o pipefail
export PYTHONPATH=$PWD
mkdir -p gpurun_out
H="--consolidate-steps 0 --sharded-steps 0 --no-persistent-graph --routed-steps 0 --global-batch 0 --recall-queries 256 --steps 30"
for v in a b c; do timeout -k 10 300 python -u bench.py $H --json-out gpurun_out/ht_$v.json > gpurun_out/ht_$v.log 2>&1 || exit 1; done
LZK_GC_FREEZE=0 timeout -k 10 300 python -u bench.py $H --json-out gpurun_out/ht_nofreeze.json > gpurun_out/ht_nofreeze.log 2>&1 || exit 2
