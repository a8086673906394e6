set -o pipefail
export PYTHONPATH=$PWD
mkdir -p gpurun_out
H="--consolidate-steps 0 --sharded-steps 0 --no-persistent-graph --routed-steps 0 --global-batch 0 --recall-queries 256 --steps 30"
for v in a b; do timeout -k 10 300 python -u bench.py $H --json-out gpurun_out/hu_$v.json > gpurun_out/hu_$v.log 2>&1 || exit 1; done
timeout -k 10 900 python -u bench.py --json-out gpurun_out/bench_r4u.json > gpurun_out/bench_r4u.log 2>&1 || exit 2
