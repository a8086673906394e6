# speculative threshold depth A/B on the headline
set -o pipefail
export PYTHONPATH=$PWD
mkdir -p gpurun_out
H="--consolidate-steps 0 --sharded-steps 0 --no-persistent-graph --routed-steps 0 --global-batch 0 --recall-queries 1024 --steps 30"
for j in 5 3 4; do LZK_SPEC_J=$j LZK_SPEC_STATS=1 timeout -k 10 300 python -u bench.py $H --json-out gpurun_out/hj_$j.json > gpurun_out/hj_$j.log 2>&1 || exit 1; done
