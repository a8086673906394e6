# host profile of the headline loop
set -o pipefail
export PYTHONPATH=$PWD
mkdir -p gpurun_out
H="--consolidate-steps 0 --sharded-steps 0 --no-persistent-graph --routed-steps 0 --global-batch 0 --recall-queries 256 --steps 30"
LZK_PROF_HEADLINE=1 timeout -k 10 300 python -u bench.py $H --json-out gpurun_out/hp.json > gpurun_out/hp.log 2> gpurun_out/hp.err || exit 1
