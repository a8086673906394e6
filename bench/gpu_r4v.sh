set -o pipefail
export PYTHONPATH=$PWD
mkdir -p gpurun_out
H="--consolidate-steps 0 --sharded-steps 0 --no-persistent-graph --routed-steps 0 --global-batch 0 --recall-queries 256 --steps 30"
for v in a b c; do LZK_STREAM_DEPTH=1 timeout -k 10 300 python -u bench.py $H --json-out gpurun_out/hv_d1_$v.json > gpurun_out/hv_d1_$v.log 2>&1 || exit 1; done
for v in a b; do LZK_STREAM_DEPTH=2 timeout -k 10 300 python -u bench.py $H --json-out gpurun_out/hv_d2_$v.json > gpurun_out/hv_d2_$v.log 2>&1 || exit 2; done
LZK_STREAM_DEPTH=1 LZK_GC_FREEZE=0 timeout -k 10 300 python -u bench.py $H --json-out gpurun_out/hv_d1_nf.json > gpurun_out/hv_d1_nf.log 2>&1 || exit 3
