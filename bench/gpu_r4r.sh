set -o pipefail
export PYTHONPATH=$PWD
mkdir -p gpurun_out
H="--consolidate-steps 0 --sharded-steps 0 --no-persistent-graph --routed-steps 0 --global-batch 0 --recall-queries 256 --steps 30"
for v in a b; do timeout -k 10 300 python -u bench.py $H --json-out gpurun_out/hr_$v.json > gpurun_out/hr_$v.log 2>&1 || exit 1; done
LZK_PROF_HEADLINE=1 timeout -k 10 300 python -u bench.py $H --json-out gpurun_out/hr_p.json > gpurun_out/hr_p.log 2> gpurun_out/hr_p.err || exit 2
