# the full 1-GPU bench after the round-4 consolidation / narrow-search work
set -o pipefail
export PYTHONPATH=$PWD
mkdir -p gpurun_out
timeout -k 10 1000 python -u bench.py --json-out gpurun_out/bench_r4m.json > gpurun_out/bench_r4m.log 2>&1 || exit 1
