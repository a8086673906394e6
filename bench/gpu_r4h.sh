# round-4 pass 7: consolidation (tests, bench, host/op profiles) + interactive latency
set -o pipefail
export PYTHONPATH=$PWD
mkdir -p gpurun_out
bash bench/gpu_r4f.sh || exit $?
bash bench/gpu_r4g.sh || exit 21
timeout -k 10 400 python -u bench/bench_latency.py --iters 100 > gpurun_out/latency_r4.json 2> gpurun_out/latency_r4.err || exit 22
