# host-side profile of the consolidation step: aten ops per call site, cProfile
set -o pipefail
export PYTHONPATH=$PWD
mkdir -p gpurun_out
LZK_PROF_OPS=1 timeout -k 10 400 python -u bench/bench_consolidate.py --steps 2 --warmup 2 > gpurun_out/cons_ops.json 2> gpurun_out/cons_ops.err || exit 1
LZK_PROF_HOST=1 timeout -k 10 400 python -u bench/bench_consolidate.py --steps 3 --warmup 2 > gpurun_out/cons_host.json 2> gpurun_out/cons_host.err || exit 2
