set -o pipefail
export PYTHONPATH=$PWD
mkdir -p gpurun_out
timeout -k 10 400 python -u bench/bench_consolidate.py --steps 5 --warmup 2 > gpurun_out/cy_sync.json 2> gpurun_out/cy_sync.err || exit 1
timeout -k 10 400 python -u bench/bench_consolidate.py --steps 5 --warmup 2 --persist-async > gpurun_out/cy_async.json 2> gpurun_out/cy_async.err || exit 2
LZK_PROF_HOST=1 timeout -k 10 400 python -u bench/bench_consolidate.py --steps 3 --warmup 2 > gpurun_out/cy_host.json 2> gpurun_out/cy_host.err || exit 3
