set -o pipefail
export PYTHONPATH=$PWD
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -v -m gpu --timeout 240 --timeout-method thread tests/kernels/test_sharded_memory_gpu.py tests/kernels/test_rccl_world1_gpu.py tests/unit/test_consolidate_batch_exact.py > gpurun_out/t_aa.log 2>&1
rc=$?
echo "pytest rc=$rc" >> gpurun_out/t_aa.log
if [ $rc -ne 0 ]; then exit 11; fi
timeout -k 10 400 python -u bench/bench_consolidate.py --sharded --clustered --nodes 10000000 --convs 128 --steps 3 --warmup 1 > gpurun_out/sh_aa.json 2> gpurun_out/sh_aa.err || exit 1
