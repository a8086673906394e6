# round-4 validation pass: the whole GPU test tier, scan A/Bs, RCCL world-1
# test, multi-tenant global pass + bench
set -o pipefail
export PYTHONPATH=$PWD
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -v -m gpu --timeout 300 --timeout-method thread tests > gpurun_out/t_gpu.log 2>&1
rc=$?
echo "pytest rc=$rc" >> gpurun_out/t_gpu.log
# 0 = passed, 1 = some tests failed: keep going; anything else (abort,
# segfault, time limit) ends the call here
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit 10; fi
LZK_SCAN8=1 timeout -k 10 400 python -u -m pytest -v --timeout 240 --timeout-method thread tests/kernels/test_tenant_engine_gpu.py -k "scan8 or i8 or lowp or zero_row or rigorous or lean" > gpurun_out/t_scan8.log 2>&1
rc=$?
echo "pytest rc=$rc" >> gpurun_out/t_scan8.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit 11; fi
timeout -k 10 400 python -u bench/ab_scan8.py > gpurun_out/ab_scan8.json 2> gpurun_out/ab_scan8.err || exit 2
timeout -k 10 300 python -u bench/ab_scan8_narrow.py > gpurun_out/ab_narrow.json 2> gpurun_out/ab_narrow.err || exit 3
timeout -k 10 400 python -u bench/bench_multitenant_service.py --users-total 4000 --rows 800 --batch 1024 --steps 5 --warmup 2 --global-batch 128 --global-steps 5 > gpurun_out/mt_bench.json 2> gpurun_out/mt_bench.err || exit 6
