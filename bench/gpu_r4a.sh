# round-4 validation pass: new kernel tests, scan A/Bs, RCCL world-1 test
set -o pipefail
export PYTHONPATH=$PWD
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/kernels/test_tenant_engine_gpu.py tests/kernels/test_graph_kernels_gpu.py -k "scan8 or i8 or zero_row or rigorous or farthest or rerank64 or lean" > gpurun_out/t_new.log 2>&1 || exit 1
timeout -k 10 400 python -u bench/ab_scan8.py > gpurun_out/ab_scan8.json 2> gpurun_out/ab_scan8.err || exit 2
timeout -k 10 300 python -u bench/ab_scan8_narrow.py > gpurun_out/ab_narrow.json 2> gpurun_out/ab_narrow.err || exit 3
timeout -k 10 330 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/kernels/test_rccl_world1_gpu.py > gpurun_out/t_rccl.log 2>&1 || exit 4
timeout -k 10 300 python -u -m pytest -x -v --timeout 240 --timeout-method thread tests/kernels/test_service_gpu.py -k "global_multi" > gpurun_out/t_mt.log 2>&1 || exit 5
timeout -k 10 400 python -u bench/bench_multitenant_service.py --users-total 4000 --rows 800 --batch 1024 --steps 5 --warmup 2 --global-batch 128 --global-steps 5 > gpurun_out/mt_bench.json 2> gpurun_out/mt_bench.err || exit 6
