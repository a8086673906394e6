# scan8 re-check: the int8 tests with the wide kernel on, then the A/B
set -o pipefail
export PYTHONPATH=$PWD
mkdir -p gpurun_out
LZK_SCAN8=1 timeout -k 10 400 python -u -m pytest -v --timeout 240 --timeout-method thread tests/kernels/test_tenant_engine_gpu.py -k "scan8 or i8 or lowp or zero_row or rigorous or lean" > gpurun_out/t_scan8.log 2>&1
rc=$?
echo "pytest rc=$rc" >> gpurun_out/t_scan8.log
if [ $rc -ne 0 ]; then exit 11; fi
timeout -k 10 400 python -u bench/ab_scan8.py > gpurun_out/ab_scan8.json 2> gpurun_out/ab_scan8.err || exit 2
