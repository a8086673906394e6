# speculative threshold check: the int8 / lean tests, the scan A/B, the headline bench
set -o pipefail
export PYTHONPATH=$PWD
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -v --timeout 240 --timeout-method thread tests/kernels/test_tenant_engine_gpu.py -k "i8 or lowp or zero_row or rigorous or lean or narrow" > gpurun_out/t_spec.log 2>&1
rc=$?
echo "pytest rc=$rc" >> gpurun_out/t_spec.log
if [ $rc -ne 0 ]; then exit 11; fi
timeout -k 10 400 python -u bench/ab_scan8.py > gpurun_out/ab_scan8.json 2> gpurun_out/ab_scan8.err || exit 2
timeout -k 10 600 python -u bench.py --consolidate-steps 0 --sharded-steps 0 --no-persistent-graph --json-out gpurun_out/bench_spec.json > gpurun_out/bench_spec.log 2>&1 || exit 3
