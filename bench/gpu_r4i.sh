# full GPU test tier (round 4 state)
set -o pipefail
export PYTHONPATH=$PWD
mkdir -p gpurun_out
timeout -k 10 1000 python -u -m pytest -x -v -m gpu --timeout 240 --timeout-method thread tests/ > gpurun_out/pytest_gpu_r4i.log 2>&1
rc=$?
echo "pytest rc=$rc" >> gpurun_out/pytest_gpu_r4i.log
exit $rc
