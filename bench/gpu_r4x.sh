# full GPU tier + smoke (round-end rehearsal)
set -o pipefail
export PYTHONPATH=$PWD
mkdir -p gpurun_out
timeout -k 10 1000 python -u -m pytest -v -m gpu --timeout 240 --timeout-method thread tests/ > gpurun_out/pytest_gpu_r4x.log 2>&1
rc=$?
echo "pytest rc=$rc" >> gpurun_out/pytest_gpu_r4x.log
if [ $rc -ne 0 ]; then exit 11; fi
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/smoke_r4x.log 2>&1 || exit 12
