# end-of-round check with cached union-find loads as default: GPU tier, smoke, full bench
set -o pipefail
export PYTHONPATH=$PWD
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -v -m gpu --timeout 120 --timeout-method thread tests/ > gpurun_out/t_ff.log 2>&1 || exit 1
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/smoke_ff.log 2>&1 || exit 2
timeout -k 10 600 python -u bench.py --json-out gpurun_out/bench_ff.json > gpurun_out/bench_ff.log 2>&1 || exit 3
