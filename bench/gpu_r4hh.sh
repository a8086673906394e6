# confirm the 4-stage union-find default: graph/digest GPU tests and the persistent-graph consolidation
set -o pipefail
export PYTHONPATH=$PWD
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -v -m gpu --timeout 120 --timeout-method thread tests/ -k "component or digest or cc_ or union or consolidat" > gpurun_out/t_hh.log 2>&1 || exit 1
timeout -k 10 300 python -u bench/bench_consolidate.py --steps 5 --warmup 2 --prune-threshold 0 > gpurun_out/hh_pers.json 2> gpurun_out/hh_pers.err || exit 2
