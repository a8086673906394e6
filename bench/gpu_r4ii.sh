# round-end numbers with every default: smoke, full bench, sharded consolidation
set -o pipefail
export PYTHONPATH=$PWD
mkdir -p gpurun_out
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/smoke_ii.log 2>&1 || exit 1
timeout -k 10 600 python -u bench.py --json-out gpurun_out/bench_ii.json > gpurun_out/bench_ii.log 2>&1 || exit 2
