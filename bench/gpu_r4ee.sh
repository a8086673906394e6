# union-find variants: probe, then the persistent-graph consolidation A/B with cached loads
set -o pipefail
export PYTHONPATH=$PWD
mkdir -p gpurun_out
timeout -k 10 200 python -u bench/probe_uf_variants.py > gpurun_out/uf_variants.log 2>&1 || exit 1
timeout -k 10 300 python -u -m pytest -x -v -m gpu --timeout 120 --timeout-method thread tests/ -k "component or digest or cc_ or union" > gpurun_out/t_uf.log 2>&1 || exit 2
LZK_UF_PLAIN=1 timeout -k 10 300 python -u -m pytest -x -v -m gpu --timeout 120 --timeout-method thread tests/ -k "component or digest or cc_ or union" > gpurun_out/t_uf_plain.log 2>&1 || exit 3
for b in 1 0; do
  LZK_UF_PLAIN=$b timeout -k 10 300 python -u bench/bench_consolidate.py --steps 5 --warmup 2 --prune-threshold 0 > gpurun_out/uf_pers_$b.json 2> gpurun_out/uf_pers_$b.err || exit 4
done
