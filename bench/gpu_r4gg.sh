# union-find stage count A/B on the persistent-graph consolidation (cached loads), alternating repeats
set -o pipefail
export PYTHONPATH=$PWD
mkdir -p gpurun_out
for s in 4 0 4 0 3 6; do
  LZK_UF_STAGES=$s timeout -k 10 300 python -u bench/bench_consolidate.py --steps 5 --warmup 2 --prune-threshold 0 >> gpurun_out/ufs_rep_$s.json 2>> gpurun_out/ufs_rep_$s.err || exit 1
done
