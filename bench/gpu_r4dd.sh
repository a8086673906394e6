# per-kernel profile of the persistent-graph consolidation (prune threshold 0); steps 1 vs 3 -> per-step by difference
set -o pipefail
export PYTHONPATH=$PWD
R=$PWD
mkdir -p gpurun_out/prof_pers
cd /tmp && export TMPDIR=/tmp
for s in 1 3; do
  timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_pers/s$s -o pers -- python3 $R/bench/bench_consolidate.py --steps $s --warmup 1 --prune-threshold 0 > $R/gpurun_out/prof_pers/pers_s$s.log 2>&1 || exit 3
  for db in $(find $R/gpurun_out/prof_pers/s$s -name "*.db"); do python3 $R/bench/rocpd_summary.py $db --top 40 --csv $R/gpurun_out/prof_pers/kernels_s$s.csv > $R/gpurun_out/prof_pers/kernels_s$s.txt; rm -f $db; done
done
