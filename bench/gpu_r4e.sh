# round-4 pass 5: consolidation stage profile (reference cadence, default
# graph and persistent 20M-edge graph) and per-step kernel launches (two
# kernel traces, 2 and 7 timed steps; the difference is 5 steps)
set -o pipefail
export PYTHONPATH=$PWD
mkdir -p gpurun_out/prof_cons
LZK_TRACE=1 timeout -k 10 400 python -u bench/bench_consolidate.py --steps 5 --warmup 2 > gpurun_out/cons_stages.json 2> gpurun_out/cons_stages.err || exit 1
LZK_TRACE=1 timeout -k 10 400 python -u bench/bench_consolidate.py --steps 5 --warmup 2 --prune-threshold 0 > gpurun_out/cons_persist_stages.json 2> gpurun_out/cons_persist_stages.err || exit 2
R=$PWD
cd /tmp && export TMPDIR=/tmp
for s in 2 7; do
  timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_cons/s$s -o cons -- python3 $R/bench/bench_consolidate.py --steps $s --warmup 1 > $R/gpurun_out/prof_cons/cons_s$s.log 2>&1 || exit 3
  for db in $(find $R/gpurun_out/prof_cons/s$s -name "*.db"); do python3 $R/bench/rocpd_summary.py $db --top 40 --csv $R/gpurun_out/prof_cons/kernels_s$s.csv > $R/gpurun_out/prof_cons/kernels_s$s.txt; rm -f $db; done
  find $R/gpurun_out/prof_cons/s$s -type f -size +4M -delete
done
