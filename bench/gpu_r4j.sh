# consolidation after the segment work: default, int8 dual scan A/B, persistent graph, stages
set -o pipefail
export PYTHONPATH=$PWD
mkdir -p gpurun_out
timeout -k 10 400 python -u bench/bench_consolidate.py --steps 5 --warmup 2 > gpurun_out/cons_r4j.json 2> gpurun_out/cons_r4j.err || exit 1
LZK_DUAL_LOWP=1 timeout -k 10 400 python -u bench/bench_consolidate.py --steps 5 --warmup 2 > gpurun_out/cons_r4j_dual.json 2> gpurun_out/cons_r4j_dual.err || exit 2
timeout -k 10 400 python -u bench/bench_consolidate.py --steps 5 --warmup 2 --prune-threshold 0 > gpurun_out/cons_r4j_persist.json 2> gpurun_out/cons_r4j_persist.err || exit 3
LZK_TRACE=1 timeout -k 10 400 python -u bench/bench_consolidate.py --steps 5 --warmup 2 > gpurun_out/cons_r4j_stages.json 2> gpurun_out/cons_r4j_stages.err || exit 4
mkdir -p gpurun_out/prof_cons2
R=$PWD
cd /tmp && export TMPDIR=/tmp
for s in 2 7; do
  timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_cons2/s$s -o cons -- python3 $R/bench/bench_consolidate.py --steps $s --warmup 1 > $R/gpurun_out/prof_cons2/cons_s$s.log 2>&1 || exit 5
  for db in $(find $R/gpurun_out/prof_cons2/s$s -name "*.db"); do python3 $R/bench/rocpd_summary.py $db --top 40 --csv $R/gpurun_out/prof_cons2/kernels_s$s.csv > $R/gpurun_out/prof_cons2/kernels_s$s.txt; rm -f $db; done
  find $R/gpurun_out/prof_cons2/s$s -type f -size +4M -delete
done
cd $R
mkdir -p gpurun_out/prof_q1
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace -d $R/gpurun_out/prof_q1/t -o q1 -- python3 $R/bench/probe_q1.py --iters 30 > $R/gpurun_out/prof_q1/q1.log 2>&1 || exit 6
for db in $(find $R/gpurun_out/prof_q1/t -name "*.db"); do python3 $R/bench/rocpd_summary.py $db --top 25 --timeline 60 > $R/gpurun_out/prof_q1/q1_timeline.txt; rm -f $db; done
find $R/gpurun_out/prof_q1/t -type f -size +4M -delete
