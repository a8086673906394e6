#!/bin/bash
# attention re-layout A/B: kernel times of the bge-base embed, new vs previous build (round-5 working script)
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=${OUT:-gpurun_out/attn_ab}
mkdir -p $OUT
for v in new old new2 old2; do
  case $v in new*) S=bench/prof_embed.py ;; old*) S=abold/bench/prof_embed.py ;; esac
  P_REPS=10 timeout -s KILL 150 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/ab_$v -o run -- python3 $S > $OUT/$v.log 2>&1 || exit 1
  cp /tmp/ab_$v/run_kernel_stats.csv $OUT/$v.csv
done
