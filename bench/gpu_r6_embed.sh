#!/bin/bash
# round 6: kernel profile of the batch embed -- bge-base bf16 (headline) and e5-large fp8 (config 5)
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
export PYTHONPATH=$PWD${PYTHONPATH:+:$PYTHONPATH}
OUT=${OUT:-gpurun_out/r6embed}
mkdir -p $OUT
for cfg in "bge-base:bf16" "e5-large:fp8"; do
  m=${cfg%%:*}; pr=${cfg##*:}
  P_MODEL=$m P_PREC=$pr P_REPS=10 timeout -s KILL 300 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/kt_$m -o run -- python3 bench/prof_embed.py > $OUT/${m}.log 2>&1 || exit 1
  cp /tmp/kt_$m/run_kernel_stats.csv $OUT/${m}_${pr}_kernel_stats.csv
done
