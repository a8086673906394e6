#!/bin/bash
# round 6: PMC counters of the headline's two halves (store search scan, bge-base embed), one pass per counter set
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
export PYTHONPATH=$PWD${PYTHONPATH:+:$PYTHONPATH}
OUT=${OUT:-gpurun_out/r6pmc}
mkdir -p $OUT
A="SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU SQ_WAIT_INST_ANY SQ_INSTS_LDS GRBM_GUI_ACTIVE"
B="FETCH_SIZE SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_ANY"
for tgt in store_search embed; do
  for pass in A B; do
    C=$A; [ $pass = B ] && C=$B
    P_REPS=3 timeout -s KILL 240 rocprofv3 --pmc $C --output-format csv -d /tmp/pmc_${tgt}_$pass -o run -- python3 bench/prof_$tgt.py > $OUT/${tgt}_$pass.log 2>&1 || exit 1
  done
  python3 bench/pmc_summary.py /tmp/pmc_${tgt}_A /tmp/pmc_${tgt}_B > $OUT/${tgt}_pmc.json || exit 1
done
