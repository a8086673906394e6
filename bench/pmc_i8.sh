#!/bin/bash
# Round-3 PMC capture of the two hot kernels (scan: bench/pmc_search.py,
# embed: bench/prof_embed.py), one counter group per rocprofv3 run, plus a
# kernel-trace stats run of the embed. Output under gpurun_out/r3_pmc_i8/.
cd "$GRAFT_REPO_ROOT" || exit 1
export PYTHONPATH="$GRAFT_REPO_ROOT" LZK_AUTOBUILD=0
cd /tmp && export TMPDIR=/tmp
OUT="$GRAFT_REPO_ROOT/gpurun_out/r3_pmc_i8"
mkdir -p "$OUT"
G1="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE"
G2="SQ_INSTS_LDS SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVES GRBM_COUNT"
G3="FETCH_SIZE GRBM_GUI_ACTIVE"
i=0
for prog in "bench/pmc_search_i8.py"; do
  for grp in "$G1" "$G2" "$G3"; do
    i=$((i+1))
    timeout -s KILL 150 rocprofv3 --pmc $grp --output-format csv -d "$OUT/p$i" -o run -- python3 "$GRAFT_REPO_ROOT/$prog" > "$OUT/p$i.log" 2>&1
    rc=$?
    echo "pass $i ($prog) rc=$rc" | tee -a "$OUT/passes.log"
    [ $rc -ne 0 ] && exit $rc
  done
done
