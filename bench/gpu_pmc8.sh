# PMC passes of the wide int8 scan: scan8 with candidates, scan8 with thr=inf,
# and the template with candidates (one counter group per rocprofv3 run)
set -o pipefail
R=$PWD
export PYTHONPATH=$R LZK_AUTOBUILD=0
OUT=$R/gpurun_out/pmc8
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
G1="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_SALU GRBM_GUI_ACTIVE"
G2="SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_INSTS_VMEM SQ_WAIT_INST_LDS GRBM_COUNT"
i=0
for mode in cand inf tmpl; do
  for grp in "$G1" "$G2"; do
    i=$((i+1))
    if [ $mode = inf ]; then export PROBE_INF=1; else unset PROBE_INF; fi
    if [ $mode = tmpl ]; then export PROBE_TEMPLATE=1; else unset PROBE_TEMPLATE; fi
    timeout -s KILL 240 rocprofv3 --pmc $grp --output-format csv -d $OUT/p$i -o run -- python3 $R/bench/probe_scan8_epilogue.py > $OUT/p$i.log 2>&1
    rc=$?
    echo "pass $i mode=$mode rc=$rc" >> $OUT/passes.log
    [ $rc -ne 0 ] && exit $rc
    python3 $R/bench/pmc_reduce.py $OUT/p$i "scan8_kernel|flat_cand_persistent" > $OUT/p$i.json
    rm -rf $OUT/p$i
  done
done
exit 0
