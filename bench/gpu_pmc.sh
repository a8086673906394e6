#!/bin/bash
# rocprofv3 counter passes over the int8 scan and the encoder GEMMs (round-5 working script)
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
export PYTHONPATH=$PWD${PYTHONPATH:+:$PYTHONPATH}
OUT=${OUT:-gpurun_out/pmc}
mkdir -p $OUT
PA="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_INSTS_VALU GRBM_GUI_ACTIVE"
PB="SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_SALU SQ_ACTIVE_INST_ANY FETCH_SIZE GRBM_COUNT"
P_REPS=3 timeout -s KILL 150 rocprofv3 --pmc $PA --output-format csv -d /tmp/pmc_embA -o run -- python3 bench/prof_embed.py > $OUT/embA.log 2>&1 || exit 1
P_REPS=3 timeout -s KILL 150 rocprofv3 --pmc $PB --output-format csv -d /tmp/pmc_embB -o run -- python3 bench/prof_embed.py > $OUT/embB.log 2>&1 || exit 1
timeout -s KILL 200 rocprofv3 --pmc $PA --output-format csv -d /tmp/pmc_scanA -o run -- python3 bench/probe_i8_scan.py 4000000 > $OUT/scanA.log 2>&1 || exit 1
timeout -s KILL 200 rocprofv3 --pmc $PB --output-format csv -d /tmp/pmc_scanB -o run -- python3 bench/probe_i8_scan.py 4000000 > $OUT/scanB.log 2>&1 || exit 1
python3 bench/pmc_summary.py /tmp/pmc_embA /tmp/pmc_embB > $OUT/embed_pmc.json && python3 bench/pmc_summary.py /tmp/pmc_scanA /tmp/pmc_scanB > $OUT/scan_pmc.json
mkdir -p $OUT/raw && for d in embA embB scanA scanB; do cp /tmp/pmc_$d/run_counter_collection.csv $OUT/raw/$d.csv; done
