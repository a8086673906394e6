#!/bin/bash
# attention kernel re-layout: parity tests + kernel time + LDS counters (round-5 working script)
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
export PYTHONPATH=$PWD${PYTHONPATH:+:$PYTHONPATH}
OUT=${OUT:-gpurun_out/attn}
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/kernels/test_encoder_parity_gpu.py -x -v --timeout 240 --timeout-method thread > $OUT/pytest.log 2>&1 || exit 1
P_REPS=10 timeout -s KILL 150 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/attn_kt -o run -- python3 bench/prof_embed.py > $OUT/kt.log 2>&1 || exit 1
cp /tmp/attn_kt/run_kernel_stats.csv $OUT/kernel_stats.csv
P_REPS=3 timeout -s KILL 150 rocprofv3 --pmc SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_BUSY_CYCLES --output-format csv -d /tmp/attn_pmc -o run -- python3 bench/prof_embed.py > $OUT/pmc.log 2>&1 || exit 1
python3 bench/pmc_summary.py /tmp/attn_pmc > $OUT/pmc.json
