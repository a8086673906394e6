#!/bin/bash
# round 6: fp8 encoder (LayerNorm-fused e4m3 inputs) -- tests, embed profile, then config 5 end to end
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
export PYTHONPATH=$PWD${PYTHONPATH:+:$PYTHONPATH}
OUT=${OUT:-gpurun_out/r6cfg5}
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/kernels/test_kernels_gpu.py tests/kernels/test_encoder_parity_gpu.py -m gpu -x -v \
  --timeout 240 --timeout-method thread -k "fp8 or layernorm or parity" > $OUT/pytest.log 2>&1 || exit 1
P_MODEL=e5-large P_PREC=fp8 P_REPS=10 timeout -s KILL 300 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/kt_e5 -o run -- python3 bench/prof_embed.py > $OUT/e5.log 2>&1 || exit 1
cp /tmp/kt_e5/run_kernel_stats.csv $OUT/e5-large_fp8_kernel_stats.csv
if [ -z "$NOCFG5" ]; then
  timeout -k 10 900 python -u bench/bench_ivfpq_scale.py --nprobes 8,16 --reranks 4096 --out $OUT/ivfpq_200M.json > $OUT/ivfpq.log 2>&1 || exit 1
fi
