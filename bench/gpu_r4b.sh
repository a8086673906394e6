# round-4 pass 2: the 1-GPU bench (default flags) and the same bench as a
# 1-rank torch.distributed.run job with every collective forced through RCCL,
# then a kernel-trace profile of a short bench run
set -o pipefail
export PYTHONPATH=$PWD
mkdir -p gpurun_out
timeout -k 10 900 python -u bench.py --json-out gpurun_out/bench_r4.json > gpurun_out/bench_r4.log 2>&1 || exit 1
timeout -k 10 900 python -u -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 1 --json-out gpurun_out/bench_r4_torchrun.json > gpurun_out/bench_r4_torchrun.log 2>&1 || exit 2
R=$PWD
mkdir -p gpurun_out/prof_ab8
cd /tmp && export TMPDIR=/tmp
AB_ROUNDS=1 timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_ab8 -o ab -- python3 $R/bench/ab_scan8.py > $R/gpurun_out/prof_ab8/ab.log 2>&1 || exit 3
