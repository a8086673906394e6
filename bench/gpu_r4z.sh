# final round-4 checks: full bench, and the 1-rank torchrun bench with every collective on RCCL
set -o pipefail
export PYTHONPATH=$PWD
mkdir -p gpurun_out
timeout -k 10 600 python -u bench.py --json-out gpurun_out/bench_final.json > gpurun_out/bench_final.log 2>&1 || exit 1
timeout -k 10 500 python -u -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29541 bench.py --gpus 1 --consolidate-steps 3 --sharded-steps 2 --json-out gpurun_out/bench_final_torchrun.json > gpurun_out/bench_final_torchrun.log 2>&1 || exit 2
