# round-4 pass 4: stage profile of the row-sharded exact cadence, and the
# 1-rank torchrun bench (routed search over RCCL)
set -o pipefail
export PYTHONPATH=$PWD
mkdir -p gpurun_out
LZK_TRACE=1 timeout -k 10 500 python -u bench/bench_consolidate.py --sharded --clustered --nodes 10000000 --convs 128 --steps 3 --warmup 1 > gpurun_out/sharded_stages.json 2> gpurun_out/sharded_stages.err || exit 1
timeout -k 10 900 python -u -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 1 --consolidate-steps 0 --sharded-steps 0 --json-out gpurun_out/bench_r4_torchrun2.json > gpurun_out/bench_r4_torchrun2.log 2>&1 || exit 2
