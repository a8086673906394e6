# int8 dual scan auto mode: default consolidation bench, clustered sharded A/B
set -o pipefail
export PYTHONPATH=$PWD
mkdir -p gpurun_out
timeout -k 10 400 python -u bench/bench_consolidate.py --steps 5 --warmup 2 > gpurun_out/cons_r4k_auto.json 2> gpurun_out/cons_r4k_auto.err || exit 1
for d in auto 0; do
  LZK_DUAL_LOWP=$d timeout -k 10 300 python -u bench/bench_consolidate.py --sharded --clustered --nodes 2000000 --convs 128 --steps 4 --warmup 1 > gpurun_out/shard_cl_$d.json 2> gpurun_out/shard_cl_$d.err || exit 2
done
