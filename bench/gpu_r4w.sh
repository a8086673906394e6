set -o pipefail
export PYTHONPATH=$PWD
mkdir -p gpurun_out
for d in auto 0; do
  LZK_DUAL_LOWP=$d timeout -k 10 400 python -u bench/bench_consolidate.py --sharded --clustered --nodes 10000000 --convs 128 --steps 3 --warmup 1 > gpurun_out/sh10_$d.json 2> gpurun_out/sh10_$d.err || exit 1
done
timeout -k 10 400 python -u bench/bench_consolidate.py --steps 5 --warmup 2 > gpurun_out/cons_r4w.json 2> gpurun_out/cons_r4w.err || exit 2
