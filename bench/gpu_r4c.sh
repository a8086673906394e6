# round-4 pass 3: kernel-trace profile of a short bench run, one 40M-row lean
# tenant, and the int8 dual consolidation scan on the clustered row-sharded
# run (LZK_DUAL_LOWP A/B)
set -o pipefail
export PYTHONPATH=$PWD
mkdir -p gpurun_out/prof_r4
R=$PWD
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_r4 -o bench -- python3 $R/bench.py --steps 5 --warmup 2 --consolidate-steps 3 --sharded-steps 2 --no-persistent-graph > $R/gpurun_out/prof_r4/bench.log 2>&1 || exit 1
cd $R
# keep only the per-kernel summary (the raw trace database exceeds what a call may return)
for db in $(find gpurun_out/prof_r4 -name "*.db"); do python3 bench/rocpd_summary.py $db --top 60 --csv gpurun_out/prof_r4/bench_kernel_stats.csv > gpurun_out/prof_r4/bench_kernel_summary.txt; rm -f $db; done
find gpurun_out/prof_r4 -name "*.csv" -size +8M -delete
timeout -k 10 420 python -u bench/bench_big_tenant.py --rows 40000000 --steps 10 --out gpurun_out/big_tenant.json > gpurun_out/big_tenant.log 2>&1 || exit 2
for d in 0 1; do
  LZK_DUAL_LOWP=$d timeout -k 10 300 python -u bench/bench_consolidate.py --sharded --clustered --nodes 2000000 --convs 128 --steps 4 --warmup 1 > gpurun_out/dual_lowp_$d.json 2> gpurun_out/dual_lowp_$d.err || exit 3
done
