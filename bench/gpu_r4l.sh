# narrow store search after the query-prep / merge work: tests, Q=1 probe + timeline, latency bench
set -o pipefail
export PYTHONPATH=$PWD
mkdir -p gpurun_out/prof_q1b
timeout -k 10 600 python -u -m pytest -x -v -m gpu --timeout 240 --timeout-method thread tests/kernels/test_query_prep_gpu.py tests/kernels/test_tenant_engine_gpu.py tests/kernels/test_kernels_gpu.py > gpurun_out/t_r4l.log 2>&1
rc=$?
echo "pytest rc=$rc" >> gpurun_out/t_r4l.log
if [ $rc -ne 0 ]; then exit 11; fi
R=$PWD
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace -d $R/gpurun_out/prof_q1b/t -o q1 -- python3 $R/bench/probe_q1.py --iters 30 > $R/gpurun_out/prof_q1b/q1.log 2>&1 || exit 6
for db in $(find $R/gpurun_out/prof_q1b/t -name "*.db"); do python3 $R/bench/rocpd_summary.py $db --top 25 --timeline 40 > $R/gpurun_out/prof_q1b/q1_timeline.txt; rm -f $db; done
find $R/gpurun_out/prof_q1b/t -type f -size +4M -delete
cd $R
timeout -k 10 400 python -u bench/bench_latency.py --iters 100 > gpurun_out/latency_r4b.json 2> gpurun_out/latency_r4b.err || exit 7
