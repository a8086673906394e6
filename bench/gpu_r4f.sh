# round-4 pass 6: sync-free consolidation points (O(edges) digest, first-rows
# kernel, deferred profile prompts): GPU tests, then the consolidation bench
set -o pipefail
export PYTHONPATH=$PWD
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -v -m gpu --timeout 240 --timeout-method thread tests/kernels/test_digest_gpu.py tests/unit/test_consolidate_batch_exact.py tests/unit/test_memory_system.py > gpurun_out/t_r4f.log 2>&1
rc=$?
echo "pytest rc=$rc" >> gpurun_out/t_r4f.log
if [ $rc -ne 0 ]; then exit 11; fi
timeout -k 10 400 python -u bench/bench_consolidate.py --steps 5 --warmup 2 > gpurun_out/cons_r4f.json 2> gpurun_out/cons_r4f.err || exit 2
LZK_TRACE=1 timeout -k 10 400 python -u bench/bench_consolidate.py --steps 5 --warmup 2 > gpurun_out/cons_r4f_stages.json 2> gpurun_out/cons_r4f_stages.err || exit 3
timeout -k 10 400 python -u bench/bench_consolidate.py --steps 5 --warmup 2 --prune-threshold 0 > gpurun_out/cons_r4f_persist.json 2> gpurun_out/cons_r4f_persist.err || exit 4
