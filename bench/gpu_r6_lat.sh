#!/bin/bash
# round 6: single-query latency over a 10M-memory tenant, then a kernel trace of it
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
export PYTHONPATH=$PWD${PYTHONPATH:+:$PYTHONPATH}
OUT=${OUT:-gpurun_out/r6lat}
mkdir -p $OUT
if [ -z "$NOTEST" ]; then
  timeout -k 10 600 python -u -m pytest tests/kernels/test_tenant_engine_gpu.py -m gpu -x -v --timeout 240 \
    --timeout-method thread -k "${TESTK:-narrow or i8 or certificate or rerank or store_search}" > $OUT/pytest.log 2>&1 || exit 1
fi
timeout -k 10 300 python bench/bench_latency.py --api-only --iters 200 > $OUT/lat.json 2> $OUT/lat.err || exit 1
timeout -s KILL 300 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/kt_lat -o run -- python3 bench/bench_latency.py --api-only --iters 100 > $OUT/lat_kt.json 2> $OUT/lat_kt.err || exit 1
cp /tmp/kt_lat/run_kernel_stats.csv $OUT/
python3 - /tmp/kt_lat/run_kernel_trace.csv > $OUT/last_search_kernels.txt <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
# the last narrow scan and the kernels around it (one store search)
idx = max(i for i, r in enumerate(rows) if "scan8_narrow" in r["Kernel_Name"])
t0 = int(rows[idx]["Start_Timestamp"])
for r in rows[max(0, idx - 12): idx + 14]:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    print(f"{(s - t0) / 1e3:9.1f}us {(e - s) / 1e3:8.1f}us  {r['Kernel_Name'][:100]}")
PY
