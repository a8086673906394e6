#!/bin/bash
# the headline's timed loop under rocprofv3 --kernel-trace: per-step kernels
# of exactly the timed steps (bench.py stops after the loop), classified by
# tools/ktrace_window.py (hand-written / ATen / library GEMM / copies)
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
export PYTHONPATH=$PWD${PYTHONPATH:+:$PYTHONPATH}
OUT=${OUT:-gpurun_out/r6headtrace}
mkdir -p $OUT
LZK_BENCH_STOP_AFTER_HEADLINE=1 timeout -s KILL 400 rocprofv3 --kernel-trace --memory-copy-trace --stats --output-format csv -d /tmp/kt_head -o run -- python3 bench.py --gpus 1 --steps 20 --warmup 5 > $OUT/head.json 2> $OUT/head.err || exit 1
MS=$(python3 -c "
import json
r=None
for l in open('$OUT/head.json'):
    try: d=json.loads(l)
    except Exception: continue
    if 'ms_per_step' in d: r=d
print(r['ms_per_step']*r['steps'])")
python3 tools/ktrace_window.py /tmp/kt_head/run_kernel_trace.csv $MS 20 $OUT/head_window.json > /dev/null || exit 1
cp /tmp/kt_head/run_kernel_stats.csv $OUT/head_kernel_stats.csv || exit 1
python3 - $MS > $OUT/head_copies.txt <<'PY' || exit 1
import csv, sys, glob
ms = float(sys.argv[1])
rows = list(csv.DictReader(open('/tmp/kt_head/run_kernel_trace.csv')))
t1 = max(int(r['End_Timestamp']) for r in rows)
t0 = t1 - int(ms * 1e6)
print('kernel trace columns:', list(rows[0].keys()))
n = 0
for r in rows:
    if r['Kernel_Name'].startswith('__amd_rocclr') and int(r['End_Timestamp']) > t0:
        n += 1
        if n <= 40:
            print({k: r[k] for k in r if k in ('Kernel_Name', 'Grid_Size', 'Grid_Size_X', 'Workgroup_Size', 'Queue_Id', 'Stream_Id')},
                  'dur_us', (int(r['End_Timestamp']) - int(r['Start_Timestamp'])) / 1e3,
                  't_ms', (int(r['Start_Timestamp']) - t0) / 1e6)
for f in glob.glob('/tmp/kt_head/*memory_copy*.csv'):
    mc = list(csv.DictReader(open(f)))
    print(f, 'columns', list(mc[0].keys()) if mc else None)
    k = 0
    for r in mc:
        if int(r.get('End_Timestamp', 0)) > t0:
            k += 1
            if k <= 40:
                print({c: r[c] for c in r if c in ('Direction', 'Size', 'Src_Agent_Id', 'Dst_Agent_Id', 'Stream_Id')},
                      'dur_us', (int(r['End_Timestamp']) - int(r['Start_Timestamp'])) / 1e3)
    print('copies in window', k)
PY
