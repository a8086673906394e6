#!/bin/bash
# Round-3 consolidation profile at the reference cadence (10M rows, 20M
# edges, prune_threshold 0): per-stage trace + rocprofv3 kernel stats.
cd "$GRAFT_REPO_ROOT" || exit 1
export PYTHONPATH="$GRAFT_REPO_ROOT" LZK_AUTOBUILD=0
OUT="$GRAFT_REPO_ROOT/gpurun_out/r3_cons"
mkdir -p "$OUT"
LZK_TRACE=1 timeout -k 10 300 python -u bench/bench_consolidate.py --steps 3 --warmup 1 --prune-threshold 0 > "$OUT/trace_p0.log" 2>&1
rc=$?; echo "trace rc=$rc" | tee -a "$OUT/passes.log"; [ $rc -ne 0 ] && exit $rc
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/kt" -o run -- python3 "$GRAFT_REPO_ROOT/bench/bench_consolidate.py" --steps 2 --warmup 1 --prune-threshold 0 > "$OUT/kt.log" 2>&1
rc=$?; echo "ktrace rc=$rc" | tee -a "$OUT/passes.log"; exit $rc
