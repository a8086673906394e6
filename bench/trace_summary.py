"""Summarise a rocprofv3 --kernel-trace csv: per-kernel totals for the last
N dispatches' window and the wall span / idle gaps of that window."""
import csv
import sys
from collections import defaultdict


def main(path, last=None):
    rows = list(csv.DictReader(open(path)))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    if last:
        rows = rows[-int(last):]
    agg = defaultdict(lambda: [0, 0])
    busy = 0
    gaps = 0
    prev_end = None
    for r in rows:
        s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        k = r["Kernel_Name"][:70]
        agg[k][0] += 1
        agg[k][1] += e - s
        busy += e - s
        if prev_end is not None and s > prev_end:
            gaps += s - prev_end
        prev_end = max(prev_end or 0, e)
    span = int(rows[-1]["End_Timestamp"]) - int(rows[0]["Start_Timestamp"])
    for k, (n, t) in sorted(agg.items(), key=lambda kv: -kv[1][1]):
        print(f"{k:70s} {n:5d} {t / 1e3:9.1f}us {t / n / 1e3:8.1f}us")
    print(f"span {span / 1e3:.1f}us busy {busy / 1e3:.1f}us gaps {gaps / 1e3:.1f}us dispatches {len(rows)}")


if __name__ == "__main__":
    main(*sys.argv[1:])
