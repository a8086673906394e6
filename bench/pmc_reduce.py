"""Reduce a rocprofv3 --pmc CSV directory to per-kernel counter sums for the
kernels whose name matches a pattern (JSON on stdout); the raw CSVs of a
python run hold every dispatch of every kernel and are too large to keep."""
import csv
import glob
import json
import re
import sys
from collections import defaultdict


def main():
    d, pat = sys.argv[1], re.compile(sys.argv[2])
    out = defaultdict(lambda: defaultdict(float))
    calls = defaultdict(set)
    for f in glob.glob(f"{d}/**/*counter_collection.csv", recursive=True):
        with open(f, newline="") as fh:
            for row in csv.DictReader(fh):
                name = row.get("Kernel_Name") or row.get("Kernel-Name") or ""
                if not pat.search(name):
                    continue
                key = name.split("(")[0][-90:]
                cnt = row.get("Counter_Name") or row.get("Counter-Name")
                val = float(row.get("Counter_Value") or row.get("Counter-Value") or 0)
                out[key][cnt] += val
                calls[key].add(row.get("Dispatch_Id") or row.get("Dispatch-Id"))
    print(json.dumps({k: {"dispatches": len(calls[k]), **v} for k, v in out.items()}, indent=1))


if __name__ == "__main__":
    main()
