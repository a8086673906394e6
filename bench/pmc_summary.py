"""Summarise rocprofv3 --pmc csv passes: per kernel (name prefix), summed
counter values over its dispatches and derived ratios. Usage:
pmc_summary.py DIR [DIR ...] -> one JSON on stdout."""
import csv
import glob
import json
import sys
from collections import defaultdict


def short(name):
    name = name.replace("(anonymous namespace)::", "")
    return name.split("(")[0][:120]


def main():
    tot = defaultdict(lambda: defaultdict(float))
    disp = defaultdict(set)
    for d in sys.argv[1:]:
        for f in glob.glob(f"{d}/**/*counter_collection.csv", recursive=True):
            with open(f) as fh:
                for row in csv.DictReader(fh):
                    k = short(row.get("Kernel_Name", "?"))
                    tot[k][row["Counter_Name"]] += float(row["Counter_Value"])
                    disp[(d, k)].add(row.get("Dispatch_Id"))
    out = {}
    for k, c in tot.items():
        n = max(len(disp.get((d, k), ())) for d in sys.argv[1:])
        r = {"dispatches": n, "counters": {a: round(v / max(n, 1), 1) for a, v in sorted(c.items())}}
        wc = c.get("SQ_WAVE_CYCLES", 0)
        if wc:
            r["wait_frac"] = round(c.get("SQ_WAIT_ANY", 0) / wc, 4)
            r["wait_inst_frac"] = round(c.get("SQ_WAIT_INST_ANY", 0) / wc, 4)
        if c.get("SQ_BUSY_CYCLES"):
            # MFMA pipe busy per SIMD-cycle (4 SIMDs per CU; SQ_BUSY_CYCLES per SE summed)
            r["mfma_busy_per_busy_cycle"] = round(c.get("SQ_VALU_MFMA_BUSY_CYCLES", 0) / c["SQ_BUSY_CYCLES"], 4)
        if c.get("SQ_LDS_IDX_ACTIVE"):
            r["lds_bank_conflict_frac"] = round(c.get("SQ_LDS_BANK_CONFLICT", 0) / c["SQ_LDS_IDX_ACTIVE"], 4)
        if c.get("FETCH_SIZE"):
            r["fetch_gb_per_dispatch"] = round(c["FETCH_SIZE"] / max(n, 1) / 1e6, 3)
        out[k] = r
    top = dict(sorted(out.items(), key=lambda kv: -kv[1]["counters"].get("SQ_BUSY_CYCLES", 0))[:12])
    print(json.dumps(top, indent=1))


if __name__ == "__main__":
    main()
