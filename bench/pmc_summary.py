"""Summarise rocprofv3 --pmc passes (bench/pmc_r3.sh output) per kernel:
median counters over the dispatches of each kernel whose name contains one
of the given substrings, plus derived rates. MI355X: GRBM_GUI_ACTIVE is
summed over the 8 XCDs; 1024 SIMDs, so MFMA busy fraction =
SQ_VALU_MFMA_BUSY_CYCLES / (128 * GRBM_GUI_ACTIVE); FETCH_SIZE is in KiB.

usage: python bench/pmc_summary.py OUT_DIR name_substr [name_substr ...]"""
import csv
import glob
import json
import os
import statistics
import sys
from collections import defaultdict


def main():
    out_dir, keys = sys.argv[1], sys.argv[2:]
    per = defaultdict(lambda: defaultdict(list))  # kernel -> counter -> values (one per dispatch)
    dur = defaultdict(list)
    for f in sorted(glob.glob(os.path.join(out_dir, "p*", "**", "*counter_collection.csv"), recursive=True)):
        seen = set()
        for r in csv.DictReader(open(f)):
            name = r["Kernel_Name"]
            k = next((k for k in keys if k in name), None)
            if k is None:
                continue
            per[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
            d = (r["Dispatch_Id"], f)
            if d not in seen:
                seen.add(d)
                dur[k].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6)
    res = {}
    for k, cs in per.items():
        m = {c: statistics.median(v) for c, v in cs.items()}
        ms = statistics.median(dur[k])
        d = {"dispatches": len(dur[k]), "kernel_ms_median_profiled": round(ms, 4),
             "counters_median": {c: round(v, 1) for c, v in sorted(m.items())}}
        gui = m.get("GRBM_GUI_ACTIVE")
        if gui:
            d["effective_clock_ghz"] = round(gui / 8 / (ms * 1e6), 3)
            if "SQ_VALU_MFMA_BUSY_CYCLES" in m:
                d["mfma_busy_frac"] = round(m["SQ_VALU_MFMA_BUSY_CYCLES"] / (128 * gui), 4)
        if m.get("SQ_LDS_IDX_ACTIVE"):
            d["lds_bank_conflict_frac"] = round(m.get("SQ_LDS_BANK_CONFLICT", 0.0) / m["SQ_LDS_IDX_ACTIVE"], 4)
        if m.get("SQ_WAVE_CYCLES"):
            d["wait_frac"] = round(m.get("SQ_WAIT_ANY", 0.0) / m["SQ_WAVE_CYCLES"], 4)
            d["wait_inst_frac"] = round(m.get("SQ_WAIT_INST_ANY", 0.0) / m["SQ_WAVE_CYCLES"], 4)
        if "FETCH_SIZE" in m:
            d["hbm_fetch_gb"] = round(m["FETCH_SIZE"] * 1024 / 1e9, 3)
            d["hbm_fetch_gbps_profiled"] = round(m["FETCH_SIZE"] * 1024 / 1e9 / (ms / 1e3), 1)
        res[k] = d
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
