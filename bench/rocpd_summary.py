"""Per-kernel summary of a rocprofv3 SQLite (rocpd) database: calls, total
and average time, and -- with --timeline -- the kernel sequence of a window.
Usage: python bench/rocpd_summary.py <db> [--top N] [--csv out.csv]"""
import argparse
import csv
import sqlite3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("db")
    ap.add_argument("--top", type=int, default=30)
    ap.add_argument("--csv", default="")
    ap.add_argument("--timeline", type=int, default=0, help="print the last N dispatches in order")
    a = ap.parse_args()
    c = sqlite3.connect(a.db)
    rows = c.execute("select s.display_name, count(*), sum(d.end - d.start), min(d.end - d.start), "
                     "max(d.end - d.start) from rocpd_kernel_dispatch d join rocpd_info_kernel_symbol s "
                     "on d.kernel_id = s.id group by s.display_name order by 3 desc").fetchall()
    tot = sum(r[2] for r in rows) or 1
    out = [{"Name": n, "Calls": k, "TotalDurationNs": t, "AverageNs": t / k, "Percentage": 100.0 * t / tot,
            "MinNs": mn, "MaxNs": mx} for n, k, t, mn, mx in rows]
    for r in out[: a.top]:
        print(f"{r['TotalDurationNs'] / 1e6:10.3f} ms {r['Percentage']:5.1f}% calls={r['Calls']:6d} "
              f"avg={r['AverageNs'] / 1e3:9.1f} us  {r['Name'][:100]}")
    if a.csv:
        with open(a.csv, "w", newline="") as f:
            w = csv.DictWriter(f, fieldnames=list(out[0].keys()))
            w.writeheader()
            w.writerows(out)
    if a.timeline:
        seq = c.execute("select s.display_name, d.start, d.end from rocpd_kernel_dispatch d join "
                        "rocpd_info_kernel_symbol s on d.kernel_id = s.id order by d.start desc limit ?",
                        (a.timeline,)).fetchall()[::-1]
        t0 = seq[0][1]
        for n, s, e in seq:
            print(f"{(s - t0) / 1e3:10.1f} us  {(e - s) / 1e3:8.1f} us  {n[:90]}")


if __name__ == "__main__":
    main()
