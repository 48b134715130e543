#!/usr/bin/env python3
"""Export the per-kernel summary of a rocprofv3 --kernel-trace --stats run (rocpd
SQLite output) as CSV: name, calls, total_ns, average_ns, percentage.

  python tools/trace_summary.py gpurun_out/<tag>/trace > profiles/<round>/kernel_stats.csv
"""
import csv
import glob
import os
import sqlite3
import sys


def main():
    d = sys.argv[1]
    dbs = glob.glob(os.path.join(d, "**", "*.db"), recursive=True)
    if not dbs:
        raise SystemExit(f"no rocpd database under {d}")
    w = csv.writer(sys.stdout)
    w.writerow(["Name", "Calls", "TotalDurationNs", "AverageNs", "Percentage"])
    for f in dbs:
        con = sqlite3.connect(f)
        rows = con.execute("select name, count(*), sum(duration), avg(duration) from kernels "
                           "group by name order by sum(duration) desc").fetchall()
        total = sum(r[2] for r in rows) or 1
        for name, calls, tot, avg in rows:
            w.writerow([name, calls, f"{tot:.0f}", f"{avg:.1f}", f"{100.0 * tot / total:.2f}"])


if __name__ == "__main__":
    main()
