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
        for name, calls, tot, avg, pct in con.execute(
                "select name, total_calls, total_duration, average, percentage from top_kernels "
                "order by total_duration desc"):
            w.writerow([name, calls, f"{tot:.0f}", f"{avg:.1f}", f"{pct:.2f}"])


if __name__ == "__main__":
    main()
