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
    # one row per (kernel, grid size): a kernel launched at several sizes (bench.py's stream
    # sub-batches beside its whole-batch timing launches) keeps its per-size average
    w.writerow(["Name", "Calls", "TotalDurationNs", "AverageNs", "Percentage", "Grid"])
    for f in dbs:
        con = sqlite3.connect(f)
        cols = [c[1] for c in con.execute("pragma table_info(kernels)").fetchall()]
        grid = next((c for c in ("grid_size", "grid_x", "grid_size_x") if c in cols), None)
        g = grid or "0"
        rows = con.execute(f"select name, count(*), sum(duration), avg(duration), {g} from kernels "
                           f"group by name, {g} order by sum(duration) desc").fetchall()
        total = sum(r[2] for r in rows) or 1
        for name, calls, tot, avg, gs in rows:
            w.writerow([name, calls, f"{tot:.0f}", f"{avg:.1f}", f"{100.0 * tot / total:.2f}", gs])


if __name__ == "__main__":
    main()
