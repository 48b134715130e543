#!/usr/bin/env python3
"""Per-call durations (µs) of the kernels matching a substring in a rocprofv3 kernel trace
(rocpd SQLite), in launch order: the per-iteration view the --stats summary averages away.

  python tools/trace_calls.py gpurun_out/<tag>/trace estep_ [last_n]
"""
import glob
import os
import re
import sqlite3
import sys


def main():
    d, pat = sys.argv[1], sys.argv[2]
    last = int(sys.argv[3]) if len(sys.argv) > 3 else 0
    for f in glob.glob(os.path.join(d, "**", "*.db"), recursive=True):
        con = sqlite3.connect(f)
        rows = con.execute("select name, start, duration from kernels order by start").fetchall()
        rows = [r for r in rows if pat in r[0]]
        for name, start, dur in rows[-last:] if last else rows:
            m = re.search(r"(\w+_kernel\w*)", name)
            print(f"{start:>20d} {dur / 1e3:10.1f}  {m.group(1) if m else name[:70]}")


if __name__ == "__main__":
    main()
