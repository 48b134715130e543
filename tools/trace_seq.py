#!/usr/bin/env python3
"""Diagnostic: the dispatch sequence of a rocprofv3 --kernel-trace run (rocpd SQLite), one
line per launch whose name contains one of the given substrings: start offset, duration and
grid, so per-launch costs (e.g. per Cholesky panel) can be read off a run.

  python tools/trace_seq.py <trace dir> panel_ backsub [--last N]
"""
import glob
import os
import re
import sqlite3
import sys


def short(name):
    name = re.sub(r"\(.*$", "", name)
    name = re.sub(r"^.*::", "", name)
    return name


def main():
    d = sys.argv[1]
    args = sys.argv[2:]
    last = None
    if "--last" in args:
        i = args.index("--last")
        last = int(args[i + 1])
        args = args[:i] + args[i + 2:]
    pats = args or [""]
    for f in glob.glob(os.path.join(d, "**", "*.db"), recursive=True):
        con = sqlite3.connect(f)
        cols = [c[1] for c in con.execute("pragma table_info(kernels)").fetchall()]
        grid = [c for c in ("grid_x", "grid_size_x", "grid_size") if c in cols]
        sel = "name, start, duration" + (f", {grid[0]}" if grid else "")
        rows = con.execute(f"select {sel} from kernels order by start").fetchall()
        rows = [r for r in rows if any(p in r[0] for p in pats)]
        if last:
            rows = rows[-last:]
        t0 = rows[0][1] if rows else 0
        for r in rows:
            g = f" grid {r[3]}" if len(r) > 3 else ""
            print(f"{(r[1] - t0) / 1e3:12.1f} us  {r[2] / 1e3:9.1f} us  {short(r[0])}{g}")


if __name__ == "__main__":
    main()
