#!/usr/bin/env python3
"""Summarise two rocprofv3 PMC passes (FETCH_SIZE, WRITE_SIZE) into per-launch HBM
bytes per kernel (bench.py sums the kernels of the roofline phase into roofline.traffic).

  python tools/pmc_summary.py --fetch gpurun_out/pmc_fetch --write gpurun_out/pmc_write \
      --config cfg1 --trials 1000 --out profiles/pmc_cfg1_latest.json

Corrections (MI355X_MICROARCH.md, "HBM [CDNA4]"): rocprofv3 reports FETCH_SIZE and
WRITE_SIZE in KiB; on gfx950 FETCH_SIZE counts wide coalesced reads at half their
bytes, so it is doubled; WRITE_SIZE is taken as is.  Infinity-Cache hits are not
excluded by these counters.
"""
import argparse
import csv
import glob
import json
import os
from collections import defaultdict


def _read(d, counter):
    """Per-kernel counter values from a rocprofv3 output dir (CSV or rocpd SQLite)."""
    per = defaultdict(list)
    dbs = glob.glob(os.path.join(d, "**", "*.db"), recursive=True)
    if dbs:
        import sqlite3
        for f in dbs:
            con = sqlite3.connect(f)
            for name, val in con.execute(
                    "select kernel_name, value from counters_collection where counter_name = ?",
                    (counter,)):
                per[name].append(float(val))
        return per
    files = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)
    if not files:
        raise SystemExit(f"no counter output under {d}")
    for f in files:
        with open(f) as fh:
            for row in csv.DictReader(fh):
                if row.get("Counter_Name") != counter:
                    continue
                per[row["Kernel_Name"]].append(float(row["Counter_Value"]))
    return per


def _short(name):
    """Kernel identifier: last scope component before the template / argument list."""
    base = name.replace("(anonymous namespace)", "")
    base = base.split("(")[0].split("<")[0]
    return base.replace("void ", "").split("::")[-1].strip()[:60]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--fetch", required=True)
    ap.add_argument("--write", required=True)
    ap.add_argument("--config", default="cfg1")
    ap.add_argument("--trials", type=int, default=1000)
    ap.add_argument("--out", required=True)
    a = ap.parse_args()
    fetch, write = _read(a.fetch, "FETCH_SIZE"), _read(a.write, "WRITE_SIZE")
    kernels = {}
    for name in sorted(set(fetch) | set(write)):
        f, w = fetch.get(name, []), write.get(name, [])
        k = _short(name)          # template instantiations of one kernel are summed
        ent = kernels.setdefault(k, {"launches_fetch": 0, "launches_write": 0,
                                     "fetch_bytes_total": 0.0, "write_bytes_total": 0.0})
        ent["launches_fetch"] += len(f)
        ent["fetch_bytes_total"] += 2.0 * 1024.0 * sum(f)
        ent["launches_write"] += len(w)
        ent["write_bytes_total"] += 1024.0 * sum(w)
    for ent in kernels.values():
        fb = ent["fetch_bytes_total"] / ent["launches_fetch"] if ent["launches_fetch"] else 0.0
        wb = ent["write_bytes_total"] / ent["launches_write"] if ent["launches_write"] else 0.0
        ent["fetch_bytes_per_launch"], ent["write_bytes_per_launch"] = fb, wb
        ent["hbm_bytes_per_launch"] = fb + wb
    out = {"config": a.config, "trials": a.trials,
           "source": "rocprofv3 --pmc FETCH_SIZE / --pmc WRITE_SIZE, separate passes; "
                     "FETCH_SIZE x2 (gfx950), KiB -> bytes",
           "kernels": kernels}
    with open(a.out, "w") as fh:
        json.dump(out, fh, indent=1)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
