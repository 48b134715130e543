#!/usr/bin/env python3
"""Issued FP64 work per launch from one rocprofv3 --pmc pass (rocpd SQLite) of tools/sq_drive.py:
for every sbce kernel the LAST `reps` dispatches (the driver's steady-state E-steps) are averaged,
and the phase's issued FP64 flops per E-step are
    64 lanes x (2 FMA_F64 + MUL_F64 + ADD_F64 + TRANS_F64)  +  512 x MFMA_MOPS_F64
(VALU counts are per wave-instruction, all lanes counted; MFMA_MOPS are in units of 512 flop).

  python tools/sq_issued.py <pmc_dir> --config cfg1 --trials 1000 --reps 3 --out sq.json
"""
import argparse
import collections
import glob
import json
import os
import sqlite3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("pmc_dir")
    ap.add_argument("--config", required=True)
    ap.add_argument("--trials", type=int, required=True)
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--out", required=True)
    a = ap.parse_args()
    rows = collections.defaultdict(lambda: collections.defaultdict(float))
    for f in glob.glob(os.path.join(a.pmc_dir, "**", "*.db"), recursive=True):
        con = sqlite3.connect(f)
        cols = [r[1] for r in con.execute("pragma table_info(counters_collection)")]
        did = next((c for c in ("dispatch_id", "correlation_id", "dispatch") if c in cols), None)
        if did:
            q = ("select kernel_name, counter_name, %s, sum(value) from counters_collection "
                 "group by kernel_name, counter_name, %s" % (did, did))
            for k, c, d, v in con.execute(q):
                rows[(k, d)][c] += v
        else:                          # no dispatch column: the i-th row of (kernel, counter)
            seen = collections.Counter()
            for k, c, v in con.execute("select kernel_name, counter_name, value from "
                                       "counters_collection order by rowid"):
                d = seen[(k, c)]
                seen[(k, c)] += 1
                rows[(k, d)][c] += v
    per = collections.defaultdict(list)                  # kernel -> [(dispatch, counters)]
    for (k, d), cv in rows.items():
        if "sbce" in k:
            per[k].append((d, cv))
    out = {}
    total = 0.0
    for k, lst in per.items():
        lst.sort(key=lambda t: t[0])
        last = [cv for _, cv in lst[-a.reps:]]
        avg = {c: sum(cv.get(c, 0.0) for cv in last) / len(last) for c in last[0]}
        valu = 64.0 * (2 * avg.get("SQ_INSTS_VALU_FMA_F64", 0) + avg.get("SQ_INSTS_VALU_MUL_F64", 0) +
                       avg.get("SQ_INSTS_VALU_ADD_F64", 0) + avg.get("SQ_INSTS_VALU_TRANS_F64", 0))
        mfma = 512.0 * avg.get("SQ_INSTS_VALU_MFMA_MOPS_F64", 0)
        name = k.replace("sbce::(anonymous namespace)::", "").replace("void ", "").split("(")[0]
        out[name] = {"dispatches": len(lst), "fp64_valu_flops": valu, "fp64_mfma_flops": mfma,
                     "counters": avg}
        if name.startswith("estep_"):                 # the E-step phase's kernels only
            total += valu + mfma
    res = {"config": a.config, "trials": a.trials, "reps": a.reps,
           "issued_fp64_flops_per_estep": total, "kernels": out,
           "formula": "64 x (2 FMA_F64 + MUL_F64 + ADD_F64 + TRANS_F64) + 512 x MFMA_MOPS_F64, "
                      "averaged over the last reps dispatches of each kernel, summed over the "
                      "estep_* kernels (every lane of an issued VALU instruction counted; the sweep's "
                      "FP32 screen MFMAs are not FP64 work and are not counted)"}
    json.dump(res, open(a.out, "w"), indent=1)
    print(json.dumps({k: (v["fp64_valu_flops"], v["fp64_mfma_flops"]) for k, v in out.items()}, indent=1))
    print("issued FP64 flops per E-step:", total)


if __name__ == "__main__":
    main()
