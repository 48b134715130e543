#!/usr/bin/env python3
"""Per-kernel averages of the SQ/GRBM counters of one rocprofv3 --pmc pass (rocpd SQLite),
with the derived MFMA-busy and issue/wait fractions.

  python tools/pmc_sq.py gpurun_out/<tag>/pmc_dir
"""
import collections
import glob
import os
import sqlite3
import sys


def main():
    dbs = glob.glob(os.path.join(sys.argv[1], "**", "*.db"), recursive=True)
    d = collections.defaultdict(dict)
    for f in dbs:
        con = sqlite3.connect(f)
        for k, c, v, n in con.execute("select kernel_name, counter_name, sum(value), count(*) "
                                      "from counters_collection group by kernel_name, counter_name"):
            d[k][c] = v / n
    for k, v in sorted(d.items(), key=lambda kv: -kv[1].get("SQ_WAVE_CYCLES", 0)):
        if "sbce" not in k:
            continue
        name = k.replace("sbce::(anonymous namespace)::", "").replace("void ", "").split("(")[0]
        line = [f"{name[:48]:48s}"]
        g = v.get("GRBM_GUI_ACTIVE")
        if g and "SQ_VALU_MFMA_BUSY_CYCLES" in v:
            # MFMA busy per SIMD: the counter sums over all SIMDs of the chip (1024)
            line.append(f"mfma_busy={v['SQ_VALU_MFMA_BUSY_CYCLES'] / (g / 8 * 1024):.3f}")
        wc = v.get("SQ_WAVE_CYCLES")
        if wc:
            for c in ("SQ_ACTIVE_INST_ANY", "SQ_WAIT_INST_ANY", "SQ_WAIT_ANY", "SQ_WAIT_INST_LDS"):
                if c in v:
                    line.append(f"{c[3:].lower()}={v[c] / wc:.3f}")
        for c in sorted(v):                  # instruction counts etc.: per-launch values
            if c.startswith("SQ_INSTS") or c == "SQ_WAVES":
                line.append(f"{c[3:].lower()}={v[c]:.4g}")
        if "SQ_LDS_BANK_CONFLICT" in v:
            line.append(f"lds_conf={v['SQ_LDS_BANK_CONFLICT']:.3g}")
        print("  ".join(line))


if __name__ == "__main__":
    main()
