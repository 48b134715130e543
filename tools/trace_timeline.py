#!/usr/bin/env python3
"""GPU busy time of a rocprofv3 --kernel-trace run (rocpd SQLite output): the span from the
first kernel start to the last kernel end, the union of all kernel intervals (time the GPU ran
at least one kernel), per-stream busy time, and the idle gaps -- whether a multi-stream run is
bound by the kernels or by the host's launch rate.

  python tools/trace_timeline.py gpurun_out/<tag>/trace [--last-frac 0.5]
"""
import glob
import os
import sqlite3
import sys


def main():
    d = sys.argv[1]
    frac = float(sys.argv[sys.argv.index("--last-frac") + 1]) if "--last-frac" in sys.argv else 1.0
    dbs = glob.glob(os.path.join(d, "**", "*.db"), recursive=True)
    if not dbs:
        raise SystemExit(f"no rocpd database under {d}")
    con = sqlite3.connect(dbs[0])
    cols = [c[1] for c in con.execute("pragma table_info(kernels)").fetchall()]
    print("columns:", cols)
    sc = next((c for c in ("stream_id", "stream", "queue_id", "queue") if c in cols), None)
    rows = con.execute(f"select start, end, {sc or 0}, name from kernels order by start").fetchall()
    t0, t1 = rows[0][0], max(r[1] for r in rows)
    cut = t1 - (t1 - t0) * frac                       # the last `frac` of the run (timed steps)
    rows = [r for r in rows if r[0] >= cut]
    t0 = rows[0][0]
    span = t1 - t0
    busy, cur_s, cur_e = 0, None, None
    gaps = []
    for s, e, _, _ in rows:
        if cur_e is None or s > cur_e:
            if cur_e is not None:
                busy += cur_e - cur_s
                gaps.append(s - cur_e)
            cur_s, cur_e = s, e
        else:
            cur_e = max(cur_e, e)
    busy += cur_e - cur_s
    per = {}
    for s, e, q, _ in rows:
        per[q] = per.get(q, 0) + (e - s)
    ksum = sum(r[1] - r[0] for r in rows)
    print(f"kernels {len(rows)}  span {span / 1e6:.2f} ms  union busy {busy / 1e6:.2f} ms "
          f"({100 * busy / span:.1f}%)  sum of kernel time {ksum / 1e6:.2f} ms "
          f"(mean concurrency while busy {ksum / max(busy, 1):.2f})")
    for q, t in sorted(per.items(), key=lambda x: -x[1]):
        print(f"  stream {q}: {t / 1e6:.2f} ms")
    # segments separated by idle gaps > 2 ms (the bench's steps vs its setup / timing phases)
    seg, segs = [rows[0]], []
    cur_e = rows[0][1]
    for r in rows[1:]:
        if r[0] - cur_e > 2e6:
            segs.append(seg)
            seg = []
        seg.append(r)
        cur_e = max(cur_e, r[1])
    segs.append(seg)
    for sg in segs:
        a0, a1 = sg[0][0], max(r[1] for r in sg)
        ks = sum(r[1] - r[0] for r in sg)
        ub, cs, ce = 0, None, None
        for s_, e_, _, _ in sg:
            if ce is None or s_ > ce:
                if ce is not None:
                    ub += ce - cs
                cs, ce = s_, e_
            else:
                ce = max(ce, e_)
        ub += ce - cs
        qs = len(set(r[2] for r in sg))
        print(f"  segment {(a0 - t0) / 1e6:9.2f} ms +{(a1 - a0) / 1e6:8.2f} ms: {len(sg):5d} kernels on {qs} "
              f"streams, busy {100 * ub / max(a1 - a0, 1):5.1f}%, concurrency {ks / max(ub, 1):.2f}")
    if "--dump" in sys.argv:                     # N kernels from the middle of the longest segment
        n = int(sys.argv[sys.argv.index("--dump") + 1])
        sg = max(segs, key=lambda x: max(r[1] for r in x) - x[0][0])
        mid = len(sg) // 2
        w = sg[max(0, mid - n // 2): mid + n // 2]
        base = w[0][0]
        for s_, e_, q, nm in w:
            short = nm.replace("(anonymous namespace)::", "").replace("void sbce::", "")[:48]
            print(f"    {(s_ - base) / 1e3:9.1f} {(e_ - base) / 1e3:9.1f} us  q{q}  {short}")
    gaps.sort()
    if gaps:
        tot = sum(gaps)
        print(f"idle gaps {len(gaps)}: total {tot / 1e6:.2f} ms, median {gaps[len(gaps) // 2] / 1e3:.1f} us, "
              f"max {gaps[-1] / 1e3:.1f} us")


if __name__ == "__main__":
    main()
