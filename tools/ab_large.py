#!/usr/bin/env python3
"""A/B of large-L M-step variants (SBCE_* switches) at BASELINE cfg 2 geometry: the min-norm
M-step from fixed PM_beta moments, HIP events on the launch stream, same process.
  python tools/ab_large.py --trials 256 ENV=VAL[,ENV=VAL] ...   (arm 'default' = no switch)"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--trials", type=int, default=256)
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("arms", nargs="*", default=["default", "SBCE_HERK_TILE=128"])
    a = ap.parse_args()
    import numpy as np
    import torch
    import __graft_entry__ as ge
    pkg = ge.package()
    pkg._lib.use_ab()       # the A/B build: SBCE_* switches, counters, clocks
    varn = float(pkg.signal_model.snr_to_varn(20.0))
    b = pkg.signal_model.synthetic_batch(a.trials, 8, 8, 256, 32, 1024, 16, varn, seed=0)
    eng = pkg.EMEngine(b, varn, mode="pm_soft", partition_r=1, solve="lstsq")
    del b
    eng.run(1)
    eng.estep()
    torch.cuda.synchronize()
    res = {}
    for rep in range(2):
        for arm in a.arms:
            env = {} if arm == "default" else dict(kv.split("=") for kv in arm.split(","))
            with pkg._lib.debug_env(**env):
                eng.mstep()
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                for _ in range(a.reps):
                    eng.mstep()
                e1.record()
                torch.cuda.synchronize()
                ms = e0.elapsed_time(e1) / a.reps
                th = eng.theta.cpu().numpy()
            res.setdefault(arm, []).append(ms)
            print(json.dumps({"arm": arm, "mstep_ms": ms, "theta_abs_sum": float(np.abs(th).sum())}),
                  flush=True)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
