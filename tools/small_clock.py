"""Diagnostic: s_memtime stamps of trial 0's solve wave in the n_tx <= 2 small M-step
(SBCE_SMALL_STOP=4, results unchanged) at BASELINE cfg 5's T_d point (the 20 SNR points batched:
1280 trials).  Prints the build, tol, per-column-pair and back-substitution intervals in cycles.

  python tools/small_clock.py [T_d]
"""
import ctypes
import importlib
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
pkg = importlib.import_module(
    "semi-blind-channel-estimation-for-mimo-ris-communication-system-using-em-algo_amd")
pkg._lib.use_ab()       # the A/B build: SBCE_* switches, counters, clocks


def main():
    td = int(sys.argv[1]) if len(sys.argv) > 1 else 120
    snr = np.arange(-5, 35, 2.0)
    varn = pkg.signal_model.snr_to_varn(snr, 42.0)
    pts = [pkg.signal_model.synthetic_batch(64, 2, 2, 15, 20, td, 64, float(v), seed=7 + j,
                                            pinv="scipy") for j, v in enumerate(varn)]
    batch = {k: np.concatenate([p[k] for p in pts]) for k in ("y_d", "y_p", "psi_d", "u_p", "theta0", "h")}
    batch["cons"] = pts[0]["cons"]
    lib = pkg._lib.load()
    with pkg._lib.debug_env(SBCE_SMALL_STOP="4"):
        eng = pkg.EMEngine(batch, np.repeat(varn, 64), mode="soft")
        eng.estep()
        for _ in range(3):
            eng.mstep()
            torch.cuda.synchronize()
            out = (ctypes.c_ulonglong * 48)()
            lib.sbce_debug_small_clock(out)
            c = np.array(out[:], dtype=np.int64)
            cols = np.diff(c[2:3 + 16])
            print(f"T_d={td}: start->loads {c[1] - c[0]}  loads->tol {c[2] - c[1]}  "
                  f"pairs {cols.tolist()} (sum {c[18] - c[2]})  factor->back {c[41] - c[40]}  "
                  f"total {c[41] - c[0]}", flush=True)


if __name__ == "__main__":
    main()
