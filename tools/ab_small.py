"""A/B of the L <= 64 M-step on BASELINE cfg 5's largest grid point (T_d = 120, the 20 SNR points
batched: 1280 trials): sbce_mstep time of the one-workgroup kernel (full, build only, build +
factorisation: SBCE_SMALL_STOP, the round-5 kernel's VALU build) vs the round-5 kernel
(SBCE_MSTEP_SMALL=1) and the batched path (SBCE_MSTEP_SMALL=0), HIP events.

  python tools/ab_small.py [T_d] [reps]
"""
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
    reps = int(sys.argv[2]) if len(sys.argv) > 2 else 20
    snr = np.arange(-5, 35, 2.0)
    varn = pkg.signal_model.snr_to_varn(snr, 42.0)
    pts = [pkg.signal_model.synthetic_batch(64, 2, 2, 15, 20, td, 64, float(v), seed=7 + j,
                                            pinv="scipy") for j, v in enumerate(varn)]
    batch = {k: np.concatenate([p[k] for p in pts]) for k in ("y_d", "y_p", "psi_d", "u_p", "theta0", "h")}
    batch["cons"] = pts[0]["cons"]
    vt = np.repeat(varn, 64)
    for arm, env in (("small", {}), ("small_v1", {"SBCE_MSTEP_SMALL": "1"}),
                     ("small_build", {"SBCE_SMALL_STOP": "1"}), ("small_col", {"SBCE_SMALL_SOLVE": "col"}),
                     ("batched", {"SBCE_MSTEP_SMALL": "0"})):
        with pkg._lib.debug_env(**env):
            eng = pkg.EMEngine(batch, vt, mode="soft")
            eng.estep()
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            eng.mstep()
            e0.record()
            for _ in range(reps):
                eng.mstep()
            e1.record()
            torch.cuda.synchronize()
            print(f"{arm:14s} T_d={td} B={eng.B}: {e0.elapsed_time(e1) / reps * 1e3:8.1f} us per M-step",
                  flush=True)


if __name__ == "__main__":
    main()
