"""Driver of the issued-work PMC passes (tools/sq_issued.sh): the E-step launches bench.py's
rooflines time, run alone after the work that sets their regime.

  cfg1: BASELINE configs[1] (1000 trials, 20 dB), a 20-iteration EM, then REPS steady-state E-steps
  cfg5: BASELINE configs[4]'s largest grid point (T_d = 120, the 20 SNR points batched: 1280
        trials), the exact soft E-step at theta = h (bench.py grid_roofline), REPS times

  python tools/sq_drive.py cfg1|cfg5 [REPS]
"""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import __graft_entry__ as ge  # noqa: E402

pkg = ge.package()


def main():
    mode = sys.argv[1]
    reps = int(sys.argv[2]) if len(sys.argv) > 2 else 3
    if mode == "cfg1":
        varn = float(pkg.signal_model.snr_to_varn(20.0))
        batch = pkg.signal_model.synthetic_batch(1000, 4, 4, 64, 16, 256, 16, varn, seed=0)
        eng = pkg.EMEngine(batch, varn)
        eng.run(20)
    else:
        snr = np.arange(-5, 35, 2.0)
        varns = pkg.signal_model.snr_to_varn(snr, 42.0)
        pts = [pkg.signal_model.synthetic_batch(64, 2, 2, 15, 20, 120, 64, float(v), pinv="scipy",
                                                seed=j) for j, v in enumerate(varns)]
        batch = {k: np.concatenate([p[k] for p in pts])
                 for k in ("y_d", "y_p", "psi_d", "u_p", "theta0", "h")}
        batch["cons"] = pts[0]["cons"]
        eng = pkg.EMEngine(batch, np.repeat(varns, 64), mode="soft", solve="chol", early_stop=True)
        eng.theta.copy_(eng.h)
    torch.cuda.synchronize()
    for _ in range(reps):
        eng.estep()
    torch.cuda.synchronize()
    print("ok", mode, eng.B)


if __name__ == "__main__":
    main()
