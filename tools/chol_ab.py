#!/usr/bin/env python3
"""A/B of the L <= 512 Cholesky schedules on the bench workload (cfg1, 1000 trials): the M-step
alone (sbce_mstep from fixed moments, HIP events on the launch stream) and the whole bench step,
per SBCE_CHOL_IMPL arm, same process.
  python tools/chol_ab.py [arm ...]      arms: default (wide schedule) n (one update per panel)
                                          l (look-ahead)
"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    arms = sys.argv[1:] or ["default", "n"]
    import numpy as np
    import torch
    import __graft_entry__ as ge
    pkg = ge.package()
    pkg._lib.use_ab()       # the A/B build: SBCE_* switches, counters, clocks
    varn = float(pkg.signal_model.snr_to_varn(20.0))
    b = pkg.signal_model.synthetic_batch(1000, 4, 4, 64, 16, 256, 16, varn, seed=0)
    res = {}
    for rep in range(2):
        for arm in arms:
            env = {} if arm == "default" else {"SBCE_CHOL_IMPL": arm}
            with pkg._lib.debug_env(**env):
                eng = pkg.EMEngine(b, varn, streams=1)
                eng.run(3)                             # theta past iteration 0
                torch.cuda.synchronize()
                eng.estep()
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                eng.mstep()
                e0.record()
                for _ in range(10):
                    eng.mstep()
                e1.record()
                torch.cuda.synchronize()
                ms = e0.elapsed_time(e1) / 10
                for streams in (1, 3):
                    eng = pkg.EMEngine(b, varn, streams=streams)
                    eng.run(20)
                    torch.cuda.synchronize()
                    t0 = time.perf_counter()
                    for _ in range(3):
                        eng.run(20)
                    torch.cuda.synchronize()
                    dt = (time.perf_counter() - t0) / 3
                    res.setdefault(f"{arm}_s{streams}", []).append(1000 * 20 / dt)
                res.setdefault(f"{arm}_mstep_ms", []).append(ms)
                th = eng.theta.cpu().numpy()
                res.setdefault(f"{arm}_theta_sum", []).append(float(np.abs(th).sum()))
            print(json.dumps({k: v[-1] for k, v in res.items() if k.startswith(arm)}), flush=True)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
