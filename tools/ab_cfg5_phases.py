"""Standalone phase times at BASELINE cfg 5's largest grid point (T_d = 120, the 20 SNR points
batched: 1280 trials, theta after one EM iteration): each detector's E-step (sbce_estep) and the
M-step, HIP events on the current stream; optional env arms ("NAME=VAL,..." per argument).

  python tools/ab_cfg5_phases.py [T_d] [arm ...]      e.g.  SBCE_PM_IMPL=wave
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


def timed(fn, reps=10):
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps * 1e3


def main():
    td = int(sys.argv[1]) if len(sys.argv) > 1 else 120
    arms = [("default", {})] + [(a, dict(kv.split("=") for kv in a.split(","))) for a in sys.argv[2:]
                                if a != "count"]
    snr = np.arange(-5, 35, 2.0)
    varn = pkg.signal_model.snr_to_varn(snr, 42.0)
    pts = [pkg.signal_model.synthetic_batch(64, 2, 2, 15, 20, td, 64, float(v), seed=7 + j,
                                            pinv="scipy") for j, v in enumerate(varn)]
    batch = {k: np.concatenate([p[k] for p in pts]) for k in ("y_d", "y_p", "psi_d", "u_p", "theta0", "h")}
    batch["cons"] = pts[0]["cons"]
    vt = np.repeat(varn, 64)
    count = "count" in sys.argv
    if count:
        arms = [(n, e) for n, e in arms if n != "count"]
    for name, env in arms:
        with pkg._lib.debug_env(**env):
            out = []
            for det in ("pm_soft", "hard", "zf", "mmse", "soft"):
                eng = pkg.EMEngine(batch, vt, mode=det, partition_r=1 if det == "pm_soft" else 0)
                eng.run(1)
                out.append(f"{det} {timed(eng.estep):7.1f}")
            out.append(f"mstep {timed(eng.mstep):7.1f}")
            print(f"{name:24s} T_d={td} B={eng.B} us: " + "  ".join(out), flush=True)
    if count:                      # where the exact soft E-step's symbols were resolved, per SNR
        import ctypes
        lib = pkg._lib.load()
        eng = pkg.EMEngine(batch, vt, mode="soft")
        eng.run(1)
        sph = (ctypes.c_ulonglong * 3)()
        npair, nmf = ctypes.c_ulonglong(0), ctypes.c_ulonglong(0)
        with pkg._lib.debug_env(SBCE_ESTEP_COUNT="1"):
            lib.sbce_debug_estep_sphere(None, 1)
            lib.sbce_debug_estep_pair(None, 1)
            lib.sbce_debug_estep_mfma(None, 1)
            eng.estep()
            torch.cuda.synchronize()
            lib.sbce_debug_estep_sphere(sph, 0)
            lib.sbce_debug_estep_pair(ctypes.byref(npair), 0)
            lib.sbce_debug_estep_mfma(ctypes.byref(nmf), 0)
        nsym = float(eng.B * td)
        print(f"soft E-step symbols: single path {sph[2] / nsym:.3f}, enumerated {sph[0] / nsym:.3f}, "
              f"factorised {npair.value / nsym:.3f}, swept {(sph[1] - npair.value) / nsym:.3f}; "
              f"sweep MFMAs {nmf.value} ({nmf.value / max(sph[1] - npair.value, 1):.0f} per swept symbol)",
              flush=True)


if __name__ == "__main__":
    main()
