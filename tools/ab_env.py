"""Diagnostic: same-process A/B of the cfg1 EM (1000 trials x 20 iterations) and its M-step
under alternating environment settings, e.g.  python tools/ab_env.py SBCE_UPD_WAVES=4 SBCE_X=0"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402
import __graft_entry__ as ge  # noqa: E402

pkg = ge.package()
pkg._lib.use_ab()       # the A/B build: SBCE_* switches, counters, clocks
varn = float(pkg.signal_model.snr_to_varn(20.0))
batch = pkg.signal_model.synthetic_batch(1000, 4, 4, 64, 16, 256, 16, varn, seed=0)
eng = pkg.EMEngine(batch, varn)


def timeit(fn, reps):
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps


arms = sys.argv[1:] or ["SBCE_X=0"]
ref = None
for rnd in range(3):
    for arm in arms:
        k, v = arm.split("=", 1)
        os.environ[k] = v
        pkg._lib.reload_debug_env()   # the library reads SBCE_* switches once
        t_em = timeit(lambda: eng.run(20), 2)
        th = eng.theta.cpu().numpy()
        eng.estep()
        t_m = timeit(eng.mstep, 5)
        t_e = timeit(eng.estep, 5)
        del os.environ[k]
        pkg._lib.reload_debug_env()   # the library reads SBCE_* switches once
        if ref is None:
            ref = th
        print(f"round {rnd} {arm:28s} EM {t_em:7.2f} ms ({20000 / t_em * 1e3:9.0f} EM-it/s)  "
              f"M-step {t_m:6.3f} ms  E-step {t_e:6.3f} ms  max|dtheta| {np.abs(th - ref).max():.1e}",
              flush=True)
