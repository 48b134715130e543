"""Diagnostic A/B: cfg1 M-step time under alternating environment settings in ONE process
(same box, same clock), e.g.  python tools/ab_mstep.py SBCE_RHS_IMPL=row SBCE_RHS_IMPL=slice"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402
import __graft_entry__ as ge  # noqa: E402

pkg = ge.package()
pkg._lib.use_ab()       # the A/B build: SBCE_* switches, counters, clocks
varn = float(pkg.signal_model.snr_to_varn(20.0))
batch = pkg.signal_model.synthetic_batch(1000, 4, 4, 64, 16, 256, 16, varn, seed=0)
eng = pkg.EMEngine(batch, varn)
eng.run(2)
eng.estep()
torch.cuda.synchronize()


def timeit(fn, reps=10):
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps


for rnd in range(3):
    for arm in sys.argv[1:]:
        k, v = arm.split("=", 1)
        os.environ[k] = v
        pkg._lib.reload_debug_env()   # the library reads SBCE_* switches once
        print(f"round {rnd} {arm:28s} mstep {timeit(eng.mstep):.4f} ms  estep {timeit(eng.estep):.4f} ms",
              flush=True)
        del os.environ[k]
        pkg._lib.reload_debug_env()   # the library reads SBCE_* switches once
