"""Diagnostic: M-step time at cfg1 with Cholesky phases disabled (sbce_debug_chol_skip bitmask,
results invalid: 1 panel update, 2 diagonal factor, 8 TRSM tiles, 16 back substitution).
Not part of the product."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402
import __graft_entry__ as ge  # noqa: E402

pkg = ge.package()
pkg._lib.use_ab()       # the A/B build: SBCE_* switches, counters, clocks
LIB = pkg._lib.load()
B = int(os.environ.get("B", "1000"))
varn = float(pkg.signal_model.snr_to_varn(20.0))
batch = pkg.signal_model.synthetic_batch(B, 4, 4, 64, 16, 256, 16, varn, seed=0)
eng = pkg.EMEngine(batch, varn)
eng.run(2)
eng.estep()
torch.cuda.synchronize()


def timeit(fn, reps=5):
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps


for impl in sys.argv[1:] or ["batched"]:
    os.environ["SBCE_CHOL_IMPL"] = impl
    pkg._lib.reload_debug_env()   # the library reads SBCE_* switches once
    for skip in (0, 1, 2, 8, 16, 2 | 8, 1 | 2 | 8 | 16):
        LIB.sbce_debug_chol_skip(skip)
        print(f"chol {impl} skip={skip:2d}: mstep {timeit(eng.mstep):.3f} ms", flush=True)
LIB.sbce_debug_chol_skip(0)
