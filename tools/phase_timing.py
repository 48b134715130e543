"""Diagnostic: time the M-step Cholesky with phases disabled (sbce_debug_chol_skip bitmask,
results invalid) and the E-step per SNR, on cfg1 shapes.  Not part of the product."""
import os
import sys
import time

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


for impl in ("mfma", "valu"):
    os.environ["SBCE_CHOL_IMPL"] = impl
    pkg._lib.reload_debug_env()   # the library reads SBCE_* switches once
    for skip in (0, 1, 2, 8, 16, 1 | 2 | 8 | 16):
        LIB.sbce_debug_chol_skip(skip)
        print(f"chol {impl} skip={skip:2d}: mstep {timeit(eng.mstep):.3f} ms", flush=True)
LIB.sbce_debug_chol_skip(0)
os.environ["SBCE_CHOL_IMPL"] = "mfma"
pkg._lib.reload_debug_env()   # the library reads SBCE_* switches once

# per-phase s_memtime sums (block 0, waves 0/1) of one MFMA Cholesky launch
import ctypes  # noqa: E402
lib = pkg._lib.load()
buf = (ctypes.c_ulonglong * 32)()
lib.sbce_debug_chol_clock(buf, 1)
LIB.sbce_debug_chol_skip(64)
eng.mstep()
torch.cuda.synchronize()
LIB.sbce_debug_chol_skip(0)
lib.sbce_debug_chol_clock(buf, 0)
names = ["C init+update", "diag factor", "barrier after diag", "trsm tiles", "end barrier",
         "back substitution"]
for wv in range(2):
    tot = sum(buf[wv * 8 + i] for i in range(6))
    print(f"wave {wv}: " + ", ".join(f"{n} {buf[wv * 8 + i]}" for i, n in enumerate(names)) +
          f"  total {tot} cycles", flush=True)
print(f"wave 0 diag detail: column loop {buf[6]} (reads+pivot {buf[15]}, writes {buf[16]}), "
      f"inverse {buf[7]}, R writes {buf[14]}", flush=True)
