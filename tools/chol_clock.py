"""Diagnostic: per-phase cycle sums of the batched panel factor launches for trial 0 of the cfg1
batch (sbce_debug_chol_skip bit 64 -> g_chol_clk[16..31], waves 0 and 1; results unchanged),
summed over the 9 factor launches of one M-step; B trials (env B, default 1000)."""
import ctypes
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
eng.mstep()
torch.cuda.synchronize()
out = (ctypes.c_ulonglong * 32)()
names = ["start/PRE", "wave0 loads", "factor A", "tile-1 TRSM", "sync 1", "B chain | TRSM A",
         "sync 2", "TRSM B"]
reps = int(os.environ.get("REPS", "5"))
LIB.sbce_debug_chol_skip(64)
LIB.sbce_debug_chol_clock(None, 1)
for _ in range(reps):
    eng.mstep()
torch.cuda.synchronize()
LIB.sbce_debug_chol_clock(out, 0)
LIB.sbce_debug_chol_skip(0)
print(f"B={B}: cycles per M-step (9 factor launches), trial 0")
for ph, nm in enumerate(names):
    w0, w1 = out[16 + ph] / reps, out[24 + ph] / reps
    print(f"  {ph} {nm:18s} wave0 {w0:9.0f}  wave1 {w1:9.0f}")
print(f"  total              wave0 {sum(out[16:24]) / reps:9.0f}  wave1 {sum(out[24:32]) / reps:9.0f}")
