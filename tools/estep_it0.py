"""Diagnostic driver: E-step launches at theta_0 (iteration 0) on the cfg1 batch, for kernel
traces of the iteration-0 sweep (env SNR, REPS; SBCE_* switches apply)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402
import __graft_entry__ as ge  # noqa: E402

pkg = ge.package()
pkg._lib.use_ab()       # the A/B build: SBCE_* switches, counters, clocks
varn = float(pkg.signal_model.snr_to_varn(float(os.environ.get("SNR", "20"))))
batch = pkg.signal_model.synthetic_batch(1000, 4, 4, 64, 16, 256, 16, varn, seed=0)
eng = pkg.EMEngine(batch, varn)
for _ in range(int(os.environ.get("REPS", "3"))):
    eng.estep()
torch.cuda.synchronize()
print("ok")
