"""Diagnostic driver: a few E-step launches on the cfg1 batch (for PMC passes)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402
import __graft_entry__ as ge  # noqa: E402

pkg = ge.package()
B = int(os.environ.get("B", "1000"))
varn = float(pkg.signal_model.snr_to_varn(float(os.environ.get("SNR", "20"))))
batch = pkg.signal_model.synthetic_batch(B, 4, 4, 64, 16, 256, 16, varn, seed=0)
eng = pkg.EMEngine(batch, varn)
eng.run(int(os.environ.get("ITERS", "2")))
for _ in range(int(os.environ.get("REPS", "3"))):
    eng.estep()
torch.cuda.synchronize()
print("ok")
