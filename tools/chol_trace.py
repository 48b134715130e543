"""Diagnostic: cfg1 M-steps (1000 trials) with the given SBCE_CHOL_IMPL, for a kernel trace of
the Cholesky launches (tools/trace_calls.py)."""
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
for arm in sys.argv[1:]:
    with pkg._lib.debug_env(SBCE_CHOL_IMPL=arm):
        for _ in range(2):
            eng.mstep()
        torch.cuda.synchronize()
print("ok")
