"""Diagnostic: cfg1 E-step at steady state (after 20 EM iterations) with the factorised-weight
pass on and off (SBCE_ESTEP_PAIR), same process; env SNR (default 20)."""
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
eng.run(20)
torch.cuda.synchronize()
for arm in ("1", "0", "1", "0"):
    with pkg._lib.debug_env(SBCE_ESTEP_PAIR=arm):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        eng.estep()
        e0.record()
        for _ in range(5):
            eng.estep()
        e1.record()
        torch.cuda.synchronize()
        print(f"pair={arm} E-step {e0.elapsed_time(e1) / 5:.3f} ms", flush=True)
