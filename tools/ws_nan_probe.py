"""Diagnostic: which phase of an EMEngine run reads workspace it did not write?  Runs the E-step
and then the M-step alone (from the same theta_0) in a workspace pre-filled with 0x00 and with 0xFF
(NaN bit patterns) and reports which outputs differ.
  python tools/ws_nan_probe.py [n_tx n_rx N T_p T_d M solve]"""
import sys
import numpy as np
import torch

sys.path.insert(0, ".")
import __graft_entry__ as ge  # noqa: E402

pkg = ge.package()
args = [int(x) for x in sys.argv[1:7]] if len(sys.argv) > 6 else [4, 4, 149, 16, 200, 16]
solve = sys.argv[7] if len(sys.argv) > 7 else "chol"
n_tx, n_rx, N, T_p, T_d, M = args
varn = float(pkg.signal_model.snr_to_varn(20.0))
b = pkg.signal_model.synthetic_batch(2, n_tx, n_rx, N, T_p, T_d, M, varn, seed=11)
out = {}
for fill in (0x00, 0xFF):
    eng = pkg.EMEngine(b, varn, solve=solve)
    eng.ws_all.fill_(fill)
    eng.estep()
    mom = eng.mom.clone()
    eng.mstep()
    th = eng.theta.clone()
    eng.ws_all.fill_(fill)
    eng.theta.copy_(eng.theta0)
    eng.mom.copy_(out[0x00][0] if fill else mom)      # the same moments into a fresh workspace
    eng.mstep()
    th2 = eng.theta.clone()
    torch.cuda.synchronize()
    out[fill] = (mom, th, th2)
m0, t0, s0 = out[0x00]
m1, t1, s1 = out[0xFF]
fin = lambda t: bool(torch.isfinite(torch.view_as_real(t)).all())
print("moments equal", torch.equal(m0, m1), "finite", fin(m1))
print("theta after estep+mstep equal", torch.equal(t0, t1), "finite", fin(t1))
print("theta of mstep alone from equal moments equal", torch.equal(s0, s1), "finite", fin(s1))
