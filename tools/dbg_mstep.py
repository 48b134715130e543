import os, sys
sys.path.insert(0, os.getcwd())
import numpy as np
import __graft_entry__ as ge
sbce = ge.package()
b = sbce.signal_model.synthetic_batch(2, 2, 2, 8, 12, 40, 4, 0.05, seed=4)
x = b["x_d"]; S = x[..., :, None] * np.conj(x[..., None, :]) + 0.1 * np.eye(2)
try:
    out = sbce.mstep_batch(b["y_d"], b["y_p"], b["psi_d"], b["u_p"], b["cons"], x, S, 0.05)
    print("mstep ok", out[3])
except Exception as e:
    print("mstep FAIL", e)
try:
    r = sbce.em_batch(b["y_d"], b["y_p"], b["psi_d"], b["u_p"], b["cons"], 0.05, 2, b["theta0"])
    print("em ok", r["status"])
except Exception as e:
    print("em FAIL", e)
