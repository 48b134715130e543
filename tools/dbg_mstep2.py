import os, sys
sys.path.insert(0, os.getcwd())
import numpy as np
import __graft_entry__ as ge
sbce = ge.package()
sbce._lib.use_ab()       # the A/B build: SBCE_* switches, counters, clocks
order = sys.argv[1]
b = sbce.signal_model.synthetic_batch(2, 2, 2, 8, 12, 40, 4, 0.05, seed=4)
x = b["x_d"]; S = x[..., :, None] * np.conj(x[..., None, :]) + 0.1 * np.eye(2)
def run(tag):
    try:
        out = sbce.mstep_batch(b["y_d"], b["y_p"], b["psi_d"], b["u_p"], b["cons"], x, S, 0.05)
        print(tag, "ok", out[3], flush=True)
    except Exception as e:
        print(tag, "FAIL", e, flush=True)
for step in order:
    if step == "d":
        with sbce._lib.debug_env(SBCE_CHOL_IMPL="batched", SBCE_BACKSUB="0", SBCE_CPLX3="1"):
            run("in-debug-env")
    elif step == "e":
        with sbce._lib.debug_env(SBCE_CPLX3="1"):
            run("cplx3-only")
    else:
        run("plain")
