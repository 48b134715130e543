"""Diagnostic: the E-step moments of the saved cfg5 trial (tools/data/cfg5_nan_trial.npz, theta_0
~1e13 from a near-singular pinv) on every E-step path: default (tree + enumeration + sweep), the
tile sweep alone (SBCE_ESTEP_SPHERE=0), the VALU kernel; which symbols come out non-finite."""
import sys
import numpy as np

sys.path.insert(0, ".")
import __graft_entry__ as ge  # noqa: E402

pkg = ge.package()
pkg._lib.use_ab()       # the A/B build: SBCE_* switches, counters, clocks
d = np.load("tools/data/cfg5_nan_trial.npz")
vn = float(d["varn"])
for name, env in (("default", {}), ("sweep_only", dict(SBCE_ESTEP_SPHERE="0")),
                  ("valu", dict(SBCE_ESTEP_IMPL="valu")), ("noprune", dict(SBCE_ESTEP_PRUNE="0"))):
    with pkg._lib.debug_env(**env):
        m, S = pkg.estep_batch(d["y_d"][None], d["psi_d"][None], d["cons"], d["theta0"][None], vn, 2)
    bad = np.where(~(np.isfinite(m[0]).all(axis=1) & np.isfinite(S[0].reshape(len(m[0]), -1)).all(axis=1)))[0]
    print(name, "non-finite symbols", bad.tolist()[:20], "of", m.shape[1])
    if len(bad):
        t = bad[0]
        print("  symbol", t, "m", m[0, t], "S diag", np.diag(S[0, t]))
