"""Symbol-error-rate path of the log-max EM — float64 restatement (oracle).

TEST INFRASTRUCTURE ONLY (see oracle/__init__.py).

"Proposed method/SER/log_max_SER.py": em (:51-84) returns theta and X_dest, the argmax
hypotheses of the LAST iteration's E-step (:77-78); the script's SER (:162) is
count_nonzero(np.array(X_d) - np.array(X_dest)) / (T_d n_tx) with X_d entries (n_tx, 1)
and X_dest entries (1, n_tx), i.e. a (T_d, n_tx, n_tx) broadcast.
"""
import numpy as np

from .em_reduced import estep_moments, mstep_build, mstep_solve


def em_hard_with_decisions(Y_d, Y_p, U_p, Psi, aps, varn, itera, theta0):
    """Log-max EM (reduced form) returning (theta, decisions of the last E-step)."""
    theta = np.asarray(theta0, dtype=complex).reshape(-1)
    dec = None
    for _ in range(itera):
        m, S, _, _ = estep_moments(theta, Y_d, Psi, aps, varn, "hard")
        dec = m.copy()
        R, rhs = mstep_build(U_p, Y_p, Psi, Y_d, m, S)
        theta = mstep_solve(R, rhs)
    return theta, dec


def ser_reference(X_d, X_dest):
    """log_max_SER.py:162 with the script's shapes."""
    X_d = np.asarray(X_d).reshape(len(X_d), -1)
    X_dest = np.asarray(X_dest).reshape(len(X_dest), -1)
    T_d, n_tx = X_d.shape
    return np.count_nonzero(X_d[:, :, None] - X_dest[:, None, :]) / (T_d * n_tx)


def ser_elementwise(X_d, X_dest):
    X_d = np.asarray(X_d).reshape(len(X_d), -1)
    X_dest = np.asarray(X_dest).reshape(len(X_dest), -1)
    return np.count_nonzero(X_d != X_dest) / X_d.size
