"""Superimposed-pilot EM — float64 restatement (oracle).

TEST INFRASTRUCTURE ONLY (see oracle/__init__.py).

Follows "Parallel/ParallelProtocol_Tp.py": em (:63-86) over T = max(T_d, T_p) symbols
carrying x_d,t + x_p,t (dataPilotSymbols :41-53, both zero-padded to T), with
hypotheses x_j + x_p,t (:72-79), no separate pilot block, theta_0 = 0 (:66) and
np.linalg.solve (:84).  Restated: the posterior of x_j given y_t is the ordinary one on
y_t - H_t x_p,t; the moments of x_j + x_p,t follow by the shift
    m' = m + x_p,   S' = S + m x_p^H + x_p m^H + x_p x_p^H.
"""
import numpy as np

from .em_reduced import estep_moments, heff, mstep_build, mstep_solve


def shifted_moments(theta, Y, Psi, aps, varn, X_sup, mode="soft"):
    n_tx = np.asarray(aps).shape[1]
    n_rx = Y.shape[1]
    H = heff(theta, Psi, n_tx, n_rx)                          # (T, n_rx, n_tx)
    Ys = Y - np.einsum("tra,ta->tr", H, X_sup)
    m, S, _, _ = estep_moments(theta, Ys, Psi, aps, varn, mode)
    mp = m + X_sup
    Sp = (S + m[:, :, None] * np.conj(X_sup)[:, None, :] + X_sup[:, :, None] * np.conj(m)[:, None, :]
          + X_sup[:, :, None] * np.conj(X_sup)[:, None, :])
    return mp, Sp


def em_superimposed(Y, Psi, aps, varn, itera, X_sup, theta0=None, mode="soft"):
    """Y (T, n_rx), Psi (N+1, T), X_sup (T, n_tx) padded pilot symbols."""
    n_tx = np.asarray(aps).shape[1]
    n_rx = Y.shape[1]
    L = Psi.shape[0] * n_tx
    theta = np.zeros(L * n_rx, dtype=complex) if theta0 is None else np.asarray(theta0, complex)
    U0 = np.zeros((0, L), dtype=complex)
    Y0 = np.zeros((0, n_rx), dtype=complex)
    for _ in range(itera):
        m, S = shifted_moments(theta, Y, Psi, aps, varn, X_sup, mode)
        R, rhs = mstep_build(U0, Y0, Psi, Y, m, S)
        theta = mstep_solve(R, rhs)
    return theta
