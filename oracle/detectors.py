"""ZF / MMSE detector EMs — float64 restatement (oracle).

TEST INFRASTRUCTURE ONLY (see oracle/__init__.py).

Follows "Proposed method/all_detectorsvsTd.py":54-96 (em_mmse) and :98-133 (em_zf).
Per data symbol, with the OFF-BY-ONE list channel H_off of PM.py:63 (:70, :111):
    z = (H^H H + varn^2 I)^{-1} H^H y      (MMSE, :71)
    z = pinv(H) y                          (ZF, :112)
then nearest_symbol_ecul (:49-52): the distances |z - s| are taken between the (n_tx, 1)
column z and every ROW s of all_possibleSymbols, which broadcasts to (n_tx, n_tx) per row;
np.argmin flattens over (J, n_tx, n_tx) and the FLAT index selects a row of
all_possibleSymbols.  The chosen row enters the M-step with weight 1 (hard decision)
through the correct regressor PsiTilde_td[:, t] (:83-84); np.linalg.solve; oracle early
stop |‖theta‖ - ‖h‖| < 1 for l != 0 (:88-90).  A flat index >= J raises IndexError in
the reference, as here.
"""
import numpy as np
from numpy.linalg import norm


def ecul_literal(z, aps):
    """nearest_symbol_ecul exactly as written (:49-52)."""
    z = np.asarray(z).reshape(-1, 1)
    distances = [np.abs(z - s) for s in aps]
    return aps[np.argmin(distances)]


def ecul_index(z, aps, M):
    """Closed form of the flat argmin: the global minimum is min_a dist(z_a, cons); its
    first flat occurrence is j = s* M^(n_tx-1-b) with b = 0 when s* = 0 and b = n_tx-1
    otherwise, i.e. flat = a* n_tx (s* = 0) or s* n_tx^2 + a* n_tx + n_tx - 1."""
    z = np.asarray(z).reshape(-1)
    n_tx = z.size
    cons = np.asarray(aps)[:M, -1]
    d = np.abs(z[:, None] - cons[None, :])             # (n_tx, M)
    a = int(np.argmin(d.min(axis=1)))
    s = int(np.argmin(d[a]))
    return a * n_tx if s == 0 else s * n_tx * n_tx + a * n_tx + n_tx - 1


def detector_moments(theta, Y_d, Psi, aps, varn, n_tx, n_rx, kind, cons=None):
    """Hard-decision moments m_t = x_t, S_t = x_t x_t^H of em_zf / em_mmse.  With
    aps=None (n_tx too large for the M^n_tx table) the decision uses ecul_index on `cons`
    (row `flat` of the itertools.product table, computed from its digits)."""
    P, T = Psi.shape
    N = P - 1
    th = np.asarray(theta, dtype=complex).reshape(-1, 1)
    h_bu = th[:n_tx * n_rx].reshape((n_rx, n_tx), order="F")
    prod = th[n_tx * n_rx:].reshape((n_tx * n_rx, N), order="F")
    m = np.zeros((T, n_tx), dtype=complex)
    for t in range(T):
        H = h_bu + (prod @ Psi[:N, t]).reshape((n_rx, n_tx), order="F")
        y = Y_d[t].reshape(-1, 1)
        if kind == "mmse":
            z = np.linalg.inv(H.conj().T @ H + varn ** 2 * np.eye(n_tx)) @ H.conj().T @ y
        else:
            z = np.linalg.pinv(H) @ y
        if aps is not None:
            m[t] = ecul_literal(z, aps)
        else:
            M = len(cons)
            tab = np.zeros((M, n_tx), dtype=complex)
            tab[:, -1] = cons                              # ecul_index reads the last column
            f = ecul_index(z, tab, M)
            if f >= M ** n_tx:
                raise IndexError("flat argmin past the hypothesis table (reference :52)")
            m[t] = [cons[(f // M ** (n_tx - 1 - b)) % M] for b in range(n_tx)]
    S = m[:, :, None] * np.conj(m[:, None, :])
    return m, S


def em_detector(Y_d, Y_p, U_p, Psi, aps, varn, itera, theta0, n_tx, n_rx, kind, h=None,
                cons=None):
    """aps=None with cons given: the decisions through ecul_index (the closed form of the flat
    argmin, pinned to ecul_literal by tests/test_oracle.py) instead of the literal scan over the
    M^n_tx rows -- the same rows, ~20x faster at 64-QAM."""
    from .em_reduced import mstep_build, mstep_solve
    theta = np.asarray(theta0, dtype=complex).reshape(-1)
    for l in range(itera):
        m, S = detector_moments(theta, Y_d, Psi, aps, varn, n_tx, n_rx, kind, cons=cons)
        R, rhs = mstep_build(U_p, Y_p, Psi, Y_d, m, S)
        theta = mstep_solve(R, rhs)
        if h is not None and np.abs(norm(theta) - norm(h)) < 1 and l != 0:
            break
    return theta
