"""Adapters from the reference's list-of-arrays interface to the C-ABI layout.

The reference passes the pilot regressors as dense Kronecker matrices
Z_p[t] = (psi_t^T (x) x_t^T) (x) I_{n_rx}  ("Proposed method/Proposed_method_NMSEvsTp.py":120)
and the hypothesis set as ``all_possibleSymbols`` in itertools.product order
(:32-38).  The reduced form needs only u_t = psi_t (x) x_t and the constellation.
"""
import numpy as np


def u_from_zp(Z_p, n_rx):
    """u_t (T x L): row 0 of u^T (x) I holds u at every n_rx-th column."""
    Z = np.asarray(Z_p)
    return Z[:, 0, ::n_rx].copy()


def cons_from_aps(all_possibleSymbols, M):
    """Constellation in table order (the last stream cycles fastest)."""
    return np.asarray(all_possibleSymbols)[:M, -1].copy()


def check_structure(Z_p, U_p, n_rx, aps, cons, K):
    """Reject inputs that the reduced form would silently mis-handle.
    ``aps`` may be None (list detectors never enumerate M**n_tx hypotheses)."""
    M = cons.size
    if M & (M - 1):
        raise ValueError("constellation size must be a power of two")
    if aps is not None:
        _check_aps(np.asarray(aps), cons, M)
    _check_zp(Z_p, U_p, n_rx, K)


def _check_aps(aps, cons, M):
    n_tx = aps.shape[1]
    if aps.shape[0] != M ** n_tx:
        raise ValueError("all_possibleSymbols must hold all M**n_tx hypotheses")
    idx = np.indices((M,) * n_tx).reshape(n_tx, -1).T
    if not np.array_equal(aps, cons[idx]):
        raise ValueError("all_possibleSymbols is not in itertools.product order of one constellation")


def _check_zp(Z_p, U_p, n_rx, K):
    if len(Z_p):
        Z0 = np.asarray(Z_p[0])
        if Z0.shape != (n_rx, K):
            raise ValueError(f"Z_p[0] has shape {Z0.shape}, expected {(n_rx, K)}")
        ref = np.kron(U_p[0][np.newaxis], np.eye(n_rx))
        if not np.allclose(Z0, ref, rtol=0, atol=1e-12 * max(1.0, np.abs(Z0).max())):
            raise ValueError("Z_p is not of the form u^T (x) I_{n_rx}")
