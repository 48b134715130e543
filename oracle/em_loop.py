"""Reference-structured float64 restatement of the EM estimators (oracle face 1).

TEST INFRASTRUCTURE ONLY (see oracle/__init__.py).

Each function follows the reference loop structure line by line, replacing the
object-dtype mpmath/gmpy2 arithmetic by float64 with a log-sum-exp shift
(mathematically identical weights; the reference uses ``gp.exp``/``mp.exp`` only
to avoid 0/0 when every ``exp(-d/varn^2)`` underflows).

Cost is O(T_d * J * K^2) per iteration: small cases only.
"""
import numpy as np
from numpy.linalg import norm


def _z(psi_t, x, n_rx):
    """Z_{t,j} = (psi_t^T (x) x_j^T) (x) I_{n_rx}
    (PMd/Proposed_method_NMSEvsTp.py:65, receivedSignals :120/:125)."""
    return np.kron(np.kron(psi_t[np.newaxis], np.asarray(x)[np.newaxis]),
                   np.eye(n_rx, dtype="complex128"))


def _pilot_terms(Y_p, Z_p):
    """Pilot normal-equation terms (PMd/Proposed_method_NMSEvsTp.py:72-74)."""
    K = Z_p[0].shape[1]
    numer = np.zeros((K, 1), dtype="complex128")
    denom = np.zeros((K, K), dtype="complex128")
    for t in range(len(Z_p)):
        numer += np.conj(Z_p[t]).T @ Y_p[t]
        denom += np.conj(Z_p[t]).T @ Z_p[t]
    return numer, denom


def em_loop(Y_d, Y_p, T_d, T_p, Z_p, PsiTilde_td, all_possibleSymbols, M, varn, itera,
            h_initial, hard=False, return_trace=False, skip_zero=True):
    """Exact soft EM — PMd/Proposed_method_NMSEvsTp.py:50-83 (identical contract at
    PMd/Proposed_method_NMSEvsTd.py:44-76, PMd/SNR/all_Detectors.py:242-274).

    ``hard=True`` gives the hard-ML ("log-max") E-step of
    PMd/ML_detecctor.py:65-77 / PMd/all_detectorsvsTd.py:143-155: only the
    posterior argmax (first index on ties, ``np.argmax``) enters the M-step.
    ``skip_zero=False`` accumulates zero-weight hypotheses too, as the reference loop does
    (:70-71): the full O(T_d J K^2) work, for bench.py's reference-structured CPU baseline.
    """
    n_rx = Y_d[0].shape[0]
    aps = np.asarray(all_possibleSymbols)
    J = aps.shape[0]
    theta = np.asarray(h_initial, dtype="complex128").reshape(-1, 1)
    K = theta.shape[0]
    trace = []
    for _ in range(itera):
        numer = np.zeros((K, 1), dtype="complex128")
        denom = np.zeros((K, K), dtype="complex128")
        for t in range(T_d):
            psi = PsiTilde_td[:, t]
            Zs = [_z(psi, aps[j], n_rx) for j in range(J)]
            d = np.array([norm(Y_d[t] - Z @ theta) ** 2 for Z in Zs])
            logw = -d / np.power(varn, 2)           # :66 exponent, posterior uses varn^2
            if hard:
                jstar = int(np.argmax(logw))        # ML_detecctor.py:75
                w = np.zeros(J)
                w[jstar] = 1.0
            else:
                w = np.exp(logw - logw.max())
                w /= w.sum()                        # :69 beta_exp
            for j in range(J):
                if skip_zero and w[j] == 0.0:
                    continue
                Z = Zs[j]
                numer += w[j] * (np.conj(Z).T @ Y_d[t])     # :70
                denom += w[j] * (np.conj(Z).T @ Z)          # :71
        pn, pd = _pilot_terms(Y_p, Z_p)
        theta = np.linalg.solve(pd + denom, pn + numer)     # :78-80 (LAPACK zgesv)
        trace.append(theta.copy())
    return (theta, trace) if return_trace else theta


def em_ml_loop(*args, **kw):
    """Hard-ML EM (PMd/ML_detecctor.py:51-86)."""
    return em_loop(*args, hard=True, **kw)


def llf_genie(theta, Y_p, Z_p, Y_d, Z_d, T_d, T_p, n_tx, M, varn):
    """Per-iteration log-likelihood function of PMd/IterationsvsLLF.py:49-50,76
    (same formula PMd/ML_detecctor.py:55-56,84).  Norms are NOT squared and Z_d is
    built from the TRUE data symbols (genie), exactly as in the reference."""
    e1 = T_d * n_tx * np.log(M)
    e2 = (T_d + T_p) * np.log(np.pi * (varn ** 2))
    theta = np.asarray(theta).reshape(-1, 1)
    rp = np.asarray(Y_p) - np.matmul(np.asarray(Z_p), theta)
    rd = np.asarray(Y_d) - np.matmul(np.asarray(Z_d), theta)
    return -e1 - e2 - (1 / varn ** 2) * norm(rp) - (1 / varn ** 2) * norm(rd)
