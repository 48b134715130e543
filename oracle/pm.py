"""Partitioned-detector (PM) EM estimators — float64 restatement (oracle).

TEST INFRASTRUCTURE ONLY (see oracle/__init__.py).

Follows "Proposed method/PM.py":47-116 (uniform list weights, lstsq) and
"Proposed method/PM_beta.py":42-112 (posterior list weights, solve), which
all_detectorsvsTd.py:176-249 and SNR/all_Detectors.py:170-240 repeat.
Reference quirks kept on purpose (SURVEY.md §7 hard part 5):
  * the list is built with the OFF-BY-ONE effective channel
      H_off = H_BU + sum_{n<N} G_{n+1} PsiTilde_td[n, t]      (PM.py:63)
  * the candidate vector is the concatenation [x_A, x_B] in the greedy
    stream order j and is then used as if it were in natural stream order
    (PM.py:101-104);
  * the soft weights use the CORRECT regressor Z_{t} built from the full
    PsiTilde_td[:, t] (PM_beta.py:88-93);
  * the oracle early stop |‖theta‖ - ‖h‖| < 1 (l != 0) (PM.py:110-112).
"""
import itertools

import numpy as np
from numpy.linalg import norm


def _stream_order(channel):
    """Greedy ordering PM.py:64-73: repeatedly remove the column with the largest
    diag(pinv(A^H A)) (np.argmax on the complex diagonal: first maximum)."""
    n_tx = channel.shape[1]
    j, j_c = [], list(range(n_tx))
    arr = channel
    for _ in range(n_tx):
        yeta = np.diag(np.linalg.pinv(np.conj(arr).T @ arr))
        k = int(np.argmax(yeta))
        j.append(j_c[k])
        arr = np.delete(arr, k, axis=1)
        del j_c[k]
    return j


def pm_list(y, channel, qamCons, partition_r, M):
    """Candidate list of one symbol (PM.py:60-104): returns (n_list, n_tx) array of
    concatenated [x_A, x_B] vectors."""
    n_tx = channel.shape[1]
    j = _stream_order(channel)
    p = int(partition_r / np.log2(M))
    chA = channel[:, j[:p + 1]]
    chB = channel[:, j[p + 1:]]
    candA = np.asarray(list(itertools.product(*([qamCons] * (p + 1)))))
    out = []
    if chB.shape[1]:
        G = np.linalg.inv(np.conj(chB).T @ chB) @ np.conj(chB).T
    for a in candA:
        if chB.shape[1]:
            z = G @ (y - chA @ a)
            # exhaustive argmin over M^{|B|} of ||z - b||^2 is separable: per-element nearest
            b = np.array([qamCons[int(np.argmin(np.abs(zz - qamCons) ** 2))] for zz in z])
            out.append(np.concatenate([a, b]))
        else:
            out.append(np.asarray(a))
    return np.asarray(out)


def pm_moments(theta, Y_d, Psi, qamCons, n_tx, n_rx, partition_r, varn, soft):
    """PM E-step of one trial: m (T,n_tx), S (T,n_tx,n_tx) summed over the list with
    weight 1 (PM.py:103-104) or posterior weights (PM_beta.py:88-95)."""
    M = len(qamCons)
    P, T = Psi.shape
    N = P - 1
    theta = np.asarray(theta, dtype=complex).reshape(-1)
    th = theta.reshape(-1, 1)
    h_bu = th[:n_tx * n_rx].reshape((n_rx, n_tx), order="F")
    prod = th[n_tx * n_rx:].reshape((n_tx * n_rx, N), order="F")
    H3 = theta.reshape(P, n_tx, n_rx)
    m = np.zeros((T, n_tx), dtype=complex)
    S = np.zeros((T, n_tx, n_tx), dtype=complex)
    for t in range(T):
        channel = h_bu + (prod @ Psi[:N, t]).reshape((n_rx, n_tx), order="F")
        lst = pm_list(Y_d[t], channel, qamCons, partition_r, M)
        if soft:
            Htrue = np.einsum("par,p->ra", H3, Psi[:, t])
            d = np.sum(np.abs(Y_d[t][None, :] - lst @ Htrue.T) ** 2, axis=1)
            w = np.exp(-(d - d.min()) / varn ** 2)
            w /= w.sum()
        else:
            w = np.ones(lst.shape[0])
        m[t] = w @ lst
        S[t] = np.einsum("j,ja,jb->ab", w, lst, np.conj(lst))
    return m, S


def em_pm(Y_d, Y_p, U_p, Psi, varn, itera, theta0, n_tx, n_rx, partition_r, qamCons,
          soft=False, h=None, return_trace=False, solve=None):
    """PM EM over one trial, array inputs (Y_d (T_d,n_rx), Psi (N+1,T_d), U_p (T_p,L)).
    Reduced-form M-step; list weights uniform (soft=False, PM.py, np.linalg.lstsq at
    PM.py:108) or posterior (soft=True, PM_beta.py, np.linalg.solve at PM_beta.py:104);
    ``solve`` ('lstsq' / 'solve') overrides the reference's choice."""
    from .em_reduced import mstep_build, mstep_solve, mstep_lstsq
    solve = solve or ("solve" if soft else "lstsq")
    theta = np.asarray(theta0, dtype=complex).reshape(-1)
    trace = []
    for l in range(itera):
        m, S = pm_moments(theta, Y_d, Psi, qamCons, n_tx, n_rx, partition_r, varn, soft)
        R, rhs = mstep_build(U_p, Y_p, Psi, Y_d, m, S)
        theta = mstep_lstsq(R, rhs)[0] if solve == "lstsq" else mstep_solve(R, rhs)
        trace.append(theta.copy())
        if h is not None and np.abs(norm(theta) - norm(h)) < 1 and l != 0:
            break
    return (theta, trace) if return_trace else theta
