"""Reduced-form float64 restatement of the EM estimator (oracle face 2).

TEST INFRASTRUCTURE ONLY (see oracle/__init__.py).

Model (SURVEY.md §8 preamble): theta = vec(H_c), H_c is n_rx x L with
L = P * n_tx (P = number of RIS-phase rows, N+1 with the direct path), column
index p*n_tx + a, so theta[(p*n_tx + a)*n_rx + r] = H_c[r, p*n_tx + a]
(PMd/PM.py:11-17 'F'-order vec).  With u_{t,j} = psi_t (x) x_j the reference's
regressor is Z_{t,j} = u^T (x) I_{n_rx} (PMd/Proposed_method_NMSEvsTp.py:65), so
  * Z theta = H_c u,  Z^H Z = conj(u u^H) (x) I,  Z^H y = vec(y u^H)
    (the commutation identity of PMd/commutation_matrix.py:3-8);
  * the K x K normal equations of PMd/Proposed_method_NMSEvsTp.py:70-80 collapse
    to ONE L x L Hermitian system with n_rx right-hand sides:  H_c R = B with
      R = sum_p u_p u_p^H + sum_t (psi_t psi_t^H) (x) S_t,
      B = sum_p y_p u_p^H + sum_t y_t (psi_t (x) m_t)^H,
    m_t = E[x | y_t], S_t = E[x x^H | y_t] under the posterior beta_{t,j}
    (PMd/Proposed_method_NMSEvsTp.py:61-69; posterior exponent uses varn**2).
"""
import numpy as np


def u_from_zp(Z_p, n_rx):
    """Pilot regressors u_p (T_p x L) from the reference's Z_p list (row 0 of
    u^T (x) I holds u at every n_rx-th column)."""
    Z = np.asarray(Z_p)
    return Z[:, 0, ::n_rx].copy()


def cons_from_aps(all_possibleSymbols, M):
    """Constellation in table order: the last stream cycles fastest in
    itertools.product order (PMd/Proposed_method_NMSEvsTp.py:32-38)."""
    return np.asarray(all_possibleSymbols)[:M, -1].copy()


def aps_from_cons(cons, n_tx):
    """All J = M^n_tx hypotheses in itertools.product order (first stream slowest)."""
    cons = np.asarray(cons)
    M = cons.size
    idx = np.indices((M,) * n_tx).reshape(n_tx, -1).T
    return cons[idx]


def heff(theta, Psi, n_tx, n_rx):
    """Effective channel per symbol H_eff(t) = sum_p psi_{p,t} H_c[:, p*n_tx:(p+1)*n_tx]
    -> (T, n_rx, n_tx)."""
    P = Psi.shape[0]
    H3 = np.asarray(theta).reshape(P, n_tx, n_rx)          # [p, a, r]
    return np.einsum("par,pt->tra", H3, Psi)


def estep_moments(theta, Y_d, Psi, aps, varn, mode="soft", chunk=8):
    """Posterior moments per data symbol.

    mode 'soft': beta_{t,j} = softmax_j(-||y_t - Z_{t,j} theta||^2 / varn^2)
                 (PMd/Proposed_method_NMSEvsTp.py:61-69)
    mode 'hard': one-hot at argmax_j beta (first index on ties)
                 (PMd/ML_detecctor.py:65-75)
    Returns m (T, n_tx), S (T, n_tx, n_tx) with S[a,b] = E[x_a conj(x_b)],
    dmin (T,) and logZ (T,) = log sum_j exp(-(d_j - dmin)/varn^2).
    """
    aps = np.asarray(aps)
    J, n_tx = aps.shape
    n_rx = Y_d.shape[1]
    H = heff(theta, Psi, n_tx, n_rx)                          # (T, n_rx, n_tx)
    T = Y_d.shape[0]
    m = np.empty((T, n_tx), dtype=complex)
    S = np.empty((T, n_tx, n_tx), dtype=complex)
    dmin = np.empty(T)
    logZ = np.empty(T)
    inv = 1.0 / np.power(varn, 2)
    outer = aps[:, :, None] * np.conj(aps)[:, None, :]       # (J, n_tx, n_tx)
    for t0 in range(0, T, chunk):
        t1 = min(T, t0 + chunk)
        Hx = np.einsum("tra,ja->tjr", H[t0:t1], aps)          # (c, J, n_rx)
        r = Y_d[t0:t1, None, :] - Hx
        d = np.sum(r.real ** 2 + r.imag ** 2, axis=2)         # (c, J)
        dm = d.min(axis=1)
        dmin[t0:t1] = dm
        if mode == "hard":
            js = np.argmin(d, axis=1)
            w = np.zeros_like(d)
            w[np.arange(t1 - t0), js] = 1.0
            logZ[t0:t1] = 0.0
        else:
            w = np.exp(-(d - dm[:, None]) * inv)
            z = w.sum(axis=1)
            logZ[t0:t1] = np.log(z)
            w /= z[:, None]
        m[t0:t1] = w @ aps
        S[t0:t1] = np.einsum("tj,jab->tab", w, outer)
    return m, S, dmin, logZ


def mstep_build(U_p, Y_p, Psi, Y_d, m, S):
    """Reduced normal equations (R: L x L Hermitian, rhs = B^H: L x n_rx)."""
    P, T = Psi.shape
    n_tx = m.shape[1]
    L = P * n_tx
    R = U_p.T @ np.conj(U_p)
    R = R + np.einsum("pt,qt,tab->paqb", Psi, np.conj(Psi), S).reshape(L, L)
    rhs = U_p.T @ np.conj(Y_p)
    rhs = rhs + np.einsum("pt,ta,tr->par", Psi, m, np.conj(Y_d)).reshape(L, -1)
    return R, rhs


def mstep_build_gemm(U_p, Y_p, Psi, Y_d, m, S):
    """mstep_build as two GEMMs (same sums, any order): R[(p,a),(q,b)] = sum_t Psi[p,t]
    S_t[a,b] conj(Psi[q,t]) -- for the full-size (L = 2056 / 4100) checks, where the einsum
    would take minutes."""
    P, T = Psi.shape
    n_tx = m.shape[1]
    L = P * n_tx
    A = (Psi[:, None, None, :] * np.transpose(S, (1, 2, 0))[None]).reshape(P * n_tx * n_tx, T)
    R4 = (A @ np.conj(Psi).T).reshape(P, n_tx, n_tx, P)            # [p, a, b, q]
    R = np.transpose(R4, (0, 1, 3, 2)).reshape(L, L) + U_p.T @ np.conj(U_p)
    rhs = U_p.T @ np.conj(Y_p)
    rhs = rhs + ((Psi[:, None, :] * m.T[None]).reshape(L, T) @ np.conj(Y_d))
    return R, rhs


def mstep_lstsq(R, rhs):
    """np.linalg.lstsq of PMd/PM.py:108 on the reduced system.  The reference's K x K
    matrix A = sum Z^H Z = conj(R) (x) I_{n_rx} (up to the vec permutation) has R's
    eigenvalues as singular values, each n_rx times, and lstsq's default rcond is
    eps * max(K, K): the same cut applied to R's spectrum (K = L n_rx).  Returns
    (theta, rank of R)."""
    L, n_rx = rhs.shape
    X, _, rank, _ = np.linalg.lstsq(R, rhs, rcond=np.finfo(float).eps * L * n_rx)
    return np.conj(X).reshape(-1), int(rank)


def mstep_solve(R, rhs):
    """H_c R = B  <=>  R H_c^H = B^H; theta[l*n_rx + r] = conj(X[l, r])
    (PMd/Proposed_method_NMSEvsTp.py:80 np.linalg.solve on the K x K form)."""
    X = np.linalg.solve(R, rhs)
    return np.conj(X).reshape(-1)


def mstep_chol_policy(R, rhs, clamp=False, rel_tol=1e-14):
    """The device's CHOL solve policy for a non-HPD R, restated unblocked (right-looking):
    the np.linalg.solve of PMd/Proposed_method_NMSEvsTp.py:80 on an HPD R; a pivot
    <= rel_tol * max diag R is flagged and its direction DROPPED (column zeroed, its y and x
    components 0) -- libsbce since round 6, include/sbce.h SBCE_SOLVE_CHOL.
    clamp=True restates the round-5 policy instead (the pivot raised to sqrt(tol), the column
    kept), which overflows on a rank-deficient R: past the numerical rank the Schur complement
    is rounding noise delta, not PSD, and each clamped column feeds delta^2 / tol back.
    Returns (theta, bad) with bad the flagged pivots."""
    A = np.array(R, dtype=complex)
    L = A.shape[0]
    tol = rel_tol * np.max(A.diagonal().real)
    bad = np.zeros(L, dtype=bool)
    with np.errstate(all="ignore"):
        for c in range(L):
            d = A[c, c].real
            bad[c] = not d > tol
            if bad[c] and not clamp:
                A[c:, c] = 0.0
                continue
            piv = np.sqrt(tol if bad[c] else d)
            A[c, c] = piv
            col = A[c + 1:, c] / piv
            A[c + 1:, c] = col
            A[c + 1:, c + 1:] -= np.outer(col, col.conj())
        Lf = np.tril(A)
        y = np.array(rhs, dtype=complex)
        for c in range(L):
            y[c] = 0.0 if Lf[c, c] == 0 else (y[c] - Lf[c, :c] @ y[:c]) / Lf[c, c]
        x = np.zeros_like(y)
        for c in range(L - 1, -1, -1):
            x[c] = 0.0 if Lf[c, c] == 0 else (y[c] - Lf[c + 1:, c].conj() @ x[c + 1:]) / Lf[c, c]
    return np.conj(x).reshape(-1), bad


def range_part(R, theta, n_rx):
    """theta's component on R's numerical range (lstsq's cut eps * K * lambda_max on R's
    eigenvalues, K = L n_rx): for any solution of a consistent R X = B^H it is the
    minimum-norm solution, the size-independent check of a rank-deficient solve."""
    w, V = np.linalg.eigh(R)
    keep = w > np.finfo(float).eps * R.shape[0] * n_rx * w.max()
    Vr = V[:, keep]
    X = np.conj(np.asarray(theta).reshape(R.shape[0], n_rx))
    return np.conj(Vr @ (Vr.conj().T @ X)).reshape(-1)


def em_reduced(Y_d, Y_p, U_p, Psi, aps, varn, itera, theta0, mode="soft",
               return_trace=False, h=None):
    """Reduced-form EM over one trial.  Inputs in array form:
    Y_d (T_d, n_rx), Y_p (T_p, n_rx), U_p (T_p, L), Psi (P, T_d), aps (J, n_tx).
    h: the oracle early stop |‖theta‖ - ‖h‖| < 1 after an iteration l != 0 of
    PMd/all_detectorsvsTd.py:169-171 (em_ml) / :291-293 (em)."""
    theta = np.asarray(theta0, dtype=complex).reshape(-1)
    trace = []
    for l in range(itera):
        m, S, _, _ = estep_moments(theta, Y_d, Psi, aps, varn, mode)
        R, rhs = mstep_build(U_p, Y_p, Psi, Y_d, m, S)
        theta = mstep_solve(R, rhs)
        trace.append(theta.copy())
        if h is not None and abs(np.linalg.norm(theta) - np.linalg.norm(h)) < 1 and l != 0:
            break
    return (theta, trace) if return_trace else theta


def nmse(theta, h):
    """PMd/Proposed_method_NMSEvsTp.py:172: ||theta - h||^2 / ||h||^2."""
    theta = np.asarray(theta).reshape(-1)
    h = np.asarray(h).reshape(-1)
    return float(np.sum(np.abs(theta - h) ** 2) / np.sum(np.abs(h) ** 2))
