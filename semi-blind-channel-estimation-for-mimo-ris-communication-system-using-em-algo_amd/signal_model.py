"""Synthetic MIMO-RIS data, host side (NumPy).  Not the hot path: it produces the
inputs that the sweep drivers and the benchmark hand to the GPU estimator.

Two generators:

* **Reference replay** (``channel_matrix``, ``symbols``, ``pilot_symbols``,
  ``irs_matrix``, ``received_signals``): the reference helpers restated with
  the SAME legacy ``RandomState`` calls in the SAME order
  ("Proposed method/Proposed_method_NMSEvsTp.py":18-47, 86-97, 114-130), so that
  ``np.random.seed(s)`` followed by the reference script's call order reproduces
  the reference's channels, symbols, phases and noise bit for bit.  The default
  ``rs`` is NumPy's global RandomState, exactly what the reference draws from.
  Observations are formed as H_c u + n (reduced form), equal to the reference's
  Z h + n up to float64 rounding.
* **Batch generator** (``synthetic_batch``): the same distributions, vectorised
  over Monte-Carlo trials with a ``numpy.random.Generator`` (statistical parity
  only), for the benchmark and large sweeps.

Layouts follow include/sbce.h: theta/h index (p*n_tx + a)*n_rx + r, RIS phases
as (P, T) like the reference's PsiTilde (row 0 = direct path = 1).
"""
import numpy as np
from scipy import linalg as sla

from .qam import qam_constellation, all_possible_symbols


def _rs(rs):
    return np.random.mtrand._rand if rs is None else rs


# ----------------------------------------------------------------- reference replay

def channel_matrix(n_tx, n_rx, N, varh=1.0, order="F", rs=None):
    """h = [vec(H_BU); vec(khatri_rao(H_BS^T, H_SU))] (PMd/Proposed_method_NMSEvsTp.py:18-24).
    ``order='C'`` reproduces the root-level scripts' row-major flatten
    (Proposed_method_NMSEvsTp.py:16)."""
    rs = _rs(rs)
    H_BU = rs.normal(loc=0, scale=np.sqrt(varh / 2), size=(n_rx, n_tx * 2)).view(np.complex128)
    H_BS = rs.normal(loc=0, scale=np.sqrt(varh / 2), size=(N, n_tx * 2)).view(np.complex128)
    H_SU = rs.normal(loc=0, scale=np.sqrt(varh / 2), size=(n_rx, N * 2)).view(np.complex128)
    return np.concatenate((H_BU.flatten(order=order),
                           sla.khatri_rao(H_BS.T, H_SU).flatten(order=order)))


def symbols(n_tx, M, T_d, rs=None):
    """X_d (T_d x (n_tx,1)) and all_possibleSymbols (PMd/Proposed_method_NMSEvsTp.py:26-39)."""
    rs = _rs(rs)
    cons = qam_constellation(M)
    X_d = [np.reshape(cons[rs.choice(range(0, M), n_tx, "True")], (n_tx, 1)) for _ in range(T_d)]
    return X_d, all_possible_symbols(cons, n_tx)


def pilot_symbols(n_tx, M, T_p, rs=None):
    """X_p (PMd/Proposed_method_NMSEvsTp.py:41-47)."""
    rs = _rs(rs)
    cons = qam_constellation(M)
    return [np.reshape(cons[rs.choice(range(0, M), n_tx, "True")], (n_tx, 1)) for _ in range(T_p)]


def irs_matrix(T_p, T_d, N, beta_min=0.0, beta_max=2 * np.pi, amp=1.0, pilot="dft_n", rs=None,
               data="random"):
    """(PsiTilde_tp, PsiTilde_td) of PMd/Proposed_method_NMSEvsTp.py:86-97.

    pilot='dft_n'  : (N+1) x T_p, rows n < N = exp(-2j pi t n / N), row N = 0 (PMd scripts)
    pilot='dft_tp' : N x T_p, exp(-2j pi t n / T_p) (root scripts :73-77; the caller
                     inserts the ones row, :129)
    pilot='dft_n_full': (N+1) x T_p, all rows filled (PMd/Log_likelihood.py:106-108)
    data='random'  : PsiTilde_td is N x T_d uniform phases in [beta_min, beta_max)
    data='dft_td'  : the root T_d script's deterministic data phases (Proposed_method_NMSEvsTd.py
                     :92-94): (N+1) x T_d exp(-2j pi t n / T_d), whose row 0 is the direct path's
                     ones -- returned as rows 1..N (N x T_d, no RNG draw) so that insert_direct
                     gives the reference's matrix, as for the random phases.
    """
    rs = _rs(rs)
    # element-wise scalar evaluation, exactly as the reference loops (bitwise replay)
    if pilot == "dft_n":
        Ptp = np.zeros((N + 1, T_p), dtype=complex)
        rows, den = N, N
    elif pilot == "dft_n_full":
        Ptp = np.zeros((N + 1, T_p), dtype=complex)
        rows, den = N + 1, N
    elif pilot == "dft_tp":
        Ptp = np.zeros((N, T_p), dtype=complex)
        rows, den = N, T_p
    else:
        raise ValueError(pilot)
    for n in range(rows):
        for t in range(T_p):
            Ptp[n, t] = np.exp((-1j * 2 * np.pi * (t) * (n)) / (den))
    if data == "dft_td":
        return Ptp, dft_phases(N + 1, T_d, T_d)[1:]
    if data != "random":
        raise ValueError(data)
    cols = []
    for _ in range(T_d):
        beta = (beta_max - beta_min) * rs.uniform(0, 1, (N, 1)) + beta_min
        cols.append(amp * np.exp(1j * beta))
    Ptd = np.concatenate(cols, axis=1) if cols else np.zeros((N, 0), dtype=complex)
    return Ptp, Ptd


def dft_phases(rows, T, den):
    """rows x T matrix exp(-2j pi t n / den), element-wise as the reference loops
    (Parallel/ParallelProtocol_Tp.py:89-94 uses rows = N+1, den = T)."""
    Psi = np.zeros((rows, T), dtype=complex)
    for n in range(rows):
        for t in range(T):
            Psi[n, t] = np.exp((-1j * 2 * np.pi * (t) * (n)) / (den))
    return Psi


def insert_direct(Psi):
    """Prepend the direct-path ones row (PMd/Proposed_method_NMSEvsTp.py:161)."""
    return np.insert(Psi, 0, np.ones((1, Psi.shape[1]), dtype="complex128"), axis=0)


def pilot_regressors(Psi_p, X_p):
    """u_p = psi_p (x) x_p (T_p x L); Z_p[t] = u_p^T (x) I_{n_rx}."""
    if isinstance(X_p, list):
        if not X_p:
            return np.zeros((0, 0), dtype=complex)
        X = np.stack([np.asarray(x).reshape(-1) for x in X_p])
    else:
        X = X_p
    return np.einsum("pt,ta->tpa", Psi_p, X).reshape(Psi_p.shape[1], -1)


def observe(h, U, n_rx, noise):
    """y_t = H_c u_t + n_t with H_c[r, l] = h[l*n_rx + r]."""
    H = np.asarray(h).reshape(-1, n_rx).T
    return U @ H.T + noise


def initial_estimate(U_p, Y_p, n_rx, pinv="numpy"):
    """h_initial = pinv(vstack Z_p) vstack Y_p (PMd/Proposed_method_NMSEvsTp.py:129), in
    reduced form H_0 = Y_p^T pinv(U_p^T) (pinv(U (x) I) = pinv(U) (x) I: the same singular
    values, n_rx times each).  pinv="numpy": np.linalg.pinv's default cut 1e-15 sigma_max;
    pinv="scipy": scipy.linalg.pinv's max(M, N) eps sigma_max on the (T_p n_rx) x K matrix --
    the one all_detectorsvsTd.py:341 uses (`from scipy import linalg`), which matters when the
    pilots leave rounding-level singular values (T_p < L)."""
    U = np.asarray(U_p)
    if pinv == "scipy":
        rc = max(U.shape[0] * n_rx, U.shape[1] * n_rx) * np.finfo(float).eps
        P = np.linalg.pinv(U.T, rcond=rc) if U.size else np.zeros(U.shape, dtype=complex)
    else:
        P = np.linalg.pinv(U.T)
    H0 = np.asarray(Y_p).T @ P
    return H0.T.reshape(-1)


def received_signals(T_p, T_d, Psi_tp, Psi_td, n_rx, n_tx, X_d, X_p, h, varn, rs=None,
                     with_initial=True, pinv="numpy"):
    """(Y_p, Y_d, U_p, U_d, h_initial) of PMd/Proposed_method_NMSEvsTp.py:114-130.

    Noise draws: one normal(0, sqrt(varn/2), (n_rx, 2)) per pilot, then per data
    symbol (same order as the reference).  U_d uses the TRUE data symbols
    (the reference's Z_d, genie regressors for the LLF)."""
    rs = _rs(rs)
    U_p = (pilot_regressors(Psi_tp[:, :T_p], X_p[:T_p]) if T_p
           else np.zeros((0, Psi_td.shape[0] * n_tx), dtype=complex))
    U_d = pilot_regressors(Psi_td, X_d)
    n_p = np.stack([rs.normal(loc=0, scale=np.sqrt(varn / 2), size=(n_rx, 2)).view(np.complex128)[:, 0]
                    for _ in range(T_p)]) if T_p else np.zeros((0, n_rx), dtype=complex)
    n_d = np.stack([rs.normal(loc=0, scale=np.sqrt(varn / 2), size=(n_rx, 2)).view(np.complex128)[:, 0]
                    for _ in range(T_d)])
    Y_p = observe(h, U_p, n_rx, n_p)
    Y_d = observe(h, U_d, n_rx, n_d)
    h0 = initial_estimate(U_p, Y_p, n_rx, pinv) if with_initial else None
    return Y_p, Y_d, U_p, U_d, h0


def gaussian_channel(varh, N, n_rx, n_tx, rs=None):
    """channelMatrix1 of MIMO_Gaussian_proposed.py:9-14 in reduced form: h =
    vec(khatri_rao(H_BS^T, H_SU)) (column-major, no direct path); the reference's full
    matrix is H = kron(h^T, I_{n_rx}) (full_gaussian_channel)."""
    rs = _rs(rs)
    H_BS = rs.normal(loc=0, scale=np.sqrt(varh / 2), size=(N, n_tx * 2)).view(np.complex128)
    H_SU = rs.normal(loc=0, scale=np.sqrt(varh / 2), size=(n_rx, N * 2)).view(np.complex128)
    return sla.khatri_rao(H_BS.T, H_SU).flatten(order="F")


def full_gaussian_channel(h, n_rx):
    return np.kron(np.asarray(h)[None, :], np.eye(n_rx, dtype=complex))


def gaussian_symbols(n_tx, T, varx, rs=None):
    """symbols / pilotSymbols of MIMO_Gaussian_proposed.py:17-22: (n_tx, T) CN(0, varx)."""
    rs = _rs(rs)
    return rs.normal(loc=0, scale=np.sqrt(varx / 2), size=(n_tx, T * 2)).view(np.complex128)


def snr_to_varn(snr_db, power=10.0):
    """varn = power / 10^(SNR/10) (PMd/SNR/all_Detectors.py:351-354; power = 16-QAM E_s)."""
    return power / np.power(10.0, np.asarray(snr_db, dtype=float) / 10.0)


# ----------------------------------------------------------------- batch generator

def synthetic_batch(B, n_tx, n_rx, N, T_p, T_d, M, varn, seed=0, varh=1.0, direct=True,
                    pilot="dft_n", pinv="numpy"):
    """Vectorised Monte-Carlo batch with the reference's distributions.  pinv: the cut of
    h_initial's pseudo-inverse, "numpy" (np.linalg.pinv's 1e-15, Proposed_method_NMSEvsTp.py:129)
    or "scipy" (max(M, N) eps, the scipy.linalg.pinv of all_detectorsvsTd.py:341; see
    initial_estimate).  With T_p > N the DFT pilot phases repeat and the numpy cut keeps
    rounding-level singular values: theta_0 ~ 1e13.

    Returns a dict of batch-major arrays in the C-ABI layout:
      y_d (B,T_d,n_rx), y_p (B,T_p,n_rx), psi_d (B,T_d,P), u_p (B,T_p,L),
      h (B,K), theta0 (B,K), x_d (B,T_d,n_tx), cons (M,)
    """
    g = np.random.default_rng(seed)
    cons = qam_constellation(M)
    s = np.sqrt(varh / 2)
    H_BU = g.normal(0, s, (B, n_rx, n_tx)) + 1j * g.normal(0, s, (B, n_rx, n_tx))
    H_BS = g.normal(0, s, (B, N, n_tx)) + 1j * g.normal(0, s, (B, N, n_tx))
    H_SU = g.normal(0, s, (B, n_rx, N)) + 1j * g.normal(0, s, (B, n_rx, N))
    # G_n[r, a] = H_SU[r, n] * H_BS[n, a]  -> h[(p*n_tx + a)*n_rx + r]
    G = np.einsum("brn,bna->bnar", H_SU, H_BS)
    blocks = [np.transpose(H_BU, (0, 2, 1))[:, None]] if direct else []
    blocks.append(G)
    Hc = np.concatenate(blocks, axis=1)                      # (B, P, n_tx, n_rx)
    P = Hc.shape[1]
    h = Hc.reshape(B, -1)
    x_d = cons[g.integers(0, M, (B, T_d, n_tx))]
    x_p = cons[g.integers(0, M, (B, T_p, n_tx))]
    ph = g.uniform(0, 2 * np.pi, (B, T_d, N))
    psi_d = np.exp(1j * ph)
    if direct:
        psi_d = np.concatenate([np.ones((B, T_d, 1), dtype=complex), psi_d], axis=2)
    n = np.arange(N)[:, None]
    t = np.arange(T_p)[None, :]
    if pilot == "dft_n":
        Ptp = np.zeros((N + 1, T_p), dtype=complex)
        Ptp[:N] = np.exp((-1j * 2 * np.pi * t * n) / N)
    else:
        raise ValueError(pilot)
    if not direct:
        Ptp = Ptp[:N]
    u_p = np.einsum("pt,bta->btpa", Ptp, x_p).reshape(B, T_p, P * n_tx)
    u_d = np.einsum("btp,bta->btpa", psi_d, x_d).reshape(B, T_d, P * n_tx)
    Hm = np.transpose(Hc.reshape(B, P * n_tx, n_rx), (0, 2, 1))   # (B, n_rx, L)
    sn = np.sqrt(varn / 2)
    y_p = np.einsum("brl,btl->btr", Hm, u_p) + (g.normal(0, sn, (B, T_p, n_rx))
                                                + 1j * g.normal(0, sn, (B, T_p, n_rx)))
    y_d = np.einsum("brl,btl->btr", Hm, u_d) + (g.normal(0, sn, (B, T_d, n_rx))
                                                + 1j * g.normal(0, sn, (B, T_d, n_rx)))
    # h_initial = H_0 = Y_p^T pinv(U_p^T), batched
    rc = (max(T_p, P * n_tx) * n_rx * np.finfo(float).eps if pinv == "scipy" else 1e-15)
    Pi = np.linalg.pinv(np.transpose(u_p, (0, 2, 1)), rcond=rc)    # (B, T_p, L)
    H0 = np.einsum("btr,btl->brl", y_p, Pi)                         # (B, n_rx, L)
    theta0 = np.transpose(H0, (0, 2, 1)).reshape(B, -1)
    return dict(y_d=y_d, y_p=y_p, psi_d=psi_d, u_p=u_p, h=h, theta0=theta0, x_d=x_d,
                cons=cons, varn=float(varn), n_tx=n_tx, n_rx=n_rx, P=P, T_p=T_p, T_d=T_d, M=M)
