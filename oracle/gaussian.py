"""Gaussian-prior EM — float64 restatement (oracle).

TEST INFRASTRUCTURE ONLY (see oracle/__init__.py).

Follows "Proposed method/MIMO_Gaussian_proposed.py": EM_Gaussian_proposed (:56-89) with
variance_z (:33-45) and the lstsq-based inv (:47-53).  The unknown is the full
n_rx x Q matrix H (Q = N n_tx n_rx^2, the regressor z_t = vec(kron(kron(psi_t^T, x_t^T),
I_{n_rx})) of received_proposed :126/:132), the symbols have the Gaussian prior
x ~ CN(0, varx I) and the E-step is the linear-Gaussian posterior of z_t:
    Sigma_t = varx^2 kron(kron(psi psi^H, I_{n_tx}), e e^H)   (e = vec(I_{n_rx});
              comm_mat(1, n) = I so the P, Q permutations of :35-36 are identities)
    mu_t    = Sigma_t H^H (varn^2 I + H Sigma_t H^H)^+ y_t             (:71-72)
    covar_t = Sigma_t - Sigma_t H^H (...)^+ H Sigma_t + ||mu_t||^2     (:73-75)
The last term is the reference's ``mean_prod``: ``mu @ conj(mu).T`` of a 1-D column
is the scalar ||mu||^2, broadcast onto EVERY entry of covar.  M-step (:77-85):
    H[r] = (sum_p y_p[r] z_p^H + sum_t y_d[r] mu_t^H) pinv(sum_p z_p z_p^H + sum_t covar_t)
with pinv = lstsq(., I) (:53).  The loop runs itera + 1 times (``while j <= itera``).

Two faces:
  * ``em_gaussian_literal`` — the Q x Q computation as written (small sizes only);
  * ``em_gaussian_reduced`` — what the GPU computes: with H_eff(t) = sum_n psi_n Hr_n
    (Hr = the reduced n_rx x (N n_tx) channel, Hr[:, c] = H[:, block c] e), per symbol
        m_t = varx^2 H_eff^H M_t^-1 y_t,  C_t = varx^2 I - varx^4 H_eff^H M_t^-1 H_eff
    (M_t = varn^2 I + varx^2 H_eff H_eff^H), evaluated in the equivalent push-through form
        A_t = H_eff^H H_eff + (varn^2 / varx^2) I,  m_t = A_t^-1 H_eff^H y_t,  C_t = varn^2 A_t^-1,
    G = sum_p u_p u_p^H + sum_t (psi_t psi_t^H) (x) C_t (the reduced M-step with S_t = C_t),
    Hr = B G^-1 (B = sum_p y_p u_p^H + sum_t y_t (psi_t (x) m_t)^H); for n_rx = 1 the
    all-ones term stays: G + c 1 1^T, c = sum_t ||psi_t||^2 ||m_t||^2.  ``expand`` maps Hr
    back to the n_rx x Q matrix the reference returns (pinv of kron(G, e e^T) + c J).
"""
import numpy as np


def z_vector(psi, x, n_rx):
    """vec(kron(kron(psi^T, x^T), I_{n_rx})) in column-major order (:126, :132)."""
    a = np.kron(psi, x)
    K = np.kron(a[None, :], np.eye(n_rx, dtype=complex))
    return K.flatten(order="F")


def sigma_z(psi, n_tx, n_rx, varx):
    """variance_z (:33-45) with the identity permutations folded away."""
    e = np.eye(n_rx, dtype=complex).flatten(order="F")
    core = np.kron(np.outer(psi, np.conj(psi)), np.eye(n_tx, dtype=complex))
    return varx ** 2 * np.kron(core, np.outer(e, np.conj(e)))


def _pinv_lstsq(A):
    return np.linalg.lstsq(A, np.eye(A.shape[0]), rcond=None)[0]


def em_gaussian_literal(Y_d, Y_p, Z_p, Psi_td, varn, itera, H0, varx, n_tx):
    """Y_d (T_d, n_rx), Y_p (T_p, n_rx), Z_p (T_p, Q), Psi_td (N, T_d), H0 (n_rx, Q)."""
    n_rx = Y_d.shape[1]
    T_d = Y_d.shape[0]
    H = np.asarray(H0, dtype=complex)
    Q = H.shape[1]
    for _ in range(itera + 1):
        A = np.zeros((Q, Q), dtype=complex)
        for z in Z_p:
            A += np.outer(z, np.conj(z))
        Bm = Y_p.T @ np.conj(Z_p)                         # (n_rx, Q): sum_p y_p z_p^H
        for t in range(T_d):
            S = sigma_z(Psi_td[:, t], n_tx, n_rx, varx)
            Mid = varn ** 2 * np.eye(n_rx) + H @ S @ np.conj(H).T
            W = S @ np.conj(H).T @ _pinv_lstsq(Mid)
            mu = W @ Y_d[t]
            A += S - W @ H @ S + np.vdot(mu, mu)
            Bm += np.outer(Y_d[t], np.conj(mu))
        H = Bm @ _pinv_lstsq(A)
    return H


def reduce_channel(H, n_tx, n_rx):
    """Hr[:, c] = H[:, c n_rx^2 : (c+1) n_rx^2] e  (only this part reaches the E-step)."""
    Q = H.shape[1]
    blocks = H.reshape(n_rx, Q // (n_rx * n_rx), n_rx, n_rx)     # [r][c][j][k], i = j n + k
    return np.einsum("rcjj->rc", blocks)


def expand(Hr, n_rx):
    """The n_rx x Q matrix H = B pinv(A) of the reference from the reduced Hr = B_r G^-1."""
    Lr = Hr.shape[1]
    if n_rx == 1:
        return Hr.copy()
    e = np.eye(n_rx).flatten(order="F")
    f = 1.0 - e
    s = Hr.sum(axis=1)
    return (np.einsum("rc,i->rci", Hr, e) / n_rx
            - (s / (Lr * (n_rx * n_rx - n_rx)))[:, None, None] * f[None, None, :]).reshape(n_rx, -1)


def gaussian_moments(Hr, Y_d, Psi_td, varn, varx, n_tx):
    """Per-symbol LMMSE mean m_t and posterior covariance C_t (reduced E-step)."""
    n_rx = Y_d.shape[1]
    T_d = Y_d.shape[0]
    N = Psi_td.shape[0]
    vx = varx ** 2
    Hc = Hr.reshape(n_rx, N, n_tx)
    m = np.zeros((T_d, n_tx), dtype=complex)
    C = np.zeros((T_d, n_tx, n_tx), dtype=complex)
    for t in range(T_d):
        He = np.einsum("rna,n->ra", Hc, Psi_td[:, t])
        # push-through form of vx H^H (varn^2 I + vx H H^H)^-1 (.) (positive definite C)
        Ainv = np.linalg.inv(np.conj(He).T @ He + (varn ** 2 / vx) * np.eye(n_tx))
        m[t] = Ainv @ (np.conj(He).T @ Y_d[t])
        C[t] = varn ** 2 * Ainv
    return m, C


def em_gaussian_reduced(Y_d, Y_p, U_p, Psi_td, varn, itera, Hr0, varx, n_tx):
    """U_p (T_p, N n_tx) pilot regressors psi_p (x) x_p; Hr0 (n_rx, N n_tx).  Returns Hr."""
    n_rx = Y_d.shape[1]
    Hr = np.asarray(Hr0, dtype=complex)
    L = Hr.shape[1]
    for _ in range(itera + 1):
        m, C = gaussian_moments(Hr, Y_d, Psi_td, varn, varx, n_tx)
        G = np.einsum("tl,tk->lk", U_p, np.conj(U_p))    # sum_p u u^H
        Bm = np.einsum("tr,tl->rl", Y_p, np.conj(U_p))
        for t in range(Y_d.shape[0]):
            psi = Psi_td[:, t]
            G += np.kron(np.outer(psi, np.conj(psi)), C[t])
            Bm += np.outer(Y_d[t], np.conj(np.kron(psi, m[t])))
        if n_rx == 1:
            c = sum(np.vdot(Psi_td[:, t], Psi_td[:, t]).real * np.vdot(m[t], m[t]).real
                    for t in range(Y_d.shape[0]))
            G = G + c * np.ones((L, L))
        Hr = Bm @ np.linalg.inv(G)
    return Hr
