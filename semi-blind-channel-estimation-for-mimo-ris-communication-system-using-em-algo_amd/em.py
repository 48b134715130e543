"""Drop-in EM estimators with the reference's own signatures, running on the
MI355X through libsbce.so (ctypes C-ABI, include/sbce.h).  PyTorch-ROCm is used
only for device buffers and the current HIP stream.

Reference operator -> entry point here:
  em(Y_d, Y_p, T_d, T_p, Z_p, PsiTilde_td, all_possibleSymbols, M, varn, itera, h_initial)
      "Proposed method/Proposed_method_NMSEvsTp.py":50-83 (also
      Proposed_method_NMSEvsTd.py:44-76, SNR/all_Detectors.py:242-274)   -> em()
  em_ml(...same...)            all_detectorsvsTd.py:135-173, SNR/all_Detectors.py:132-167
                                                                        -> em_ml()
  em(..., Z_d, ..., n_tx)      IterationsvsLLF.py:45-77  (returns theta, LLF)
                                                                        -> em_llf()
  em(...) with LLF             ML_detecctor.py:51-86 (reads the global Z_d)
                                                                        -> em_ml_llf(..., Z_d=)
  em(... no h_initial ...)     root Proposed_method_NMSEvsTp.py:43-69 (zero init)
                                                                        -> em_zero_init()
  em_pm(..., h, n_tx, partition_r, X_d, qamCons)
                               PM.py:47-116 (uniform list weights)      -> em_pm()
  em_pm(... no all_possibleSymbols ...)
                               PM_beta.py:42-112 (posterior list weights) -> em_pm_soft()
  em_zf / em_mmse(..., h_initial, h)
                               all_detectorsvsTd.py:98-133 / :54-96      -> em_zf(), em_mmse()
  EM_Gaussian_proposed(y_d, y_p, T_d, T_p, z_p, PsiTilde_td, varn, itera, H_initial, varx, n_tx)
                               MIMO_Gaussian_proposed.py:56-89 (Gaussian prior)
                                                                        -> EM_Gaussian_proposed()
Batched form for sweeps / benchmark: ``em_batch`` (one sbce_em call for all trials).

Semantics kept from the reference: inputs are not mutated, theta is returned
as a fresh (K,1) complex128 array, the posterior exponent uses varn**2
(PMd/Proposed_method_NMSEvsTp.py:66) while the data were generated with noise
variance varn.  The reference's per-iteration ``print(norm(theta))`` is
available with ``verbose=True``.  Near-singular normal equations do not raise
(``np.linalg.solve`` only raises on an exactly zero LU pivot, which float
rounding essentially never produces): the device Cholesky drops a pivot at or below
1e-14 max diag R and flags the trial (``last_status``): theta stays finite and its
range-space part is lstsq's minimum-norm solution (where the reference's LU returns
rounding noise).  ``solve='lstsq'`` is np.linalg.lstsq of PM.py:108
(the minimum-norm solution with lstsq's default singular-value cut, include/sbce.h
SBCE_SOLVE_MINNORM): the reference's policy for rank-deficient normal equations and
the intended fallback of all_detectorsvsTd.py:238-241.  ``solve='drop'`` is the same
solve as 'chol' (kept for older callers).
"""
import ctypes

import numpy as np

from . import _lib
from .layout import cons_from_aps, u_from_zp, check_structure


def _torch():
    import torch
    if not torch.cuda.is_available():
        raise _lib.SbceUnavailable("no HIP device visible: the sbce estimator has no CPU path")
    return torch


def _dev(torch, arr, dtype=None):
    a = np.ascontiguousarray(arr, dtype=dtype)
    return torch.from_numpy(a).to("cuda", non_blocking=False)


_MODES = {"soft": _lib.SBCE_ESTEP_SOFT, "hard": _lib.SBCE_ESTEP_HARD, "pm": _lib.SBCE_ESTEP_PM,
          "pm_soft": _lib.SBCE_ESTEP_PM_SOFT, "zf": _lib.SBCE_ESTEP_ZF,
          "mmse": _lib.SBCE_ESTEP_MMSE, "gauss": _lib.SBCE_ESTEP_GAUSS}
_SOLVES = {"chol": _lib.SBCE_SOLVE_CHOL, "drop": _lib.SBCE_SOLVE_CHOL_DROP,
           "lstsq": _lib.SBCE_SOLVE_MINNORM}


def _varn_arg(torch, varn, B):
    """(dims.varn, per-trial device tensor or None) for a scalar or (B,) noise variance."""
    if np.ndim(varn) == 0 and not (isinstance(varn, torch.Tensor) and varn.dim() > 0):
        v = float(varn)
        if not v > 0:
            raise ValueError("varn must be > 0")
        return v, None
    v = np.ascontiguousarray(varn.cpu().numpy() if isinstance(varn, torch.Tensor) else varn,
                             dtype=np.float64).reshape(-1)
    if v.size != B:
        raise ValueError(f"per-trial varn has {v.size} entries, batch is {B}")
    if not np.all(v > 0):
        raise ValueError("varn must be > 0")
    return float(v[0]), torch.from_numpy(v).to("cuda")


def em_batch(y_d, y_p, psi_d, u_p, cons, varn, itera, theta0, mode="soft", x_d_true=None,
             h_true=None, solve="chol", return_device=False, partition_r=0,
             return_decisions=False, x_sup=None, varx=1.0):
    """Run ``itera`` EM iterations on a batch of independent trials.

    Array layouts (complex128, batch-major, include/sbce.h):
      y_d (B,T_d,n_rx), y_p (B,T_p,n_rx), psi_d (B,T_d,P) [RIS phases per data
      symbol, row 0 of the reference's PsiTilde_td = direct path], u_p (B,T_p,L),
      cons (M,), theta0 (B,K) with K = P*n_tx*n_rx.
    Optional: x_d_true (B,T_d,n_tx) -> per-iteration LLF (IterationsvsLLF.py:76);
    h_true (B,K) -> the reference's oracle early stop (PM.py:110-112).
    mode: "soft" | "hard" | "pm" | "pm_soft" | "zf" | "mmse"; partition_r selects the PM
    list size.  return_decisions (hard modes): x_dest (B,T_d,n_tx), the last E-step's
    decisions (SER/log_max_SER.py:77-78).  x_sup (B,T_d,n_tx): pilot symbols superimposed
    on the data (Parallel/ParallelProtocol_Tp.py:63-86), soft/hard modes.  mode "gauss":
    Gaussian-prior EM (MIMO_Gaussian_proposed.py:56-89) with prior variance parameter varx;
    psi_d then has P = N rows (no direct path), cons is ignored, theta is the reduced
    channel (gauss_expand_batch gives the reference's n_rx x Q matrix).
    Inputs may be numpy arrays or CUDA complex128 tensors (used in place).  varn may be one
    value or one per trial ((B,) array: the trials of several SNR points in one call, include/
    sbce.h sbce_ptrs.varn_t; each trial's result is that of a call with its own varn).
    Returns dict(theta (B,K), llf (B,itera) or None, status (B,), iters_done (B,)).
    """
    torch = _torch()
    lib = _lib.load()

    def dev(x):
        if x is None:
            return None
        if isinstance(x, torch.Tensor):
            t = x if x.is_cuda else x.to("cuda")
            return t.contiguous()
        return _dev(torch, x, np.complex128)

    Yd, Yp, Ps, Up, Cs = dev(y_d), dev(y_p), dev(psi_d), dev(u_p), dev(cons)
    th = dev(theta0).clone()
    B, T_d, n_rx = Yd.shape
    T_p = Yp.shape[1]
    P = Ps.shape[2]
    L = Up.shape[2]
    if L % P:
        raise ValueError("u_p width must be P*n_tx")
    n_tx = L // P
    M = Cs.shape[0]
    if th.shape != (B, L * n_rx):
        raise ValueError(f"theta0 shape {tuple(th.shape)} != {(B, L * n_rx)}")
    varn0, Vt = _varn_arg(torch, varn, B)
    dims = _lib.Dims(B, n_tx, n_rx, P, T_p, T_d, M, int(partition_r), varn0, float(varx))
    ws_bytes = _lib.workspace_bytes(dims, _SOLVES[solve])
    ws = torch.empty(max(ws_bytes, 16), dtype=torch.uint8, device="cuda")
    status = torch.zeros(B, dtype=torch.int32, device="cuda")
    iters_done = torch.zeros(B, dtype=torch.int32, device="cuda")
    Xd = dev(x_d_true)
    Ht = dev(h_true)
    llf = torch.zeros((B, max(itera, 1)), dtype=torch.float64, device="cuda") if Xd is not None else None
    xdest = (torch.zeros((B, T_d, n_tx), dtype=torch.complex128, device="cuda")
             if return_decisions else None)
    Xs = dev(x_sup)
    ptrs = _lib.Ptrs(Yd.data_ptr(), Yp.data_ptr() if T_p else Yd.data_ptr(), Ps.data_ptr(),
                     Up.data_ptr() if T_p else Yd.data_ptr(), Cs.data_ptr(), th.data_ptr(),
                     Xd.data_ptr() if Xd is not None else None,
                     llf.data_ptr() if llf is not None else None,
                     Ht.data_ptr() if Ht is not None else None, iters_done.data_ptr(),
                     status.data_ptr(), ws.data_ptr(), ws.numel(),
                     xdest.data_ptr() if xdest is not None else None,
                     Xs.data_ptr() if Xs is not None else None,
                     Vt.data_ptr() if Vt is not None else None)
    stream = torch.cuda.current_stream().cuda_stream
    _lib.check(lib.sbce_em(dims, ptrs, int(itera), _MODES[mode], _SOLVES[solve], stream), "sbce_em")
    out = dict(theta=th, llf=llf, status=status, iters_done=iters_done)
    if xdest is not None:
        out["x_dest"] = xdest
    if return_device:
        return out
    torch.cuda.current_stream().synchronize()
    return {k: (v.cpu().numpy() if v is not None else None) for k, v in out.items()}


def _prepare_single(Y_d, Y_p, Z_p, PsiTilde_td, all_possibleSymbols, M, h_initial, n_tx=None,
                    cons=None):
    n_rx = np.asarray(Y_d[0]).shape[0]
    aps = None if all_possibleSymbols is None else np.asarray(all_possibleSymbols)
    if aps is not None:
        n_tx = aps.shape[1]
        cons = cons_from_aps(aps, int(M)) if cons is None else np.asarray(cons, dtype=complex)
    else:
        cons = np.asarray(cons, dtype=complex).reshape(-1)
    Psi = np.asarray(PsiTilde_td)
    P = Psi.shape[0]
    K = P * n_tx * n_rx
    U_p = u_from_zp(Z_p, n_rx) if len(Z_p) else np.zeros((0, P * n_tx), dtype=complex)
    check_structure(Z_p, U_p, n_rx, aps, cons, K)
    y_d = np.stack([np.asarray(y).reshape(-1) for y in Y_d])[None]
    y_p = (np.stack([np.asarray(y).reshape(-1) for y in Y_p])[None] if len(Y_p)
           else np.zeros((1, 0, n_rx), dtype=complex))
    th0 = (np.zeros(K, dtype=complex) if h_initial is None
           else np.asarray(h_initial, dtype=complex).reshape(-1))
    if th0.size != K:
        raise ValueError(f"h_initial has {th0.size} entries, expected K={K}")
    return dict(y_d=y_d, y_p=y_p, psi_d=Psi.T[None], u_p=U_p[None], cons=cons,
                theta0=th0[None], n_tx=n_tx, n_rx=n_rx, P=P, K=K)


last_status = 0


def _finish(res, verbose, itera):
    global last_status
    last_status = int(res["status"][0])
    th = res["theta"][0].reshape(-1, 1)
    if verbose:
        print(np.linalg.norm(th))
    return th


def em(Y_d, Y_p, T_d, T_p, Z_p, PsiTilde_td, all_possibleSymbols, M, varn, itera, h_initial,
       verbose=False, solve="chol"):
    """Exact soft EM (PMd/Proposed_method_NMSEvsTp.py:50-83) on the GPU."""
    d = _prepare_single(Y_d[:T_d], Y_p[:T_p], Z_p[:T_p], np.asarray(PsiTilde_td)[:, :T_d],
                        all_possibleSymbols, M, h_initial)
    if verbose:
        print("inital theta", np.linalg.norm(d["theta0"]))
    res = em_batch(d["y_d"], d["y_p"], d["psi_d"], d["u_p"], d["cons"], varn, itera, d["theta0"],
                   mode="soft", solve=solve)
    return _finish(res, verbose, itera)


def em_ml(Y_d, Y_p, T_d, T_p, Z_p, PsiTilde_td, all_possibleSymbols, M, varn, itera, h_initial,
          verbose=False, solve="chol"):
    """Hard-ML ("log-max") EM (PMd/all_detectorsvsTd.py:135-173)."""
    d = _prepare_single(Y_d[:T_d], Y_p[:T_p], Z_p[:T_p], np.asarray(PsiTilde_td)[:, :T_d],
                        all_possibleSymbols, M, h_initial)
    res = em_batch(d["y_d"], d["y_p"], d["psi_d"], d["u_p"], d["cons"], varn, itera, d["theta0"],
                   mode="hard", solve=solve)
    return _finish(res, verbose, itera)


def _x_from_zd(Z_d, Psi, n_tx, n_rx):
    """True data symbols from the genie regressors Z_d[t] = (psi_t (x) x_t)^T (x) I."""
    U = u_from_zp(Z_d, n_rx)                          # (T, P*n_tx)
    P = Psi.shape[0]
    U3 = U.reshape(U.shape[0], P, n_tx)
    p0 = np.argmax(np.abs(Psi), axis=0)               # a non-zero phase per symbol
    t = np.arange(U.shape[0])
    return U3[t, p0, :] / Psi[p0, t][:, None]


def em_llf(Y_d, Y_p, T_d, T_p, Z_p, Z_d, PsiTilde_td, all_possibleSymbols, M, varn, itera,
           h_initial, n_tx, mode="soft"):
    """Soft EM + per-iteration LLF (PMd/IterationsvsLLF.py:45-77).
    Returns (theta (K,1), logLikelihood (itera,1))."""
    d = _prepare_single(Y_d[:T_d], Y_p[:T_p], Z_p[:T_p], np.asarray(PsiTilde_td)[:, :T_d],
                        all_possibleSymbols, M, h_initial)
    if d["n_tx"] != n_tx:
        raise ValueError("n_tx does not match all_possibleSymbols")
    xd = _x_from_zd(Z_d[:T_d], np.asarray(PsiTilde_td)[:, :T_d], n_tx, d["n_rx"])[None]
    res = em_batch(d["y_d"], d["y_p"], d["psi_d"], d["u_p"], d["cons"], varn, itera, d["theta0"],
                   mode=mode, x_d_true=xd)
    th = _finish(res, False, itera)
    return th, res["llf"][0].reshape(itera, 1)


def em_ml_llf(Y_d, Y_p, T_d, T_p, Z_p, PsiTilde_td, all_possibleSymbols, M, varn, itera,
              h_initial, Z_d):
    """Hard-ML EM + LLF (PMd/ML_detecctor.py:51-86; the reference reads Z_d as a
    module global, here it is an explicit argument)."""
    n_tx = np.asarray(all_possibleSymbols).shape[1]
    return em_llf(Y_d, Y_p, T_d, T_p, Z_p, Z_d, PsiTilde_td, all_possibleSymbols, M, varn, itera,
                  h_initial, n_tx, mode="hard")


def _pm(Y_d, Y_p, T_d, T_p, Z_p, PsiTilde_td, aps, M, varn, itera, h_initial, h, n_tx,
        partition_r, qamCons, mode, solve, verbose):
    cons = np.asarray(qamCons, dtype=complex).reshape(-1)
    if cons.size != int(M):
        raise ValueError("qamCons must hold the M constellation points")
    d = _prepare_single(Y_d[:T_d], Y_p[:T_p], Z_p[:T_p], np.asarray(PsiTilde_td)[:, :T_d], aps, M,
                        h_initial, n_tx=int(n_tx), cons=cons)
    if d["n_tx"] != int(n_tx):
        raise ValueError("n_tx does not match all_possibleSymbols")
    hh = None if h is None else np.asarray(h, dtype=complex).reshape(1, -1)
    res = em_batch(d["y_d"], d["y_p"], d["psi_d"], d["u_p"], cons, varn, itera, d["theta0"],
                   mode=mode, h_true=hh, solve=solve, partition_r=int(partition_r))
    return _finish(res, verbose, itera)


def em_pm(Y_d, Y_p, T_d, T_p, Z_p, PsiTilde_td, all_possibleSymbols, M, varn, itera, h_initial, h,
          n_tx, partition_r, X_d, qamCons, verbose=False, solve="lstsq"):
    """Partitioned list-detector EM, every list member weight 1 (PMd/PM.py:47-116).

    The list of M**(p+1) candidates (p = int(partition_r / log2 M)) is built per
    symbol from the reference's off-by-one channel (PM.py:63) with greedy stream
    ordering and per-element slicing of the B partition; the candidate vector is
    the concatenation [x_A, x_B] used in natural stream order (PM.py:101-104).
    ``h`` drives the reference's oracle early stop (PM.py:110-112) when given;
    ``X_d`` is accepted for signature parity (the reference only reads its
    length).  ``all_possibleSymbols`` may be None (n_tx = 8 makes it 4.3e9 rows).
    The reference solves with lstsq (PM.py:108): solve='lstsq' (default) is its device
    counterpart, the minimum-norm solution with lstsq's singular-value cut."""
    return _pm(Y_d, Y_p, T_d, T_p, Z_p, PsiTilde_td, all_possibleSymbols, M, varn, itera,
               h_initial, h, n_tx, partition_r, qamCons, "pm", solve, verbose)


def em_pm_soft(Y_d, Y_p, T_d, T_p, Z_p, PsiTilde_td, M, varn, itera, h_initial, h, n_tx,
               partition_r, X_d, qamCons, verbose=False, solve="chol"):
    """Partitioned list-detector EM with posterior list weights
    exp(-||y - H_t x||^2 / varn^2), normalised over the list (PMd/PM_beta.py:42-112;
    the same signature as PM_beta.em_pm, which takes no all_possibleSymbols)."""
    return _pm(Y_d, Y_p, T_d, T_p, Z_p, PsiTilde_td, None, M, varn, itera, h_initial, h, n_tx,
               partition_r, qamCons, "pm_soft", solve, verbose)


def _detector(Y_d, Y_p, T_d, T_p, Z_p, PsiTilde_td, all_possibleSymbols, M, varn, itera,
              h_initial, h, mode, solve, verbose):
    d = _prepare_single(Y_d[:T_d], Y_p[:T_p], Z_p[:T_p], np.asarray(PsiTilde_td)[:, :T_d],
                        all_possibleSymbols, M, h_initial)
    hh = None if h is None else np.asarray(h, dtype=complex).reshape(1, -1)
    res = em_batch(d["y_d"], d["y_p"], d["psi_d"], d["u_p"], d["cons"], varn, itera, d["theta0"],
                   mode=mode, h_true=hh, solve=solve)
    return _finish(res, verbose, itera)


def em_zf(Y_d, Y_p, T_d, T_p, Z_p, PsiTilde_td, all_possibleSymbols, M, varn, itera, h_initial, h,
          verbose=False, solve="chol"):
    """Zero-forcing detector EM (PMd/all_detectorsvsTd.py:98-133): per symbol
    z = pinv(H_off) y on the reference's off-by-one channel (:111), the flattened-argmin
    nearest_symbol_ecul decision (:49-52) as a weight-1 hypothesis, np.linalg.solve M-step,
    oracle early stop on h.  Where the reference's flat index runs past the hypothesis
    table (an IndexError there) the trial is flagged SBCE_STATUS_DETECTOR (last_status)."""
    return _detector(Y_d, Y_p, T_d, T_p, Z_p, PsiTilde_td, all_possibleSymbols, M, varn, itera,
                     h_initial, h, "zf", solve, verbose)


def em_mmse(Y_d, Y_p, T_d, T_p, Z_p, PsiTilde_td, all_possibleSymbols, M, varn, itera, h_initial,
            h, verbose=False, solve="chol"):
    """MMSE detector EM (PMd/all_detectorsvsTd.py:54-96): z = (H^H H + varn^2 I)^{-1} H^H y
    (:71), otherwise as em_zf.  (The reference's per-iteration LLF there reads a global
    Z_d and is never returned; it is not part of the result.)"""
    return _detector(Y_d, Y_p, T_d, T_p, Z_p, PsiTilde_td, all_possibleSymbols, M, varn, itera,
                     h_initial, h, "mmse", solve, verbose)


def em_ml_ser(Y_d, Y_p, T_d, T_p, Z_p, PsiTilde_td, all_possibleSymbols, M, varn, itera,
              h_initial, verbose=False, solve="chol"):
    """Log-max EM of PMd/SER/log_max_SER.py:51-84: returns (theta (K,1), X_dest) with
    X_dest the list of (1, n_tx) argmax decisions of the last iteration (:77-78)."""
    d = _prepare_single(Y_d[:T_d], Y_p[:T_p], Z_p[:T_p], np.asarray(PsiTilde_td)[:, :T_d],
                        all_possibleSymbols, M, h_initial)
    res = em_batch(d["y_d"], d["y_p"], d["psi_d"], d["u_p"], d["cons"], varn, itera, d["theta0"],
                   mode="hard", solve=solve, return_decisions=True)
    th = _finish(res, verbose, itera)
    return th, [x[None, :] for x in res["x_dest"][0]]


def em_superimposed(Y, T, Z, X_d, X_p, T_p, T_d, n_tx, PsiTilde_t, all_possibleSymbols, M, varn,
                    itera, N, verbose=False, solve="chol"):
    """Superimposed-pilot EM (Parallel/ParallelProtocol_Tp.py:63-86, same signature):
    T = max(T_d, T_p) symbols y_t carrying x_d,t + x_p,t (both zero-padded), soft
    posterior over x_j + x_p,t, no separate pilot block, theta_0 = 0.  Z is accepted for
    signature parity (the reference only passes it through)."""
    aps = np.asarray(all_possibleSymbols)
    n_tx = aps.shape[1]
    Psi = np.asarray(PsiTilde_t)[:, :T]
    n_rx = np.asarray(Y[0]).shape[0]
    Xp = np.zeros((T, n_tx), dtype=complex)
    xp = np.stack([np.asarray(x).reshape(-1) for x in X_p]) if len(X_p) else Xp[:0]
    Xp[:min(T, xp.shape[0])] = xp[:T]
    L = Psi.shape[0] * n_tx
    y = np.stack([np.asarray(v).reshape(-1) for v in Y[:T]])[None]
    res = em_batch(y, np.zeros((1, 0, n_rx), dtype=complex), Psi.T[None],
                   np.zeros((1, 0, L), dtype=complex), cons_from_aps(aps, int(M)), varn, itera,
                   np.zeros((1, L * n_rx), dtype=complex), mode="soft", solve=solve,
                   x_sup=Xp[None])
    return _finish(res, verbose, itera)


_GAUSS_CONS = np.array([1.0 + 0j, -1.0 + 0j])      # placeholder table: the Gaussian E-step has none


def gauss_expand_batch(theta, n_tx, n_rx, return_device=False):
    """The reference's n_rx x (N n_tx n_rx^2) channel matrix H_l (MIMO_Gaussian_proposed.py:
    77-85) from reduced Gaussian-EM estimates theta (B, N n_tx n_rx), on the device
    (sbce_gauss_expand)."""
    torch = _torch()
    lib = _lib.load()
    th = theta if isinstance(theta, torch.Tensor) else _dev(torch, theta, np.complex128)
    th = th.contiguous()
    B, K = th.shape
    P = K // (n_tx * n_rx)
    Q = P * n_tx * n_rx * n_rx
    dims = _lib.Dims(B, n_tx, n_rx, P, 0, 1, 2, 0, 1.0, 1.0)
    out = torch.empty((B, n_rx, Q), dtype=torch.complex128, device="cuda")
    _lib.check(lib.sbce_gauss_expand(dims, th.data_ptr(), out.data_ptr(),
                                     torch.cuda.current_stream().cuda_stream), "sbce_gauss_expand")
    if return_device:
        return out
    return out.cpu().numpy()


def gaussian_regressors(z_p, N, n_tx, n_rx):
    """u_p = psi_p (x) x_p from the reference's z_p = vec(kron(u_p^T, I_{n_rx})) =
    u_p (x) vec(I_{n_rx}) (received_proposed :126); raises if z_p has another structure."""
    L = N * n_tx
    e = np.eye(n_rx).flatten(order="F")
    if not len(z_p):
        return np.zeros((0, L), dtype=complex)
    Z = np.stack([np.asarray(z).reshape(-1) for z in z_p])
    if Z.shape[1] != L * n_rx * n_rx:
        raise ValueError(f"z_p has {Z.shape[1]} rows, expected N n_tx n_rx^2 = {L * n_rx * n_rx}")
    U = Z[:, ::n_rx * n_rx]                           # first vec(I) entry of each block (= 1)
    if not np.allclose(Z, np.einsum("tl,i->tli", U, e).reshape(Z.shape), rtol=1e-12, atol=0):
        raise ValueError("z_p is not kron(psi_p (x) x_p, vec(I_n_rx)) (received_proposed :126)")
    return U


def reduce_gaussian_channel(H, n_tx, n_rx):
    """Reduced channel theta[c n_rx + r] = H[r, c n_rx^2 : (c+1) n_rx^2] . vec(I): the only
    part of H the Gaussian E-step sees (H Sigma_t, Sigma_t = kron(., e e^H))."""
    H = np.asarray(H, dtype=complex)
    Lr = H.shape[1] // (n_rx * n_rx)
    Hr = np.einsum("rcjj->rc", H.reshape(n_rx, Lr, n_rx, n_rx))
    return Hr.T.reshape(-1)


last_gaussian_reduced = None


def EM_Gaussian_proposed(y_d, y_p, T_d, T_p, z_p, PsiTilde_td, varn, itera, H_initial, varx,
                         n_tx, verbose=False, solve="drop"):
    """Gaussian-prior EM (Proposed method/MIMO_Gaussian_proposed.py:56-89, same signature):
    x ~ CN(0, varx I) with the reference's prior covariance varx^2 kron(kron(psi psi^H, I),
    vec(I) vec(I)^H) (:33-45), itera + 1 iterations (``while j <= itera``), returns the
    n_rx x (N n_tx n_rx^2) matrix H_l.  The device runs the reduced form (include/sbce.h,
    SBCE_ESTEP_GAUSS / sbce_gauss_expand).  The reference's M-step inverse is the lstsq
    pseudo-inverse (:47-53), so the default solve is the pivot-dropping Cholesky ("drop"),
    identical to the plain inverse whenever the reduced G is well conditioned.  (At the
    script's own defaults the reference iteration diverges after one step, NMSE ~1e6 and
    growing; past that point neither its output nor this one is numerically meaningful.)"""
    global last_gaussian_reduced
    Psi = np.asarray(PsiTilde_td)[:, :T_d]
    N = Psi.shape[0]
    n_rx = np.asarray(y_d[0]).shape[0]
    U_p = gaussian_regressors(z_p[:T_p], N, n_tx, n_rx)
    yd = np.stack([np.asarray(v).reshape(-1) for v in y_d[:T_d]])[None]
    yp = (np.stack([np.asarray(v).reshape(-1) for v in y_p[:T_p]])[None] if T_p
          else np.zeros((1, 0, n_rx), dtype=complex))
    th0 = reduce_gaussian_channel(H_initial, n_tx, n_rx)[None]
    res = em_batch(yd, yp, Psi.T[None], U_p[None], _GAUSS_CONS, varn, int(itera) + 1, th0,
                   mode="gauss", solve=solve, varx=varx, return_device=True)
    torch = _torch()
    global last_status
    last_status = int(res["status"][0].item())
    last_gaussian_reduced = res["theta"][0].cpu().numpy()
    H = gauss_expand_batch(res["theta"], n_tx, n_rx)[0]
    if verbose:
        print(np.linalg.norm(H))
    torch.cuda.current_stream().synchronize()
    return H


def ser_batch(x_dest, x_d_true):
    """Per-trial SER on the device (sbce_ser): (ser_reference, ser_elementwise), the first
    being the expression of PMd/SER/log_max_SER.py:162."""
    torch = _torch()
    lib = _lib.load()
    xd = x_dest if isinstance(x_dest, torch.Tensor) else _dev(torch, x_dest, np.complex128)
    xt = x_d_true if isinstance(x_d_true, torch.Tensor) else _dev(torch, x_d_true, np.complex128)
    B, T_d, n_tx = xd.shape
    dims = _lib.Dims(B, n_tx, 1, 1, 0, T_d, 2, 0, 1.0)
    out = torch.zeros((B, 2), dtype=torch.float64, device="cuda")
    _lib.check(lib.sbce_ser(dims, xd.contiguous().data_ptr(), xt.contiguous().data_ptr(),
                            out.data_ptr(), torch.cuda.current_stream().cuda_stream), "sbce_ser")
    out = out.cpu().numpy()
    return out[:, 0], out[:, 1]


def em_zero_init(Y_d, Y_p, T_d, T_p, Z_p, PsiTilde_td, all_possibleSymbols, M, varn, itera):
    """Root-level em() (Proposed_method_NMSEvsTp.py:43-69): theta_0 = 0."""
    return em(Y_d, Y_p, T_d, T_p, Z_p, PsiTilde_td, all_possibleSymbols, M, varn, itera, None)


# ------------------------------------------------------------------ diagnostic stages
def _stage_setup(torch, y_d, y_p, psi_d, u_p, cons, theta, varn, partition_r=0, varx=1.0,
                 workspace=True):
    def dev(x):
        return _dev(torch, x, np.complex128)
    Yd, Yp, Ps, Up, Cs, Th = (dev(y_d), dev(y_p), dev(psi_d), dev(u_p), dev(cons), dev(theta))
    B, T_d, n_rx = Yd.shape
    T_p, P, L = Yp.shape[1], Ps.shape[2], Up.shape[2]
    n_tx = L // P
    dims = _lib.Dims(B, n_tx, n_rx, P, T_p, T_d, Cs.shape[0], int(partition_r), float(varn),
                     float(varx))
    ws = torch.empty(max(_lib.workspace_bytes(dims), 16), dtype=torch.uint8, device="cuda")
    status = torch.zeros(B, dtype=torch.int32, device="cuda")
    ptrs = _lib.Ptrs(Yd.data_ptr(), Yp.data_ptr() if T_p else Yd.data_ptr(), Ps.data_ptr(),
                     Up.data_ptr() if T_p else Yd.data_ptr(), Cs.data_ptr(), Th.data_ptr(), None,
                     None, None, None, status.data_ptr(), ws.data_ptr() if workspace else None,
                     ws.numel() if workspace else 0)
    keep = (Yd, Yp, Ps, Up, Cs, Th, ws, status)
    return dims, ptrs, keep


def estep_batch(y_d, psi_d, cons, theta, varn, n_tx, mode="soft", partition_r=0, varx=1.0,
                workspace=True):
    """One device E-step (sbce_estep): returns m (B,T_d,n_tx), S (B,T_d,n_tx,n_tx).
    workspace=False passes no workspace (the exact sweep then prepares each symbol in
    its own kernel instead of the separate preparation pass)."""
    torch = _torch()
    lib = _lib.load()
    B, T_d, n_rx = np.shape(y_d)
    P = np.shape(psi_d)[2]
    y_p = np.zeros((B, 0, n_rx), dtype=complex)
    u_p = np.zeros((B, 0, P * n_tx), dtype=complex)
    dims, ptrs, keep = _stage_setup(torch, y_d, y_p, psi_d, u_p, cons, theta, varn, partition_r,
                                    varx, workspace)
    mom = torch.zeros((B, T_d, n_tx + n_tx * n_tx), dtype=torch.complex128, device="cuda")
    stream = torch.cuda.current_stream().cuda_stream
    _lib.check(lib.sbce_estep(dims, ptrs, _MODES[mode], mom.data_ptr(), stream), "sbce_estep")
    torch.cuda.current_stream().synchronize()
    mom = mom.cpu().numpy()
    return mom[..., :n_tx], mom[..., n_tx:].reshape(B, T_d, n_tx, n_tx)


def mstep_batch(y_d, y_p, psi_d, u_p, cons, m, S, varn, solve="chol", return_tol=False,
                ws_fill=None):
    """One device M-step (sbce_mstep) from given moments: returns theta (B,K),
    R (B,L,L), rhs (B,L,n_rx), status (B,) [, tol (B,): the min-norm pivot threshold
    32 eps K lambda_max(R) (sbce_debug_minnorm_tol), return_tol=True with solve='lstsq'].
    ws_fill: a byte value the workspace is filled with first (tests: results must not
    depend on what a workspace held)."""
    torch = _torch()
    lib = _lib.load()
    B, T_d, n_rx = np.shape(y_d)
    L = np.shape(u_p)[2]
    n_tx = np.shape(m)[2]
    theta = np.zeros((B, L * n_rx), dtype=complex)
    dims, ptrs, keep = _stage_setup(torch, y_d, y_p, psi_d, u_p, cons, theta, varn)
    if ws_fill is not None:
        keep[6].fill_(int(ws_fill))
    mom = np.concatenate([np.asarray(m).reshape(B, T_d, n_tx),
                          np.asarray(S).reshape(B, T_d, n_tx * n_tx)], axis=2)
    Mo = _dev(torch, mom, np.complex128)
    R = torch.zeros((B, L, L), dtype=torch.complex128, device="cuda")
    rhs = torch.zeros((B, L, n_rx), dtype=torch.complex128, device="cuda")
    stream = torch.cuda.current_stream().cuda_stream
    _lib.check(lib.sbce_mstep(dims, ptrs, Mo.data_ptr(), _SOLVES[solve], R.data_ptr(),
                              rhs.data_ptr(), stream), "sbce_mstep")
    tol = None
    if return_tol:
        tol = np.zeros(B)
        fn = lib.sbce_debug_minnorm_tol
        fn.restype = ctypes.c_int
        torch.cuda.current_stream().synchronize()
        _lib.check(fn(ctypes.byref(dims), ctypes.byref(ptrs), tol.ctypes.data_as(ctypes.c_void_p),
                      ctypes.c_void_p(stream)), "sbce_debug_minnorm_tol")
    torch.cuda.current_stream().synchronize()
    th = keep[5].cpu().numpy()
    # the device keeps only R's lower triangle (its strict upper part is factorisation
    # workspace): return the Hermitian completion
    R = np.tril(R.cpu().numpy())
    R = R + np.conj(np.swapaxes(np.tril(R, -1), 1, 2))
    out = (th, R, rhs.cpu().numpy(), keep[7].cpu().numpy())
    return out + (tol,) if return_tol else out


def nmse_batch(theta, h):
    """Per-trial NMSE on the device (sbce_nmse), PMd/Proposed_method_NMSEvsTp.py:172."""
    torch = _torch()
    lib = _lib.load()
    th = theta if isinstance(theta, torch.Tensor) else _dev(torch, theta, np.complex128)
    hh = h if isinstance(h, torch.Tensor) else _dev(torch, h, np.complex128)
    B, K = th.shape
    dims = _lib.Dims(B, 1, 1, K, 0, 1, 2, 0, 1.0)   # only batch and K = n_psi*n_tx*n_rx matter
    out = torch.zeros(B, dtype=torch.float64, device="cuda")
    _lib.check(lib.sbce_nmse(dims, th.data_ptr(), hh.data_ptr(), out.data_ptr(),
                             torch.cuda.current_stream().cuda_stream), "sbce_nmse")
    return out


class EMEngine:
    """Pre-allocated device state for repeated batched EM runs (benchmark / sweeps).

    All buffers (observations, phases, pilot regressors, theta, workspace) stay
    resident in HBM; ``run()`` resets theta from theta0 with a device copy and
    issues ONE sbce_em call on the current stream.  Nothing is allocated or
    synchronised inside ``run()``.

    ``streams = K > 1``: ``run()`` issues the batch as K contiguous sub-batches, one sbce_em
    call each on its own HIP stream (forked from and joined back into the current stream).
    Trials are independent and every kernel treats them independently, so theta is bitwise
    the same; the sub-batches' kernels overlap -- the latency-bound launches of one (the
    Cholesky panel factors, the enumeration tail) run beside the MFMA-bound ones of another.
    Each sub-batch has its own workspace (its work lists and counters are per call); the
    inputs, theta and status are views of the whole-batch tensors.  ``estep()``, ``mstep()``
    and ``mstep_phase()`` (kernel timing) stay whole-batch launches.
    """

    def __init__(self, batch, varn, mode="soft", solve="chol", x_d_true=None, h_true=None,
                 partition_r=0, varx=1.0, x_sup=None, streams=1, early_stop=False):
        """early_stop=True: the reference's oracle early stop on the true channel (PM.py:110-112,
        all_detectorsvsTd.py's five EMs) with h_true (or batch["h"]); ``iters_done`` then holds
        the iterations each trial of the last run() performed."""
        torch = _torch()
        self.torch = torch

        def dev(x):
            if x is None:
                return None
            if isinstance(x, torch.Tensor):
                return x.to("cuda").contiguous()
            return _dev(torch, x, np.complex128)

        self.y_d, self.y_p = dev(batch["y_d"]), dev(batch["y_p"])
        self.psi_d, self.u_p = dev(batch["psi_d"]), dev(batch["u_p"])
        self.cons, self.theta0 = dev(batch["cons"]), dev(batch["theta0"])
        self.h = dev(h_true if h_true is not None else batch.get("h"))
        self.theta = self.theta0.clone()
        B, T_d, n_rx = self.y_d.shape
        T_p, P, L = self.y_p.shape[1], self.psi_d.shape[2], self.u_p.shape[2]
        self.n_tx, self.n_rx, self.B, self.T_d, self.T_p, self.P = L // P, n_rx, B, T_d, T_p, P
        self.M = self.cons.shape[0]
        # one noise variance, or one per trial (the SNR axis of a sweep batched into one call)
        self.varn, self.varn_t = _varn_arg(torch, varn, B)
        if mode == "gauss" and not varx > 0:
            raise ValueError("mode 'gauss' needs a prior variance varx > 0")
        if x_sup is not None and mode not in ("soft", "hard"):
            raise ValueError("superimposed pilots (x_sup) need the soft or hard E-step")
        self.dims = _lib.Dims(B, self.n_tx, n_rx, P, T_p, T_d, self.M, int(partition_r), self.varn,
                              float(varx))
        self.mode, self.solve = _MODES[mode], _SOLVES[solve]
        # ONE device buffer: the whole-batch workspace (estep / mstep / mstep_phase) and, when the
        # batch runs as stream sub-batches, their workspaces as disjoint slices of the same memory
        # (run() and the whole-batch diagnostics are never in flight together)
        K = int(streams)
        sub = K > 1 and B >= 2 * K and T_p and x_sup is None
        bounds = np.linspace(0, B, K + 1).astype(int) if sub else np.array([0, B])
        sub_dims = [_lib.Dims(int(b1 - b0), self.n_tx, n_rx, P, T_p, T_d, self.M, int(partition_r),
                              self.varn, float(varx)) for b0, b1 in zip(bounds[:-1], bounds[1:])]
        sub_bytes = [(_lib.workspace_bytes(d, self.solve) + 255) // 256 * 256 for d in sub_dims]
        whole = _lib.workspace_bytes(self.dims, self.solve)
        self.ws_all = torch.empty(max(whole, sum(sub_bytes) if sub else 0, 16), dtype=torch.uint8,
                                  device="cuda")
        self.ws = self.ws_all[:max(whole, 16)]
        self.status = torch.zeros(B, dtype=torch.int32, device="cuda")
        self.x_d = dev(x_d_true)
        self.mom = torch.zeros((B, T_d, self.n_tx + self.n_tx ** 2), dtype=torch.complex128,
                               device="cuda")
        self.x_sup = dev(x_sup)
        # T_p == 0 (superimposed protocol): an empty tensor's data_ptr() is 0, which the ABI
        # rejects; the pilot buffers are never read then, so pass y_d as a placeholder (em_batch)
        yp = self.y_p.data_ptr() if T_p else self.y_d.data_ptr()
        up = self.u_p.data_ptr() if T_p else self.y_d.data_ptr()
        if early_stop and self.h is None:
            raise ValueError("early_stop needs the true channel (h_true or batch['h'])")
        self.early_stop = bool(early_stop)
        self.iters_done = torch.zeros(B, dtype=torch.int32, device="cuda")
        hp = self.h.data_ptr() if self.early_stop else None
        self.ptrs = _lib.Ptrs(self.y_d.data_ptr(), yp, self.psi_d.data_ptr(), up,
                              self.cons.data_ptr(), self.theta.data_ptr(), None, None, hp,
                              self.iters_done.data_ptr(), self.status.data_ptr(), self.ws.data_ptr(),
                              self.ws.numel(), None,
                              self.x_sup.data_ptr() if self.x_sup is not None else None,
                              self.varn_t.data_ptr() if self.varn_t is not None else None)
        self.subs = []
        self._minnorm_ws = False        # the workspace holds a whole-batch min-norm M-step
        if sub:
            off = 0
            for (b0, b1), dims, nb in zip(zip(bounds[:-1], bounds[1:]), sub_dims, sub_bytes):
                ws = self.ws_all[off:off + nb]
                off += nb
                ptrs = _lib.Ptrs(self.y_d[b0:b1].data_ptr(), self.y_p[b0:b1].data_ptr(),
                                 self.psi_d[b0:b1].data_ptr(), self.u_p[b0:b1].data_ptr(),
                                 self.cons.data_ptr(), self.theta[b0:b1].data_ptr(), None, None,
                                 self.h[b0:b1].data_ptr() if self.early_stop else None,
                                 self.iters_done[b0:b1].data_ptr(), self.status[b0:b1].data_ptr(),
                                 ws.data_ptr(), ws.numel(), None, None,
                                 self.varn_t[b0:b1].data_ptr() if self.varn_t is not None else None)
                self.subs.append((dims, ptrs, ws, torch.cuda.Stream()))

    def run(self, itera, stream=None):
        """One full EM (itera iterations) over the whole batch, stream-ordered on `stream`
        (default: the current stream)."""
        # with stream sub-batches the workspace holds their layouts, not the whole batch's
        self._minnorm_ws = not self.subs and self.solve == _lib.SBCE_SOLVE_MINNORM
        cur = self.torch.cuda.current_stream() if stream is None else stream
        with self.torch.cuda.stream(cur):
            self.theta.copy_(self.theta0)
        if not self.subs:
            rc = self.lib.sbce_em(self.dims, self.ptrs, int(itera), self.mode, self.solve,
                                  cur.cuda_stream)
            _lib.check(rc, "sbce_em")
            return self.theta
        ev = self.torch.cuda.Event()
        ev.record(cur)
        for dims, ptrs, _, st in self.subs:
            st.wait_event(ev)
            _lib.check(self.lib.sbce_em(dims, ptrs, int(itera), self.mode, self.solve, st.cuda_stream),
                       "sbce_em")
        for _, _, _, st in self.subs:
            cur.wait_stream(st)
        return self.theta

    def capture(self, itera, stream=None):
        """run(itera) captured as ONE HIP graph (stream capture through torch.cuda.CUDAGraph; the
        library's launches on the capturing stream are recorded like torch's own).  sbce_em's
        launch sequence is fixed by the shapes -- the early stop and the sphere pass's work lists
        are device-side -- so ``graph.replay()`` (on the current stream) reruns the whole EM on
        this engine's buffers: one host launch instead of ~4 per iteration, for the sweep grids'
        many small calls, which are host-launch-bound otherwise.  Call run() once before (the
        first launch of each kernel loads its code object)."""
        torch = self.torch
        g = torch.cuda.CUDAGraph()
        side = stream if stream is not None else torch.cuda.Stream()
        side.wait_stream(torch.cuda.current_stream())
        with torch.cuda.graph(g, stream=side):
            self.run(itera)
        torch.cuda.current_stream().wait_stream(side)
        return g

    def estep(self):
        """One E-step launch over the batch from the current theta (for kernel timing)."""
        rc = self.lib.sbce_estep(self.dims, self.ptrs, self.mode, self.mom.data_ptr(),
                                 self.torch.cuda.current_stream().cuda_stream)
        _lib.check(rc, "sbce_estep")

    def mstep(self):
        """One M-step launch sequence from the last E-step moments (for kernel timing)."""
        rc = self.lib.sbce_mstep(self.dims, self.ptrs, self.mom.data_ptr(), self.solve, None,
                                 None, self.torch.cuda.current_stream().cuda_stream)
        _lib.check(rc, "sbce_mstep")
        self._minnorm_ws = self.solve == _lib.SBCE_SOLVE_MINNORM

    @property
    def lib(self):
        """libsbce.so -- or libsbce_ab.so inside _lib.debug_env() (A/B and counter runs on the
        same device state: one C-ABI, the workspace carve is the same code)."""
        return _lib.load()

    def mstep_phase(self, phase):
        """One piece of the M-step from the last moments (kernel timing, sbce_debug_mstep_phase):
        0 pilot factorisation, 1 the R build kernel alone, 2 R and B^H."""
        self._minnorm_ws = False                       # R (where G lives) is rebuilt
        fn = self.lib.sbce_debug_mstep_phase
        fn.restype = ctypes.c_int
        rc = fn(ctypes.byref(self.dims), ctypes.byref(self.ptrs), ctypes.c_void_p(self.mom.data_ptr()),
                int(phase), ctypes.c_void_p(self.torch.cuda.current_stream().cuda_stream))
        _lib.check(rc, "sbce_debug_mstep_phase")

    def nmse(self):
        """Per-trial NMSE of the current theta against h (device, sbce_nmse)."""
        return nmse_batch(self.theta, self.h)

    def minnorm_rank(self):
        """(B, 3) int32: active extent, rank of G and whether the refinement step ran, of the
        last whole-batch min-norm M-step (sbce_debug_minnorm_rank; solve='lstsq' only)."""
        if not self._minnorm_ws:
            raise RuntimeError("minnorm_rank: the workspace does not hold a whole-batch min-norm "
                               "M-step (call mstep() with solve='lstsq' first; a streamed run() or "
                               "mstep_phase() overwrites it)")
        out = self.torch.zeros((self.B, 3), dtype=self.torch.int32, device="cuda")
        fn = self.lib.sbce_debug_minnorm_rank
        fn.restype = ctypes.c_int
        rc = fn(ctypes.byref(self.dims), ctypes.byref(self.ptrs), ctypes.c_void_p(out.data_ptr()),
                ctypes.c_void_p(self.torch.cuda.current_stream().cuda_stream))
        _lib.check(rc, "sbce_debug_minnorm_rank")
        return out.cpu().numpy()
