/*
 * sbce.h — C-ABI of libsbce.so, the MI355X-native EM semi-blind channel
 * estimator for the MIMO-RIS cascaded channel.
 *
 * Drop-in boundary.  The reference has no native code: its
 * operator is the Python function
 *     em(Y_d, Y_p, T_d, T_p, Z_p, PsiTilde_td, all_possibleSymbols, M, varn,
 *        itera, h_initial) -> theta (K,1) complex128
 * ("Proposed method/Proposed_method_NMSEvsTp.py":50-83, called at :165; same
 * contract at "Proposed method/Proposed_method_NMSEvsTd.py":44/150 and
 * "Proposed method/SNR/all_Detectors.py":242/377).  The build's Python shim
 * (package em.py) keeps that signature, stacks the per-symbol lists into
 * batch-major device buffers and calls sbce_em() through ctypes.  Every entry
 * point below is what that ctypes binding declares.
 *
 * Conventions
 *   - complex numbers are interleaved float64 pairs (re, im), i.e. numpy
 *     complex128 / torch.complex128 memory;
 *   - every pointer in sbce_ptrs is a DEVICE pointer owned by the caller
 *     (e.g. torch.empty(..., device="cuda").data_ptr()); the library never
 *     allocates, keeps no global state and never synchronises the stream;
 *   - all work is stream-ordered on `hip_stream` (a hipStream_t, 0 = default);
 *   - return value 0 on success, a negative SBCE_E* code otherwise; nothing
 *     throws across the ABI.  Per-trial numerical status goes to ptrs->status.
 *
 * Batch-major layouts (B = dims.batch, P = dims.n_psi = N+1 with the direct
 * path, L = P*n_tx, K = L*n_rx):
 *   y_d      [B][T_d][n_rx]          data observations   (reference Y_d list)
 *   y_p      [B][T_p][n_rx]          pilot observations  (reference Y_p list)
 *   psi_d    [B][T_d][P]             RIS phases, TRANSPOSED reference
 *                                    PsiTilde_td ((N+1) x T_d, row 0 = direct)
 *   u_p      [B][T_p][L]             pilot regressors u_p = psi_p (x) x_p, i.e.
 *                                    Z_p[t] = u_p^T (x) I_{n_rx}
 *   cons     [M]                     constellation, table order of
 *                                    all_possibleSymbols' last column
 *   theta    [B][K]                  in: h_initial, out: estimate; reference
 *                                    vec order theta[(p*n_tx+a)*n_rx + r]
 *   x_d_true [B][T_d][n_tx]          optional (LLF genie term)
 *   llf      [B][iters] float64      optional output (IterationsvsLLF.py:76)
 *   h_true   [B][K]                  optional: enables the reference's oracle
 *                                    early stop (PM.py:110-112)
 *   iters_done [B] int32             optional output: iterations performed
 *   status   [B] int32               per-trial flags (SBCE_STATUS_*)
 *   x_dest   [B][T_d][n_tx]          optional output: last-iteration decisions
 *   x_sup    [B][T_d][n_tx]          optional superimposed pilot symbols
 *   varn_t   [B] float64             optional per-trial noise variances (ABI 6)
 */
#ifndef SBCE_H_
#define SBCE_H_

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define SBCE_ABI_VERSION 6

/* return codes */
#define SBCE_OK 0
#define SBCE_EINVAL (-1)        /* bad dims / null pointer / misaligned */
#define SBCE_EUNSUPPORTED (-2)  /* shape outside the compiled kernel set */
#define SBCE_EHIP (-3)          /* a HIP launch failed */
#define SBCE_EWORKSPACE (-4)    /* workspace too small */

/* E-step modes */
#define SBCE_ESTEP_SOFT 0       /* exact posterior over all M^n_tx hypotheses:
                                   Proposed_method_NMSEvsTp.py:61-71 */
#define SBCE_ESTEP_HARD 1       /* argmax posterior ("log-max"):
                                   ML_detecctor.py:65-77 */
#define SBCE_ESTEP_PM 2         /* partitioned list detector, every list member
                                   weight 1: PM.py:57-104 (dims.partition_r) */
#define SBCE_ESTEP_PM_SOFT 3    /* partitioned list detector, posterior list
                                   weights: PM_beta.py:55-95 (dims.partition_r) */
#define SBCE_ESTEP_ZF 4         /* zero-forcing hard decision (n_rx >= n_tx):
                                   all_detectorsvsTd.py:98-133 */
#define SBCE_ESTEP_MMSE 5       /* MMSE hard decision: all_detectorsvsTd.py:54-96 */
#define SBCE_ESTEP_GAUSS 6      /* Gaussian-prior EM (x ~ CN(0, varx^2 I), no constellation):
                                   MIMO_Gaussian_proposed.py:56-89.  m_t = LMMSE mean, S_t = the
                                   posterior covariance WITHOUT m m^H (the reference adds the
                                   scalar ||mu_t||^2 to every entry instead, :73-75; for n_rx = 1
                                   that term is kept as R += c 1 1^T, for n_rx >= 2 it cancels
                                   in the pseudo-inverse, see sbce_gauss_expand).  P = N rows of
                                   psi (no direct path); dims.varx used; cons ignored */

/* M-step solve modes (SURVEY.md §7 hard part 3) */
#define SBCE_SOLVE_CHOL 0       /* Hermitian Cholesky of the reduced L x L system
                                   (== LU of the K x K reference system,
                                   Proposed_method_NMSEvsTp.py:80, on HPD R).  A pivot
                                   <= 1e-14 max diag R (R not numerically HPD: rank-deficient
                                   when T_p + n_tx T_d < L) sets SBCE_STATUS_NONHPD and its
                                   direction is dropped: theta stays finite, solves the normal
                                   equations, and its range-space part is lstsq's minimum-norm
                                   solution (the reference's LU returns rounding noise there) */
#define SBCE_SOLVE_CHOL_DROP 1  /* the same solve (kept for ABI 1-6 callers): non-HPD pivots
                                   dropped, a basic solution on the kept coordinates, NOT
                                   minimum-norm */
#define SBCE_SOLVE_MINNORM 2    /* minimum-norm least squares, np.linalg.lstsq of PM.py:108
                                   (the intended fallback of all_detectorsvsTd.py:238-241):
                                   R's rank is cut at eps*K*lambda_max(R) (lstsq's default
                                   rcond = eps*max(K,K) on the K x K system, whose singular
                                   values are R's eigenvalues), lambda_max by 4 Lanczos steps;
                                   R = G G^H by a Cholesky that drops the pivots below 32x the
                                   cut (above its rounding noise), theta = conj(G (G^H G)^-2
                                   G^H B^H).  Equal to lstsq when no pivot lies between 4x the
                                   cut and 2048x it (else SBCE_STATUS_RANK) and no eigenvalue
                                   of R lies just below the cut */

/* per-trial status bits */
#define SBCE_STATUS_NONHPD 1
#define SBCE_STATUS_PILOT 2     /* n_tx in {4, 8}: u_p is not a Kronecker product
                                   psi_p (x) x_p (PM.py:119-130), so the MFMA build's
                                   factored pilot term does not apply; R of the trial is
                                   rebuilt by the general (VALU) path (informational) */
#define SBCE_STATUS_DETECTOR 4  /* ZF/MMSE: the reference's flattened argmin indexed past
                                   all_possibleSymbols (IndexError at
                                   all_detectorsvsTd.py:52); row flat mod M^n_tx used */
#define SBCE_STATUS_DEBUG 8     /* a diagnostic phase-skip mask (sbce_debug_chol_skip, not
                                   part of this header's API) or a non-default kernel selected
                                   by an SBCE_* debug environment variable was active */
#define SBCE_STATUS_RANK 16     /* SBCE_SOLVE_MINNORM: a Cholesky pivot lay between 4x lstsq's
                                   rank cut and 2048x it, where the pivot-based rank may differ
                                   from the singular-value rank np.linalg.lstsq uses */

typedef struct sbce_dims {
    int32_t batch;      /* B: independent Monte-Carlo trials */
    int32_t n_tx;       /* streams (1..4 exact/hard E-step, 1..8 PM/ZF/MMSE E-steps) */
    int32_t n_rx;       /* receive antennas (1..8) */
    int32_t n_psi;      /* P = rows of PsiTilde_td (N+1 with the direct path) */
    int32_t t_p;        /* pilot symbols */
    int32_t t_d;        /* data symbols */
    int32_t m;          /* constellation size (power of two, 2..64) */
    int32_t partition_r;/* PM modes: list = M^(p+1) with p = int(partition_r /
                           log2 M) (PM.py:74), at most 64 members; else 0 */
    double varn;        /* noise variance parameter; posterior uses varn^2 */
    double varx;        /* SBCE_ESTEP_GAUSS only: symbol variance parameter, the prior
                           covariance uses varx^2 (MIMO_Gaussian_proposed.py:44); else ignored */
} sbce_dims;

typedef struct sbce_ptrs {
    const void* y_d;
    const void* y_p;
    const void* psi_d;
    const void* u_p;
    const void* cons;
    void* theta;
    const void* x_d_true;   /* may be NULL */
    double* llf;            /* may be NULL (requires x_d_true) */
    const void* h_true;     /* may be NULL */
    int32_t* iters_done;    /* may be NULL */
    int32_t* status;        /* may be NULL */
    void* workspace;
    size_t workspace_bytes;
    void* x_dest;           /* may be NULL; hard E-step modes only (HARD/ZF/MMSE):
                               [B][T_d][n_tx] decisions of the last E-step
                               (SER/log_max_SER.py:77-78) */
    const void* x_sup;      /* may be NULL; SOFT/HARD only: [B][T_d][n_tx] pilot
                               symbols superimposed on the data, hypotheses x_j + x_sup[t]
                               (Parallel/ParallelProtocol_Tp.py:63-86; t_p is then 0) */
    const double* varn_t;   /* may be NULL (ABI 6): [B] noise variance parameter of each trial,
                               used instead of dims.varn (which must still be > 0) by the E-step
                               posterior (varn^2) and the LLF.  Lets one call carry the trials of
                               several SNR points of a sweep (all_detectorsvsTd.py's grid, SNR/
                               all_Detectors.py:351-354): every trial's result is the one a call
                               with dims.varn = varn_t[b] gives.  8-byte aligned, values > 0 */
} sbce_ptrs;

/* ABI version (SBCE_ABI_VERSION). */
int sbce_abi_version(void);

/* Static description of an error code. */
const char* sbce_strerror(int code);

/* Device workspace needed by sbce_em / sbce_estep / sbce_mstep for `d` (every solve mode).
 * The size depends on the library version: re-query it after upgrading the library. */
int sbce_workspace_bytes(const sbce_dims* d, size_t* bytes);

/* Device workspace for `d` with ONE solve mode (SBCE_SOLVE_*): the min-norm Gram matrix
 * ([B][L][L] complex) and the tiled factorisation's tile inverses are only carved when that solve
 * needs them, so a SBCE_SOLVE_CHOL workspace at L <= 512 is about half the size.  sbce_em /
 * sbce_mstep accept any workspace at least this large for their solve_mode (ABI 5). */
int sbce_workspace_bytes_solve(const sbce_dims* d, int solve_mode, size_t* bytes);

/* Full EM: `iters` iterations of E-step + M-step on every trial of the batch.
 * Replaces em() at Proposed_method_NMSEvsTp.py:50-83 (estep_mode SOFT) and the
 * hard-ML em() at ML_detecctor.py:51-86 (estep_mode HARD, llf != NULL). */
int sbce_em(const sbce_dims* d, const sbce_ptrs* p, int iters, int estep_mode,
            int solve_mode, void* hip_stream);

/* One E-step: theta -> per-symbol posterior moments, written to `moments`
 * [B][T_d][n_tx + n_tx*n_tx] complex (m_t, then S_t row-major,
 * S_t[a][b] = E[x_a conj(x_b)]).  Test/diagnostic entry point for the
 * E-step of Proposed_method_NMSEvsTp.py:61-69. */
int sbce_estep(const sbce_dims* d, const sbce_ptrs* p, int estep_mode,
               void* moments, void* hip_stream);

/* One M-step from given moments: builds R = sum_p u u^H + sum_t (psi psi^H)(x)S_t
 * and B^H, solves R X = B^H and writes theta = conj(X) in reference vec order
 * (Proposed_method_NMSEvsTp.py:70-80 with commutation_matrix.py:3-8 applied).
 * If `r_out` / `rhs_out` are non-NULL the normal equations ([B][L][L] and
 * [B][L][n_rx] complex) are copied there before the solve. */
int sbce_mstep(const sbce_dims* d, const sbce_ptrs* p, const void* moments,
               int solve_mode, void* r_out, void* rhs_out, void* hip_stream);

/* Per-trial symbol error rates of decisions x_dest against x_d_true ([B][T_d][n_tx]):
 * ser_out[2b] = the SER expression of SER/log_max_SER.py:162 (count_nonzero of the
 * (T_d,n_tx,1) - (T_d,1,n_tx) broadcast, / (T_d n_tx)); ser_out[2b+1] = element-wise SER. */
int sbce_ser(const sbce_dims* d, const void* x_dest, const void* x_d_true, double* ser_out,
             void* hip_stream);

/* Gaussian-prior EM output in the reference's format: the n_rx x (N n_tx n_rx^2) matrix
 * H_l = B pinv(A) of MIMO_Gaussian_proposed.py:77-85, from the reduced estimate theta
 * ([B][K], K = N n_tx n_rx, the M-step of sbce_em with SBCE_ESTEP_GAUSS).  With
 * e = vec(I_{n_rx}), f = 1 - e, Lr = N n_tx and theta_r = row r of the reduced channel,
 *   n_rx >= 2:  H_l[r] = kron(theta_r, e^T) / n_rx - (theta_r . 1) / (Lr (n_rx^2 - n_rx)) kron(1, f^T)
 *   n_rx == 1:  H_l = theta^T
 * (the all-ones term c J the reference adds to A has range outside span kron(., e) for
 * n_rx >= 2, where c drops out of pinv(A)).  h_out: [B][n_rx][N n_tx n_rx^2] complex. */
int sbce_gauss_expand(const sbce_dims* d, const void* theta, void* h_out, void* hip_stream);

/* Per-trial NMSE ||theta - h||^2 / ||h||^2 (Proposed_method_NMSEvsTp.py:172). */
int sbce_nmse(const sbce_dims* d, const void* theta, const void* h_true,
              double* nmse_out, void* hip_stream);

#ifdef __cplusplus
}
#endif

#endif /* SBCE_H_ */
