// Batched Hermitian solve of the reduced M-step system  R X = B^H  (one trial per
// workgroup), replacing np.linalg.solve ("Proposed method/Proposed_method_NMSEvsTp.py":80,
// LAPACK zgesv on the K x K system) by a Cholesky factorisation of the L x L
// Hermitian R (commutation_matrix.py:3-8 identity, SURVEY.md §8 preamble).
//
// Both kernels are left-looking blocked Cholesky with panel width NB = 16 and a
// fused forward substitution y = L^{-1} B^H, followed by a blocked back
// substitution L^H x = y; they differ in how the panel update
//     A[i, jb:jb+16] -= L[i, 0:jb] L[jb:jb+16, 0:jb]^H        (i >= jb)
// and the panel TRSM run:
//
//   chol_mfma_kernel (L <= 512, default): the trailing rows are cut into 16-row
//     tiles owned round-robin by the waves; each tile's 16 x 16 complex update is
//     4 chained v_mfma_f64_16x16x4f64 per 4 columns of k (re/im split), with the
//     panel's top block L[jb:jb+16, k-chunk] staged once in LDS as the shared B
//     operand and the tile rows streamed from R as the A operand.  The TRSM
//     X = A D^{-H} is 16 more MFMAs per tile.  The MFMA operands cost 2 loads per
//     64 FMAs instead of 17 per 16 for the per-row VALU form.
//   chol_solve_kernel (VALU, L <= 1024): thread per panel row, row register-resident.
//
// The 16 x 16 diagonal block is factored by ONE wave in registers (lane r holds
// row r) with wave-level syncs only; its inverse D^{-1} (lower) drives the TRSM
// and both triangular block solves (conj(D^{-1}) is kept in R's unused strict
// upper diagonal block for the back substitution).
// Pivots <= 1e-14 * max(diag R) are flagged (status bit 0); solve_mode DROP
// zeroes that direction, CHOL clamps the pivot to the tolerance.
#include <stdlib.h>

#include "sbce_internal.h"

namespace sbce {

namespace {

constexpr int NB = 16;   // panel width (columns)
constexpr int KC = 32;   // k-chunk of the left-looking update

typedef double d4v __attribute__((ext_vector_type(4)));

// ---------------------------------------------------------------- shared pieces
// Factor the (updated) w x w diagonal block held in wave-0 registers (lane r < w
// holds row r in dr[0..15]); writes D (lower, LDS), Di = D^{-1} (lower, LDS),
// dinv[c] = 1/L[c][c], and conj(Di) into R's strict upper diagonal block.
__device__ __forceinline__ void factor_diag(cd* dr, int w, int lane, double tol, int solve_mode, cd* D, cd* Di,
                            double* dinv, int* flag, cd* Rdiag, int L) {
    const bool mine = lane < w;
    cd* colbuf = Di;      // scratch until the inverse is built
#pragma unroll
    for (int c = 0; c < NB; ++c) {
        if (c < w) {
            if (lane == c) colbuf[NB] = dr[c];
            wave_sync();
            const double dia = colbuf[NB].x;
            const bool bad = !(dia > tol);
            const bool drop = bad && solve_mode == SBCE_SOLVE_CHOL_DROP;
            const double piv = sqrt(bad ? tol : dia);
            const double inv = drop ? 0.0 : 1.0 / piv;
            if (lane == 0) { dinv[c] = inv; if (bad) *flag = 1; }
            if (lane == c) dr[c] = cmk(drop ? 0.0 : piv, 0.0);
            else if (mine && lane > c) dr[c] = cscale(dr[c], inv);
            if (mine && lane > c) colbuf[lane] = dr[c];
            wave_sync();
#pragma unroll
            for (int c2 = c + 1; c2 < NB; ++c2) {
                if (c2 < w && mine && lane >= c2) dr[c2] = csub(dr[c2], cmulc(dr[c], colbuf[c2]));
                if ((c2 & 3) == 3) __builtin_amdgcn_sched_barrier(0);   // bound load hoisting
            }
            wave_sync();
        }
    }
    if (lane < NB) {
#pragma unroll
        for (int c = 0; c < NB; ++c) D[lane * NB + c] = (c <= lane && mine) ? dr[c] : czero();
    }
    wave_sync();
    // Di = D^{-1}: lane j < w builds column j by forward substitution in LDS
    if (lane < NB) {
        const int j = lane;
        for (int i = 0; i < NB; ++i) {
            cd acc = (i == j) ? cmk(1.0, 0.0) : czero();
            for (int k = j; k < i; ++k) acc = csub(acc, cmul(D[i * NB + k], Di[k * NB + j]));
            Di[i * NB + j] = (i >= j && i < w && j < w) ? cscale(acc, dinv[i]) : czero();
        }
    }
    wave_sync();
    // conj(Di[c2][c]) (c2 > c) -> R's unused strict upper diagonal block (back substitution)
    for (int e = lane; e < NB * NB; e += 64) {
        const int c = e / NB, c2 = e - c * NB;
        if (c2 > c && c2 < w) Rdiag[(size_t)c * L + c2] = cconj(Di[c2 * NB + c]);
    }
}

// y_blk <- Di y_blk  (one wave; w*NR <= 128 outputs)
__device__ __forceinline__ void forward_y_block(const cd* Di, cd* yblk, int w, int NR, int lane) {
    const int e0 = lane, e1 = lane + 64;
    cd t0 = czero(), t1 = czero();
    if (e0 < w * NR) {
        const int c = e0 / NR, r = e0 - c * NR;
        for (int c2 = 0; c2 <= c; ++c2) t0 = cfma(t0, Di[c * NB + c2], yblk[c2 * NR + r]);
    }
    if (e1 < w * NR) {
        const int c = e1 / NR, r = e1 - c * NR;
        for (int c2 = 0; c2 <= c; ++c2) t1 = cfma(t1, Di[c * NB + c2], yblk[c2 * NR + r]);
    }
    wave_sync();
    if (e0 < w * NR) yblk[e0] = t0;
    if (e1 < w * NR) yblk[e1] = t1;
}

// Blocked back substitution L^H x = y (whole workgroup), then theta = conj(x).
__device__ __forceinline__ void back_substitute(const cd* R, cd* y, int L, int NR, int tid, int nth, int lane,
                                int wave, int kb_stop) {
    const int nblk = (L + NB - 1) / NB;
    for (int kb = nblk - 1; kb >= kb_stop; --kb) {
        const int k0 = kb * NB;
        const int w = (L - k0) < NB ? (L - k0) : NB;
        if (wave == 0) {
            // x_blk = D^{-H} z_blk:  x[c] = z[c] / L[c][c] + sum_{c2>c} conj(Di[c2][c]) z[c2]
            // (conj(Di[c2][c]) kept in R's strict upper diagonal block); w*NR <= 128 outputs
            const int e0 = lane, e1 = lane + 64;
            cd t0 = czero(), t1 = czero();
#pragma unroll
            for (int h = 0; h < 2; ++h) {
                const int e = h ? e1 : e0;
                if (e < w * NR) {
                    const int c = e / NR, r = e - c * NR;
                    const cd* Rc = R + (size_t)(k0 + c) * L + k0;
                    const double lcc = Rc[c].x;
                    cd acc = (lcc > 0.0) ? cscale(y[(k0 + c) * NR + r], 1.0 / lcc) : czero();
                    for (int c2 = c + 1; c2 < w; ++c2) acc = cfma(acc, Rc[c2], y[(k0 + c2) * NR + r]);
                    if (h) t1 = acc; else t0 = acc;
                }
            }
            wave_sync();
            if (e0 < w * NR) y[k0 * NR + e0] = t0;
            if (e1 < w * NR) y[k0 * NR + e1] = t1;
        }
        __syncthreads();
        // y[k] -= sum_c conj(L[k0+c][k]) x[k0+c]   for k < k0
        for (int e = tid; e < k0 * NR; e += nth) {
            const int k = e / NR, r = e - k * NR;
            cd acc = y[k * NR + r];
#pragma unroll
            for (int c = 0; c < NB; ++c)
                if (c < w) acc = csub(acc, cmulc(y[(k0 + c) * NR + r], R[(size_t)(k0 + c) * L + k]));
            y[k * NR + r] = acc;
        }
        __syncthreads();
    }
}

// max diag(R) * 1e-14 (whole workgroup); also copies B^H into the LDS y when YLDS.
template <bool YLDS>
__device__ __forceinline__ double prologue(const cd* R, const cd* rhs, cd* y, double* red, int* flag, int L,
                           int NR, int tid, int nth, int lane, int wave) {
    double mx = 0.0;
    for (int i = tid; i < L; i += nth) mx = fmax(mx, R[(size_t)i * L + i].x);
    for (int off = 32; off >= 1; off >>= 1) mx = fmax(mx, shfl_xor_d(mx, off));
    if (lane == 0) red[wave] = mx;
    if (YLDS)
        for (int e = tid; e < L * NR; e += nth) y[e] = rhs[e];
    if (tid == 0) *flag = 0;
    __syncthreads();
    double tol = 0.0;
    for (int w = 0; w < (nth >> 6); ++w) tol = fmax(tol, red[w]);
    return tol * 1e-14;
}

// ---------------------------------------------------------------- VALU kernel
template <int RPT, bool YLDS>
__global__ __launch_bounds__(512) void chol_solve_kernel(MstepArgs a, int L, int NR, int skip) {
    // skip: DIAGNOSTIC phase mask (timing only, results invalid): 1 update, 2 diag factor,
    // 4 forward y, 8 trsm rows, 16 back substitution
    const int b = blockIdx.x;
    if (a.done && a.done[b]) return;
    extern __shared__ __attribute__((aligned(16))) char smem[];
    cd* T = reinterpret_cast<cd*>(smem);        // [NB][KC]
    cd* D = T + NB * KC;                        // [NB][NB] factored diagonal block
    cd* Di = D + NB * NB;                       // [NB][NB] its inverse (lower)
    double* dinv = reinterpret_cast<double*>(Di + NB * NB);   // [NB]
    double* red = dinv + NB;                    // [16] reduction scratch
    int* flag = reinterpret_cast<int*>(red + 16);
    cd* ylds = reinterpret_cast<cd*>(red + 18);  // [L][NR] when YLDS
    cd* R = a.R + (size_t)b * L * L;
    cd* y = YLDS ? ylds : a.rhs + (size_t)b * L * NR;
    const int tid = threadIdx.x, nth = blockDim.x;
    const int lane = tid & 63, wave = tid >> 6;
    const double tol = prologue<YLDS>(R, a.rhs + (size_t)b * L * NR, y, red, flag, L, NR, tid,
                                      nth, lane, wave);

    for (int jb = 0; jb < L; jb += NB) {
        const int w = (L - jb) < NB ? (L - jb) : NB;
        const int rows = L - jb;
        cd row[RPT][NB];
#pragma unroll
        for (int s = 0; s < RPT; ++s) {
            const int i = tid + s * nth;
#pragma unroll
            for (int c = 0; c < NB; ++c)
                row[s][c] = (i < rows && c < w) ? R[(size_t)(jb + i) * L + jb + c] : czero();
        }
        // ---- left-looking update with the already factored columns 0..jb-1 ----
        for (int k0 = 0; k0 < ((skip & 1) ? 0 : jb); k0 += KC) {
            const int kc = (jb - k0) < KC ? (jb - k0) : KC;
            __syncthreads();
            for (int e = tid; e < NB * KC; e += nth) {
                const int c = e / KC, k = e - c * KC;
                T[e] = (c < w && k < kc) ? R[(size_t)(jb + c) * L + k0 + k] : czero();
            }
            __syncthreads();
#pragma unroll
            for (int s = 0; s < RPT; ++s) {
                const int i = tid + s * nth;
                if (i < rows) {
                    const cd* Li = R + (size_t)(jb + i) * L + k0;
                    // fixed 8-wide k sub-chunks: 8 row loads in flight, then 16 x 8 cMACs
                    for (int kk = 0; kk < kc; kk += 8) {
                        cd lik[8];
#pragma unroll
                        for (int u = 0; u < 8; ++u) lik[u] = (kk + u < kc) ? Li[kk + u] : czero();
#pragma unroll
                        for (int c = 0; c < NB; ++c) {
#pragma unroll
                            for (int u = 0; u < 8; ++u) {
                                const cd t = T[c * KC + kk + u];   // zero-padded past kc
                                // row[c] -= lik * conj(t)
                                row[s][c].x = fma(-lik[u].x, t.x, row[s][c].x);
                                row[s][c].x = fma(-lik[u].y, t.y, row[s][c].x);
                                row[s][c].y = fma(-lik[u].y, t.x, row[s][c].y);
                                row[s][c].y = fma(lik[u].x, t.y, row[s][c].y);
                            }
                        }
                    }
                }
            }
        }
        if (wave == 0 && !(skip & 2))
            factor_diag(row[0], w, lane, tol, a.solve_mode, D, Di, dinv, flag,
                        R + (size_t)jb * L + jb, L);
        if (wave == 0 && !(skip & 4)) forward_y_block(Di, y + jb * NR, w, NR, lane);
        __syncthreads();
        // ---- panel rows: TRSM L_i = A_i D^{-H} (independent FMAs), y update, write-back ----
#pragma unroll
        for (int s = 0; s < RPT; ++s) {
            const int i = tid + s * nth;
            cd* dst = R + (size_t)(jb + i) * L + jb;
            if (i < w) {
                for (int c = 0; c <= i; ++c) dst[c] = D[i * NB + c];
            } else if (i < rows && !(skip & 8)) {
                // in place, highest column first (row[c2 < c] still holds A_i)
                cd* xr = row[s];
#pragma unroll
                for (int c = NB - 1; c >= 0; --c) {
                    cd v = czero();
#pragma unroll
                    for (int c2 = 0; c2 <= c; ++c2) v = cfmac(v, row[s][c2], Di[c * NB + c2]);
                    xr[c] = v;
                }
                for (int r = 0; r < NR; ++r) {
                    cd acc = y[(jb + i) * NR + r];
#pragma unroll
                    for (int c = 0; c < NB; ++c)
                        if (c < w) acc = csub(acc, cmul(xr[c], y[(jb + c) * NR + r]));
                    y[(jb + i) * NR + r] = acc;
                }
#pragma unroll
                for (int c = 0; c < NB; ++c)
                    if (c < w) dst[c] = xr[c];
            }
        }
        __syncthreads();
    }
    const int nblk = (L + NB - 1) / NB;
    back_substitute(R, y, L, NR, tid, nth, lane, wave, (skip & 16) ? nblk : 0);
    cd* th = a.theta + (size_t)b * L * NR;
    for (int e = tid; e < L * NR; e += nth) th[e] = cconj(y[e]);
    if (tid == 0 && a.status) a.status[b] |= *flag ? SBCE_STATUS_NONHPD : 0;
}

// ---------------------------------------------------------------- MFMA kernel
// Tile tau (rows jb + 16 tau ..) of panel jb belongs to wave tau % nw, slot tau / nw.
// Lane l of a 16 x 16 f64 MFMA: A[i = l&15][k = l>>4], B[k = l>>4][j = l&15],
// C/D value q at row (l>>4) + 4q, column l&15.
constexpr int KCM = 16;                // k-chunk: A prefetched to registers, B staged in LDS
constexpr int KCP = KCM + 1;           // padded LDS row (complex) of the B block

// One-wave factorisation of the w x w diagonal block held in LDS A[16][16] (lower part
// valid; lane l owns entries (row (l>>4) + 4h, col l&15), h < 4 -- few registers, so the
// MFMA update loop keeps its occupancy), then Di = D^{-1} by columns (lane j < 16, forward
// substitution from LDS).  Writes Di to LDS and the factor rows + conj(Di) (strict upper)
// into R's diagonal block.
__device__ __forceinline__ void factor_diag_lds(cd* A, int w, int lane, double tol,
                                                int solve_mode, cd* Di, int* flag, cd* Rdiag,
                                                int L) {
    const int col = lane & 15, r0 = lane >> 4;
    bool bad_any = false;
#pragma unroll 1
    for (int c = 0; c < w; ++c) {
        const double dia = A[c * NB + c].x;
        const bool bad = !(dia > tol);
        bad_any |= bad;
        const bool drop = bad && solve_mode == SBCE_SOLVE_CHOL_DROP;
        const double piv = sqrt(bad ? tol : dia);
        const double inv = drop ? 0.0 : 1.0 / piv;
        wave_sync();
        if (col == c) {
#pragma unroll
            for (int h = 0; h < 4; ++h) {
                const int r = r0 + 4 * h;
                if (r == c) A[c * NB + c] = cmk(drop ? 0.0 : piv, 0.0);
                else if (r > c && r < w) A[r * NB + c] = cscale(A[r * NB + c], inv);
            }
        }
        wave_sync();
        if (col > c && col < w) {
            const cd lc = cconj(A[col * NB + c]);            // conj(L[col][c])
#pragma unroll
            for (int h = 0; h < 4; ++h) {
                const int r = r0 + 4 * h;
                if (r >= col && r < w) A[r * NB + col] = csub(A[r * NB + col], cmul(A[r * NB + c], lc));
            }
        }
        wave_sync();
    }
    if (bad_any && lane == 0) *flag = 1;
    // Di[k][j] = (delta_kj - sum_{j<=m<k} L[k][m] Di[m][j]) / L[k][k]   (lane j, rows in order)
    if (lane < NB) {
        const int j = lane;
#pragma unroll 1
        for (int k = 0; k < NB; ++k) {
            cd acc = (k == j) ? cmk(1.0, 0.0) : czero();
#pragma unroll 4
            for (int m = j; m < k; ++m) acc = csub(acc, cmul(A[k * NB + m], Di[m * NB + j]));
            const double lkk = (k < w) ? A[k * NB + k].x : 0.0;
            const double inv = lkk > 0.0 ? 1.0 / lkk : 0.0;
            Di[k * NB + j] = (k < w && j <= k && j < w) ? cscale(acc, inv) : czero();
        }
    }
    wave_sync();
    // factor rows (c <= r) and conj(Di[c][r]) (c > r) into R's diagonal block
#pragma unroll
    for (int h = 0; h < 4; ++h) {
        const int r = r0 + 4 * h;
        if (r < w && col < w)
            Rdiag[(size_t)r * L + col] = (col <= r) ? A[r * NB + col] : cconj(Di[col * NB + r]);
    }
}

template <int MAXT, bool YLDS>
__global__ __launch_bounds__(512) void chol_mfma_kernel(MstepArgs a, int L, int NR) {
    const int b = blockIdx.x;
    if (a.done && a.done[b]) return;
    extern __shared__ __attribute__((aligned(16))) char smem[];
    const int tid = threadIdx.x, nth = blockDim.x;
    const int lane = tid & 63, nw = nth >> 6;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);   // wave-uniform (SGPR) tile ids
    cd* Bt = reinterpret_cast<cd*>(smem);       // [NB][KCP]  top block of the k-chunk
    cd* Di = Bt + NB * KCP;                     // [NB][NB]
    cd* Xd = Di + NB * NB;                      // [NB][NB]   diagonal tile hand-off
    double* red = reinterpret_cast<double*>(Xd + NB * NB);   // [16]
    int* flag = reinterpret_cast<int*>(red + 16);
    cd* ylds = reinterpret_cast<cd*>(red + 18);
    cd* R = a.R + (size_t)b * L * L;
    cd* y = YLDS ? ylds : a.rhs + (size_t)b * L * NR;
    const double tol = prologue<YLDS>(R, a.rhs + (size_t)b * L * NR, y, red, flag, L, NR, tid,
                                      nth, lane, wave);
    const int li = lane & 15, lk = lane >> 4;

    for (int jb = 0; jb < L; jb += NB) {
        const int w = (L - jb) < NB ? (L - jb) : NB;
        const int ntile = (L - jb + NB - 1) / NB;
        // ---- update of this wave's tiles, written back in place (R[rows, jb:jb+16]) ----
        if (jb > 0) {
            d4v cre[MAXT], cim[MAXT];
#pragma unroll
            for (int u = 0; u < MAXT; ++u) {
                const int tau = wave + u * nw;
#pragma unroll
                for (int q = 0; q < 4; ++q) {
                    const int r = jb + tau * NB + lk + 4 * q;
                    cd v = czero();
                    if (tau < ntile && r < L && li < w) v = R[(size_t)r * L + jb + li];
                    cre[u][q] = v.x;
                    cim[u][q] = v.y;
                }
            }
            for (int k0 = 0; k0 < jb; k0 += KCM) {
                cd av[MAXT][KCM / 4];
#pragma unroll
                for (int u = 0; u < MAXT; ++u) {
                    int r = jb + (wave + u * nw) * NB + li;
                    r = r < L ? r : L - 1;                // rows past L: harmless duplicates
                    const cd* ar = R + (size_t)r * L + k0 + lk;
#pragma unroll
                    for (int s = 0; s < KCM / 4; ++s)
                        av[u][s] = (wave + u * nw < ntile) ? ar[4 * s] : czero();
                }
                __syncthreads();
                for (int e = tid; e < NB * KCM; e += nth) {
                    const int c = e / KCM, k = e - c * KCM;
                    Bt[c * KCP + k] = (c < w) ? R[(size_t)(jb + c) * L + k0 + k] : czero();
                }
                __syncthreads();
#pragma unroll
                for (int s = 0; s < KCM / 4; ++s) {
                    const cd t = Bt[li * KCP + 4 * s + lk];
#pragma unroll
                    for (int u = 0; u < MAXT; ++u) {
                        // unconditional (idle slots multiply zeros): a branch around an MFMA
                        // chain makes the compiler copy the accumulators at every join
                        // re -= ar tr + ai ti ;  im -= ai tr - ar ti
                        const cd v = av[u][s];
                        cre[u] = __builtin_amdgcn_mfma_f64_16x16x4f64(-v.x, t.x, cre[u], 0, 0, 0);
                        cre[u] = __builtin_amdgcn_mfma_f64_16x16x4f64(-v.y, t.y, cre[u], 0, 0, 0);
                        cim[u] = __builtin_amdgcn_mfma_f64_16x16x4f64(-v.y, t.x, cim[u], 0, 0, 0);
                        cim[u] = __builtin_amdgcn_mfma_f64_16x16x4f64(v.x, t.y, cim[u], 0, 0, 0);
                    }
                }
            }
            __syncthreads();    // every wave is done reading R[jb.., 0:jb] and R[jb..jb+16, ..]
#pragma unroll
            for (int u = 0; u < MAXT; ++u) {
                const int tau = wave + u * nw;
#pragma unroll
                for (int q = 0; q < 4; ++q) {
                    const int r = jb + tau * NB + lk + 4 * q;
                    if (tau < ntile && r < L && li < w)
                        R[(size_t)r * L + jb + li] = cmk(cre[u][q], cim[u][q]);
                }
            }
            __syncthreads();
        }
        // ---- diagonal tile: wave 0 ----
        if (wave == 0) {
#pragma unroll
            for (int h = 0; h < 4; ++h) {
                const int r = lk + 4 * h;
                Xd[r * NB + li] = (r < w && li < w) ? R[(size_t)(jb + r) * L + jb + li] : czero();
            }
            wave_sync();
            factor_diag_lds(Xd, w, lane, tol, a.solve_mode, Di, flag, R + (size_t)jb * L + jb, L);
            forward_y_block(Di, y + jb * NR, w, NR, lane);
        }
        __syncthreads();
        // ---- TRSM X = C D^{-H} for the other tiles, computed as X^T = conj(Di) C^T so the
        //      C operand loads straight from R; lane (li, lk) ends with X[li][lk + 4q] ----
#pragma unroll
        for (int u = 0; u < MAXT; ++u) {
            const int tau = wave + u * nw;
            if (tau == 0 || tau >= ntile) continue;
            const int row0 = jb + tau * NB;
            const int ri = row0 + li < L ? row0 + li : L - 1;
            cd* crow = R + (size_t)ri * L + jb;
            d4v xre = {0.0, 0.0, 0.0, 0.0}, xim = {0.0, 0.0, 0.0, 0.0};
#pragma unroll
            for (int s = 0; s < NB / 4; ++s) {
                const cd d = Di[li * NB + 4 * s + lk];     // A[j][k] = conj(Di[j][4s+k])
                const cd c = crow[4 * s + lk];             // B[k][i] = C[i][4s+k]
                // X^T = conj(Di) C^T:  re += dr cr + di ci ;  im += dr ci - di cr
                xre = __builtin_amdgcn_mfma_f64_16x16x4f64(d.x, c.x, xre, 0, 0, 0);
                xre = __builtin_amdgcn_mfma_f64_16x16x4f64(d.y, c.y, xre, 0, 0, 0);
                xim = __builtin_amdgcn_mfma_f64_16x16x4f64(d.x, c.y, xim, 0, 0, 0);
                xim = __builtin_amdgcn_mfma_f64_16x16x4f64(-d.y, c.x, xim, 0, 0, 0);
            }
            const bool live = row0 + li < L;
            cd xv[4];
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                const int j = lk + 4 * q;
                xv[q] = cmk(xre[q], xim[q]);
                if (live && j < w) crow[j] = xv[q];
            }
            // y[row0+li] -= sum_j X[li][j] y_blk[j]: 4 columns per lane, reduced over lk
            for (int r = 0; r < NR; ++r) {
                cd p = czero();
#pragma unroll
                for (int q = 0; q < 4; ++q) {
                    const int j = lk + 4 * q;
                    if (j < w) p = cfma(p, xv[q], y[(jb + j) * NR + r]);
                }
                p.x += shfl_xor_d(p.x, 16); p.y += shfl_xor_d(p.y, 16);
                p.x += shfl_xor_d(p.x, 32); p.y += shfl_xor_d(p.y, 32);
                if (lk == 0 && live) y[(row0 + li) * NR + r] = csub(y[(row0 + li) * NR + r], p);
            }
        }
        __syncthreads();
    }
    back_substitute(R, y, L, NR, tid, nth, lane, wave, 0);
    cd* th = a.theta + (size_t)b * L * NR;
    for (int e = tid; e < L * NR; e += nth) th[e] = cconj(y[e]);
    if (tid == 0 && a.status) a.status[b] |= *flag ? SBCE_STATUS_NONHPD : 0;
}

template <int RPT, bool YLDS>
hipError_t launch_rpt(const Problem& pb, const MstepArgs& a, int nth, size_t lds, hipStream_t s) {
    const char* sk = getenv("SBCE_CHOL_SKIP");      // diagnostic only (see kernel)
    const int skip = sk ? atoi(sk) : 0;
    hipLaunchKernelGGL((chol_solve_kernel<RPT, YLDS>), dim3(pb.B), dim3(nth), lds, s, a, pb.L, pb.NR,
                       skip);
    return hipGetLastError();
}

template <bool YLDS>
hipError_t launch_y(const Problem& pb, const MstepArgs& a, int nth, int rpt, size_t lds,
                    hipStream_t s) {
    switch (rpt) {
        case 1: return launch_rpt<1, YLDS>(pb, a, nth, lds, s);
        case 2: return launch_rpt<2, YLDS>(pb, a, nth, lds, s);
    }
    return hipErrorInvalidValue;
}

template <bool YLDS>
hipError_t launch_mfma_y(const Problem& pb, const MstepArgs& a, int nw, int maxt, size_t lds,
                         hipStream_t s) {
    const dim3 g(pb.B), blk(64 * nw);
    switch (maxt) {
        case 1: hipLaunchKernelGGL((chol_mfma_kernel<1, YLDS>), g, blk, lds, s, a, pb.L, pb.NR); break;
        case 2: hipLaunchKernelGGL((chol_mfma_kernel<2, YLDS>), g, blk, lds, s, a, pb.L, pb.NR); break;
        case 3: hipLaunchKernelGGL((chol_mfma_kernel<3, YLDS>), g, blk, lds, s, a, pb.L, pb.NR); break;
        case 4: hipLaunchKernelGGL((chol_mfma_kernel<4, YLDS>), g, blk, lds, s, a, pb.L, pb.NR); break;
        default: return hipErrorInvalidValue;
    }
    return hipGetLastError();
}

}  // namespace

bool chol_supported(const Problem& pb) { return pb.L >= 1 && pb.L <= 1024; }

hipError_t launch_chol_solve(const Problem& pb, const MstepArgs& a, hipStream_t s) {
    if (!chol_supported(pb)) return hipErrorInvalidValue;
    const size_t ybytes = (size_t)pb.L * pb.NR * sizeof(cd);
    const char* impl = getenv("SBCE_CHOL_IMPL");    // "valu" forces the VALU kernel (A/B runs)
    const bool force_valu = impl && impl[0] == 'v';
    if (!force_valu && pb.L <= 512) {
        const int ntile = (pb.L + NB - 1) / NB;
        const int nw = ntile < 8 ? ntile : 8;
        const int maxt = (ntile + nw - 1) / nw;
        const size_t base = (size_t)(NB * KCP + 2 * NB * NB) * sizeof(cd) + 18 * sizeof(double);
        if (ybytes <= 48 * 1024) return launch_mfma_y<true>(pb, a, nw, maxt, base + ybytes, s);
        return launch_mfma_y<false>(pb, a, nw, maxt, base, s);
    }
    int nth = (pb.L + 63) / 64 * 64;
    if (nth > 512) nth = 512;
    const int rpt = (pb.L + nth - 1) / nth;
    const size_t base = (size_t)(NB * KC + 2 * NB * NB) * sizeof(cd) + (NB + 18) * sizeof(double);
    if (ybytes <= 48 * 1024) return launch_y<true>(pb, a, nth, rpt, base + ybytes, s);
    return launch_y<false>(pb, a, nth, rpt, base, s);
}

}  // namespace sbce
