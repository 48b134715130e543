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
// Pivots <= 1e-14 * max(diag R) are flagged (status bit 0) and their direction is dropped
// (column zeroed, y and x components 0) in every public solve mode.  A clamp (pivot raised to
// sqrt(tol), the column kept) is unstable on a rank-deficient R: past the numerical rank the
// Schur complement is rounding noise, not PSD, so a column of noise delta divided by sqrt(tol)
// feeds back delta^2 / tol into the next pivots and overflows within ~10 columns (round 5's
// all-NaN theta at L = 600; oracle.em_reduced.mstep_chol_policy(clamp=True) shows it on the CPU).
// Dropped, the solution's range-space part is lstsq's minimum-norm solution (to ~1e-13).  Only
// the min-norm solve's C = G^H G (HPD by construction) clamps (kSolveClampHpd).
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
            const bool drop = bad && solve_mode != kSolveClampHpd;
            const double piv = sqrt(bad ? tol : dia);
            const double inv = drop ? 0.0 : 1.0 / piv;
            if (lane == 0) { dinv[c] = inv; if (bad) *flag |= 1; }
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

// The same with the block staged in LDS (yb: NB*NR entries, raw on entry): the result goes
// to yb (zero past w rows) and to y in global memory, so the next reader of the block
// waits on LDS, not on a global store-then-load round trip.  NR <= 8.
__device__ __forceinline__ void forward_y_lds(const cd* Di, cd* yb, cd* yglob, int w, int NR,
                                              int lane) {
    const int e0 = lane, e1 = lane + 64;
    cd t0 = czero(), t1 = czero();
    // all 16 terms with every load issued up front (Di's strict upper part is zero, so the terms
    // past the row's diagonal add nothing), four partial sums: a dependent chain of 4, not 16
    auto row = [&](int e) {
        const int c = e / NR, r = e - c * NR;
        cd p[4] = {czero(), czero(), czero(), czero()};
#pragma unroll
        for (int c2 = 0; c2 < NB; ++c2) p[c2 & 3] = cfma(p[c2 & 3], Di[c * NB + c2], yb[c2 * NR + r]);
        return cadd(cadd(p[0], p[1]), cadd(p[2], p[3]));
    };
    if (e0 < w * NR) t0 = row(e0);
    if (e1 < w * NR) t1 = row(e1);
    wave_sync();
    if (e0 < NB * NR) yb[e0] = t0;
    if (e1 < NB * NR) yb[e1] = t1;
    if (e0 < w * NR) yglob[e0] = t0;
    if (e1 < w * NR) yglob[e1] = t1;
    wave_sync();
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
    __syncthreads();                                 // red[] is reused afterwards
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
    if (tid == 0 && a.status)
        a.status[b] |= ((*flag & 1) ? a.clamp_status : 0) | ((*flag & 2) ? SBCE_STATUS_RANK : 0) |
                       ((skip & 31) ? SBCE_STATUS_DEBUG : 0);
}

// ---------------------------------------------------------------- MFMA kernel
// Tile tau (rows jb + 16 tau ..) of panel jb belongs to wave tau % nw, slot tau / nw.
// Lane l of a 16 x 16 f64 MFMA: A[i = l&15][k = l>>4], B[k = l>>4][j = l&15],
// C/D value q at row (l>>4) + 4q, column l&15.
constexpr int KCM = 16;                // k-chunk of the A-operand register pipeline

// Di = L^-1 of a factored 16 x 16 diagonal block (A: L's lower part, pivots on the diagonal;
// dinv: 1 / pivot, 0 for dropped / absent directions) by recursive doubling: Di[k][k] = dinv[k],
// then for s = 1, 2, 4, 8 the off-diagonal block of every 2s x 2s diagonal block,
//   Di21 = -D22 (L21 D11),
// from the two s x s blocks inverted at the level before -- two lane-parallel products per level
// (one output entry per lane) instead of 16 dependent row steps with cross-lane reductions.
// A dropped direction (dinv = 0) zeroes its row and column of Di, as the row recurrence does.
// P (L21 D11) is staged in Di's upper-right 8 x 8 quarter (strictly upper: no block of the
// recursion touches it), zeroed at the end.
__device__ __forceinline__ void diag_inverse_rd(const cd* A, cd* Di, const double* dinv, int w, int lane) {
#pragma unroll
    for (int h = 0; h < 4; ++h) {
        const int e = lane + 64 * h, r = e >> 4, c = e & 15;
        Di[e] = (r == c && r < w) ? cmk(dinv[r], 0.0) : czero();
    }
    wave_sync();
    cd* P = Di + 8;                                          // P[e] at Di[(e >> 3) * 16 + 8 + (e & 7)]
#pragma unroll
    for (int ls = 0; ls < 4; ++ls) {
        const int s = 1 << ls;
        const bool on = lane < 8 * s;                        // 8 s entries at this level
        const int bi = lane >> (2 * ls), rem = lane & (s * s - 1);
        const int i = rem >> ls, j = rem & (s - 1);
        const int b0 = bi * 2 * s;
        // every operand read unconditionally (the entries a guard skips are finite: zeros of Di's
        // strict upper part, or P entries) and the guarded FMAs as selects, so the reads can issue
        // ahead of the FMA chain instead of one LDS latency per product (same sums, same order)
        if (on) {                                            // P = L21 D11 (D11 lower: m >= j)
            const cd* Lr = A + (b0 + s + i) * NB + b0;
            cd acc = czero();
#pragma unroll
            for (int m = 0; m < s; ++m)
                acc = csel(m >= j, cfma(acc, Lr[m], Di[(b0 + m) * NB + b0 + j]), acc);
            P[(lane >> 3) * NB + (lane & 7)] = acc;
        }
        wave_sync();
        if (on) {                                            // Di21 = -D22 P (D22 lower: m <= i)
            const cd* Dr = Di + (b0 + s + i) * NB + b0 + s;
            cd acc = czero();
#pragma unroll
            for (int m = 0; m < s; ++m) {
                const int pe = bi * s * s + m * s + j;
                acc = csel(m <= i, cfma(acc, Dr[m], P[(pe >> 3) * NB + (pe & 7)]), acc);
            }
            Di[(b0 + s + i) * NB + b0 + j] = (b0 + s + i < w) ? cmk(-acc.x, -acc.y) : czero();
        }
        wave_sync();
    }
    P[(lane >> 3) * NB + (lane & 7)] = czero();
    wave_sync();
}

// One-wave factorisation of the w x w diagonal block held in LDS A[16][16] (lower part
// valid).  Lane l owns entries (row (l>>4) + 4h, col l&15), h < 4.  Column c costs ONE
// LDS round trip: every lane reads the pivot and the column entries it needs, then
//   L[r][c] = A[r][c] / p,   A[r][c2] -= A[r][c] conj(A[c2][c]) / p^2   (r >= c2 > c)
// are written together (the trailing update uses the unscaled column, so no second
// pass).  Per lane, the role in column step c depends only on its column: col > c trailing,
// col == c the column, col < c final (not stored), so every entry is m A[r][col] + A[r][c] f
// with (m, f) per lane -- 6 FP64 ops per entry, no per-entry selects; the pivot's 1/sqrt is
// seeded by v_rsq_f64 (fast_rsqrt64).  Di = D^{-1} by recursive doubling (diag_inverse_rd).
// Few registers, so the MFMA phases keep their occupancy.  Writes Di to LDS and the factor
// rows + conj(Di) (strict upper) into R's diagonal block.  The strict upper part of A is never
// multiplied into a lower entry: it may hold the workspace's old contents (NaN included).
__device__ __forceinline__ void factor_diag_lds(cd* A, int w, int lane, double tol,
                                                int solve_mode, cd* Di, double* dinv, int* flag,
                                                cd* Rdiag, int L,
                                                unsigned long long* clk = nullptr) {
    const int col = lane & 15, r0 = lane >> 4;
    unsigned long long tc = clk ? __builtin_amdgcn_s_memtime() : 0;
    bool bad_any = false, near_any = false;
#pragma unroll 1
    for (int c = 0; c < w; ++c) {
        const double dia = A[c * NB + c].x;
        const cd lc = A[col * NB + c];                      // A[col][c] (unscaled)
        cd arc[4], arx[4];
#pragma unroll
        for (int h = 0; h < 4; ++h) {
            const int r = r0 + 4 * h;
            arc[h] = A[r * NB + c];
            arx[h] = A[r * NB + col];
        }
        const bool bad = !(dia > tol);
        bad_any |= bad;
        // min-norm solve (tol = 32 x lstsq's cut, minnorm.hip): a pivot between 4 cut and
        // 64 tol may be decided differently from the singular values lstsq thresholds
        near_any |= solve_mode == SBCE_SOLVE_MINNORM && dia > tol * (1.0 / 8) && dia < tol * 64;
        const bool drop = bad && solve_mode != kSolveClampHpd;
        const double pv = bad ? tol : dia;
        const double rs = fast_rsqrt64(pv);
        const double piv = drop ? 0.0 : pv * rs;
        const double inv = drop ? 0.0 : rs;
        const cd lcs = cscale(cconj(lc), inv * inv);
        if (clk && lane == 0) { const unsigned long long t2 = __builtin_amdgcn_s_memtime(); clk[9] += t2 - tc; tc = t2; }
        wave_sync();                                         // all reads of column c done
        dinv[c] = inv;                                       // same value from every lane
        const bool gt = col > c, eq = col == c;
        const double m = eq ? 0.0 : 1.0;
        const double fx = gt ? -lcs.x : (eq ? inv : 0.0);
        const double fy = gt ? -lcs.y : 0.0;
        if (col >= c) {
#pragma unroll
            for (int h = 0; h < 4; ++h) {
                const int r = r0 + 4 * h;
                const cd v = cmk(fma(arc[h].x, fx, fma(-arc[h].y, fy, m * arx[h].x)),
                                 fma(arc[h].x, fy, fma(arc[h].y, fx, m * arx[h].y)));
                A[r * NB + col] = v;
            }
            if (eq && r0 == (c & 3)) A[c * NB + c] = cmk(piv, 0.0);
        }
        wave_sync();
        if (clk && lane == 0) { const unsigned long long t2 = __builtin_amdgcn_s_memtime(); clk[10] += t2 - tc; tc = t2; }
    }
    if (bad_any) *flag |= 1;
    if (near_any) *flag |= 2;
    if (clk && lane == 0) { const unsigned long long t2 = __builtin_amdgcn_s_memtime(); clk[0] += t2 - tc; tc = t2; }
    diag_inverse_rd(A, Di, dinv, w, lane);
    if (clk && lane == 0) { const unsigned long long t2 = __builtin_amdgcn_s_memtime(); clk[1] += t2 - tc; tc = t2; }
    // factor rows (c <= r) and conj(Di[c][r]) (c > r) into R's diagonal block
#pragma unroll
    for (int h = 0; h < 4; ++h) {
        const int r = r0 + 4 * h;
        if (r < w && col < w)
            Rdiag[(size_t)r * L + col] = csel(col <= r, A[r * NB + col], cconj(Di[col * NB + r]));
    }
    if (clk && lane == 0) { const unsigned long long t2 = __builtin_amdgcn_s_memtime(); clk[8] += t2 - tc; }
}

// Blocked back substitution L^H x = y for the MFMA kernel: every thread owns column
// k = tid (+ nth) of the update and loads its 16 factor entries BEFORE the barrier that
// publishes the block solution, so each block pays one memory latency, not three.
template <int H = 2>     // rows k of the update per thread (H * nth >= L)
__device__ __forceinline__ void back_substitute_pf(const cd* R, cd* y, int L, int NR, int tid,
                                                   int nth, int lane, int wave, int kb_stop,
                                                   int ld, cd* dblk) {
    // dblk: LDS [NB][NB] scratch for the diagonal block (its rows hold L[c][c] on the
    // diagonal and conj(Di[c2][c]) above it), loaded by the whole workgroup at once
    const int nblk = (L + NB - 1) / NB;
    // diagonal blocks are prefetched one step ahead (one entry per thread when nth >= 256)
    const bool pf = nth >= NB * NB;
    auto dload = [&](int kb) {
        const int k0 = kb * NB, w = (L - k0) < NB ? (L - k0) : NB;
        const int c = (tid >> 4) & 15, c2 = tid & 15;
        return (kb >= 0 && tid < NB * NB && c < w && c2 < w && c2 >= c)
                   ? R[(size_t)(k0 + c) * ld + k0 + c2] : czero();
    };
    cd dnext = pf ? dload(nblk - 1) : czero();
    for (int kb = nblk - 1; kb >= kb_stop; --kb) {
        const int k0 = kb * NB;
        const int w = (L - k0) < NB ? (L - k0) : NB;
        // prefetch: conj(L[k0+c][k]) for this thread's columns k < k0
        cd lv[H][NB];
#pragma unroll
        for (int h = 0; h < H; ++h) {
            const int k = tid + h * nth;
#pragma unroll
            for (int c = 0; c < NB; ++c)
                lv[h][c] = (k < k0 && c < w) ? R[(size_t)(k0 + c) * ld + k] : czero();
        }
        if (pf) {
            if (tid < NB * NB) dblk[tid] = dnext;
            dnext = dload(kb - 1);
        } else {
            for (int e = tid; e < NB * NB; e += nth) {
                const int c = e >> 4, c2 = e & 15;
                dblk[e] = (c < w && c2 < w && c2 >= c) ? R[(size_t)(k0 + c) * ld + k0 + c2] : czero();
            }
        }
        __syncthreads();
        if (wave == 0) {
            // x_blk = D^{-H} z_blk:  x[c] = z[c] / L[c][c] + sum_{c2>c} conj(Di[c2][c]) z[c2]
            const int e0 = lane, e1 = lane + 64;
            cd t0 = czero(), t1 = czero();
#pragma unroll
            for (int h = 0; h < 2; ++h) {
                const int e = h ? e1 : e0;
                if (e < w * NR) {
                    const int c = e / NR, r = e - c * NR;
                    const cd* Rc = dblk + c * NB;
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
#pragma unroll
        for (int h = 0; h < H; ++h) {
            const int k = tid + h * nth;
            if (k < k0) {
                for (int r = 0; r < NR; ++r) {
                    cd acc = y[k * NR + r];
#pragma unroll
                    for (int c = 0; c < NB; ++c)
                        if (c < w) acc = csub(acc, cmulc(y[(k0 + c) * NR + r], lv[h][c]));
                    y[k * NR + r] = acc;
                }
            }
        }
        __syncthreads();
    }
}

// DIAGNOSTIC (skip & 64): per-phase s_memtime sums of waves 0 and 1 of block 0
__device__ unsigned long long g_chol_clk[32];

// DIAGNOSTIC phase-skip mask of the Cholesky kernels (timing only, results invalid).  Set
// only through sbce_debug_chol_skip(); every trial factored while it is nonzero carries
// SBCE_STATUS_DEBUG, so a result computed with skipped phases can never pass as valid.  A/B
// build only (sbce_internal.h SBCE_AB): the product library's mask is the constant 0.
#if SBCE_AB
int g_chol_skip = 0;
#else
constexpr int g_chol_skip = 0;
#endif

// Geometry of one chol_mfma_kernel launch: the factored L x L matrix starts at row/col
// `off` of trial b's matrix (a.R + b*stride), leading dimension ld.  SOLVE = false
// factors in place only (a diagonal tile of the large-L path, tol from tolp[b]).
struct CholGeom {
    int ld, off;
    size_t stride;
    const double* tolp;
    const int32_t* ext;    // SOLVE = false: per-trial active columns (null: all); tiles at or
                           // past ext[b] are left untouched (min-norm path, minnorm.hip)
};

template <int MAXT, bool YLDS, int NWB, int KB, bool SOLVE = true>
__global__ __launch_bounds__(64 * NWB) __attribute__((amdgpu_waves_per_eu(2)))
void chol_mfma_kernel(MstepArgs a, int L, int NR, int skip, CholGeom g) {
    constexpr int KBP = KB + 1;                 // padded LDS row (complex) of the panel block
    const int ld = g.ld;
    // skip: DIAGNOSTIC phase mask (timing only, results invalid): 1 update, 2 diag factor,
    // 8 trsm tiles, 16 back substitution
    const int b = blockIdx.x;
    if (a.done && a.done[b]) return;
    if (!SOLVE && g.ext && g.off >= g.ext[b]) return;
    extern __shared__ __attribute__((aligned(16))) char smem[];
    const int tid = threadIdx.x, nth = blockDim.x;
    const int lane = tid & 63, nw = nth >> 6;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);   // wave-uniform tile ids
    cd* Bp = reinterpret_cast<cd*>(smem);       // [NB][KBP]  panel top rows, one k-block
    cd* Di = Bp + NB * KBP;                     // [NB][NB]
    cd* Xs = Di + NB * NB;                      // [nw][NB][NB] per-wave tile scratch
    double* red = reinterpret_cast<double*>(Xs + nw * NB * NB);   // [16]
    int* flag = reinterpret_cast<int*>(red + 16);
    cd* ylds = reinterpret_cast<cd*>(red + 18);
    cd* R = a.R + (size_t)b * g.stride + (size_t)g.off * ld + g.off;
    cd* y = SOLVE ? (YLDS ? ylds : a.rhs + (size_t)b * L * NR) : nullptr;
    cd* X = Xs + wave * NB * NB;
    double tol;
    if (SOLVE) {
        tol = prologue<YLDS>(R, a.rhs + (size_t)b * L * NR, y, red, flag, L, NR, tid, nth, lane,
                             wave);
    } else {
        tol = g.tolp[b];
        if (tid == 0) *flag = 0;
        __syncthreads();
    }
    const int li = lane & 15, lk = lane >> 4;
    const bool clk = (skip & 64) && b == 0 && wave < 2 && lane == 0;
    unsigned long long tclk = clk ? __builtin_amdgcn_s_memtime() : 0;
#define SBCE_CLK(ph)                                                          \
    if (clk) {                                                                \
        const unsigned long long t2 = __builtin_amdgcn_s_memtime();           \
        g_chol_clk[wave * 8 + (ph)] += t2 - tclk;                             \
        tclk = t2;                                                            \
    }

    for (int jb = 0; jb < L; jb += NB) {
        const int w = (L - jb) < NB ? (L - jb) : NB;
        const int ntile = (L - jb + NB - 1) / NB;
        const int nact = (ntile - wave + nw - 1) / nw;     // active tile slots of this wave
        // A-operand rows of this wave's tiles (rows past L read row L-1: harmless)
        const cd* arow[MAXT];
#pragma unroll
        for (int u = 0; u < MAXT; ++u) {
            int r = jb + (wave + u * nw) * NB + li;
            r = r < L ? r : L - 1;
            arow[u] = R + (size_t)r * ld + lk;
        }
        // ---- C tiles <- A[rows, jb:jb+16] (C layout) ----
        d4v cre[MAXT], cim[MAXT];
#pragma unroll
        for (int u = 0; u < MAXT; ++u) {
            const int tau = wave + u * nw;
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                const int r = jb + tau * NB + lk + 4 * q;
                cd v = czero();
                if (tau < ntile && r < L && li < w) v = R[(size_t)r * ld + jb + li];
                cre[u][q] = v.x;
                cim[u][q] = v.y;
            }
        }
        // ---- left-looking update over k-blocks of KBMAX columns: the panel's top rows
        //      are staged once per block; each wave streams its tiles' rows with the next
        //      16-column chunk's loads in flight while the current chunk's MFMAs run ----
        for (int kb0 = 0; kb0 < ((skip & 1) ? 0 : jb); kb0 += KB) {
            const int kbs = (jb - kb0) < KB ? (jb - kb0) : KB;         // multiple of 16
            cd av[MAXT][4];
#pragma unroll
            for (int u = 0; u < MAXT; ++u)
#pragma unroll
                for (int s2 = 0; s2 < 4; ++s2) av[u][s2] = arow[u][kb0 + 4 * s2];
            __syncthreads();
            for (int e = tid; e < NB * kbs; e += nth) {
                const int c = e / kbs, k = e - c * kbs;
                Bp[c * KBP + k] = (c < w) ? R[(size_t)(jb + c) * ld + kb0 + k] : czero();
            }
            __syncthreads();
            for (int k0 = 0; k0 < kbs; k0 += KCM) {
                // register pipeline (next chunk's loads in flight) only where the registers
                // allow it; MAXT >= 4 relies on the second resident workgroup instead
                constexpr bool PIPE = MAXT <= 3;
                cd an[PIPE ? MAXT : 1][4];
                const bool more = k0 + KCM < kbs;
                if (PIPE) {
#pragma unroll
                    for (int u = 0; u < MAXT; ++u)
#pragma unroll
                        for (int s2 = 0; s2 < 4; ++s2)
                            an[PIPE ? u : 0][s2] = more ? arow[u][kb0 + k0 + KCM + 4 * s2] : czero();
                } else if (k0 > 0) {
#pragma unroll
                    for (int u = 0; u < MAXT; ++u)
#pragma unroll
                        for (int s2 = 0; s2 < 4; ++s2) av[u][s2] = arow[u][kb0 + k0 + 4 * s2];
                }
#pragma unroll
                for (int s2 = 0; s2 < 4; ++s2) {
                    const cd t = Bp[li * KBP + k0 + 4 * s2 + lk];
#pragma unroll
                    for (int u = 0; u < MAXT; ++u) {
                        if (u >= nact) break;          // wave-uniform (SGPR) bound: no exec masking
                        // re -= ar tr + ai ti ;  im -= ai tr - ar ti
                        const cd v = av[u][s2];
                        cre[u] = __builtin_amdgcn_mfma_f64_16x16x4f64(-v.x, t.x, cre[u], 0, 0, 0);
                        cre[u] = __builtin_amdgcn_mfma_f64_16x16x4f64(-v.y, t.y, cre[u], 0, 0, 0);
                        cim[u] = __builtin_amdgcn_mfma_f64_16x16x4f64(-v.y, t.x, cim[u], 0, 0, 0);
                        cim[u] = __builtin_amdgcn_mfma_f64_16x16x4f64(v.x, t.y, cim[u], 0, 0, 0);
                    }
                }
                if (PIPE) {
#pragma unroll
                    for (int u = 0; u < MAXT; ++u)
#pragma unroll
                        for (int s2 = 0; s2 < 4; ++s2) av[u][s2] = an[PIPE ? u : 0][s2];
                }
            }
        }
        SBCE_CLK(0)
        // ---- diagonal tile (tau = 0: wave 0, slot 0), factored in LDS ----
        if (wave == 0) {
#pragma unroll
            for (int q = 0; q < 4; ++q) X[(lk + 4 * q) * NB + li] = cmk(cre[0][q], cim[0][q]);
            wave_sync();
            if (!(skip & 2))
                factor_diag_lds(X, w, lane, tol, a.solve_mode, Di, red, flag,
                                R + (size_t)jb * ld + jb, ld, clk ? g_chol_clk + 6 : nullptr);
            if (SOLVE) forward_y_block(Di, y + jb * NR, w, NR, lane);
        }
        SBCE_CLK(1)
        __syncthreads();
        SBCE_CLK(2)
        // ---- TRSM X = C D^{-H} for the other tiles, as X^T = conj(Di) C^T (C transposed
        //      through the wave's LDS scratch); lane (li, lk) ends with X[li][lk + 4q] ----
#pragma unroll
        for (int u = 0; u < MAXT; ++u) {
            const int tau = wave + u * nw;
            if (tau == 0 || tau >= ntile || (skip & 8)) continue;
            const int row0 = jb + tau * NB;
#pragma unroll
            for (int q = 0; q < 4; ++q) X[(lk + 4 * q) * NB + li] = cmk(cre[u][q], cim[u][q]);
            wave_sync();
            d4v xre = {0.0, 0.0, 0.0, 0.0}, xim = {0.0, 0.0, 0.0, 0.0};
#pragma unroll
            for (int s2 = 0; s2 < NB / 4; ++s2) {
                const cd d = Di[li * NB + 4 * s2 + lk];    // A[j][k] = conj(Di[j][4s+k])
                const cd c = X[li * NB + 4 * s2 + lk];     // B[k][i] = C[i][4s+k]
                // X^T = conj(Di) C^T:  re += dr cr + di ci ;  im += dr ci - di cr
                xre = __builtin_amdgcn_mfma_f64_16x16x4f64(d.x, c.x, xre, 0, 0, 0);
                xre = __builtin_amdgcn_mfma_f64_16x16x4f64(d.y, c.y, xre, 0, 0, 0);
                xim = __builtin_amdgcn_mfma_f64_16x16x4f64(d.x, c.y, xim, 0, 0, 0);
                xim = __builtin_amdgcn_mfma_f64_16x16x4f64(-d.y, c.x, xim, 0, 0, 0);
            }
            const bool live = row0 + li < L;
            cd* crow = R + (size_t)(live ? row0 + li : L - 1) * ld + jb;
            cd xv[4];
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                const int j = lk + 4 * q;
                xv[q] = cmk(xre[q], xim[q]);
                if (live && j < w) crow[j] = xv[q];
            }
            // y[row0+li] -= sum_j X[li][j] y_blk[j]: 4 columns per lane, reduced over lk
            for (int r = 0; r < (SOLVE ? NR : 0); ++r) {
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
            wave_sync();
        }
        SBCE_CLK(3)
        __syncthreads();
        SBCE_CLK(4)
    }
    if (SOLVE) {
        back_substitute_pf(R, y, L, NR, tid, nth, lane, wave, (skip & 16) ? (L + NB - 1) / NB : 0,
                           ld, Di);
        SBCE_CLK(5)
        cd* th = a.theta + (size_t)b * L * NR;
        for (int e = tid; e < L * NR; e += nth) th[e] = cconj(y[e]);
    }
#undef SBCE_CLK
    if (tid == 0 && a.status)
        a.status[b] |= ((*flag & 1) ? a.clamp_status : 0) | ((*flag & 2) ? SBCE_STATUS_RANK : 0) |
                       ((skip & 31) ? SBCE_STATUS_DEBUG : 0);
}

// ---------------------------------------------------------------- batched panel kernels
// The same left-looking blocked factorisation and fused forward substitution as
// chol_mfma_kernel, but one LAUNCH per 32-column panel step over every trial instead of
// one workgroup walking all panels of its trial: the panel update is a batched GEMM with
// one wave per 16-row tile (high occupancy hides the streamed rows' latency), the serial
// diagonal factors of ~1000 trials run side by side in the factor launch, and no kernel
// needs the register budget of a whole trial's tiles.  y lives in the rhs buffer.
//
// panel_update_kernel (jb > 0): C_tau = A[rows tau, jb:jb+32] - L[rows tau, 0:jb] L[jb:jb+32, 0:jb]^H
// for the 16-row tiles tau = 0.. of panel jb; block = NWU waves = NWU row tiles of ONE trial,
// the panel's top rows staged per KBU-column chunk in LDS by LDS-DMA (shared B operand),
// each wave's rows streamed from R with the next 16 columns in flight; every A value
// feeds both 16-column halves (the left-looking re-reads of a 16-column panel halved).
// Blocks of one trial sit on one XCD.
constexpr int KBU = 64;
constexpr int PW = 32;    // panel width: two 16-column sub-panels
// Body of the update of trial b, row-tile group grp, by the columns [0, kend) (kend = jb: the
// whole left part; the look-ahead step passes kend = jb - PW).  Bp: PW * (KBU + 1) LDS entries.
// G3: the complex products by three real MFMAs instead of four (csub_step, sbce_internal.h).
template <int NWU, bool G3 = false>
__device__ __forceinline__ void panel_update_body(const MstepArgs& a, int L, int jb, int kend, int ntile,
                                                  int b, int grp, int skip, cd* Bp, int kbeg = 0) {
    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int li = lane & 15, lk = lane >> 4;
    const int tau = grp * NWU + wave;
    const bool active = tau < ntile;                         // wave-uniform
    const int w2 = (L - jb) < PW ? (L - jb) : PW;
    cd* R = a.R + (size_t)b * L * L;
    const int row0 = jb + tau * NB;
    int r = row0 + li;
    r = r < L ? r : L - 1;                                   // rows past L: harmless reads
    const cd* arow = R + (size_t)r * L + lk;
    // tile 0's right half lies in the strict upper triangle: neither loaded nor stored
    const int nv = tau == 0 ? 1 : 2;
    d4v cre[2], cim[2], c2[2];
#pragma unroll
    for (int v = 0; v < 2; ++v) {
        cre[v] = d4v{0.0, 0.0, 0.0, 0.0};
        cim[v] = d4v{0.0, 0.0, 0.0, 0.0};
        c2[v] = d4v{0.0, 0.0, 0.0, 0.0};
        if (active && v < nv) {
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                const int rr = row0 + lk + 4 * q, c = 16 * v + li;
                if (rr < L && c < w2) {
                    const cd x = R[(size_t)rr * L + jb + c];
                    cre[v][q] = x.x;
                    cim[v][q] = x.y;
                }
            }
        }
        csub_init<G3>(cre[v], cim[v], c2[v]);
    }
    for (int kb0 = kbeg; kb0 < ((skip & 1) ? 0 : kend); kb0 += KBU) {
        const int kbs = (kend - kb0) < KBU ? (kend - kb0) : KBU;    // multiple of 16
        cd av[4];
        if (active) {
#pragma unroll
            for (int s2 = 0; s2 < 4; ++s2) av[s2] = arow[kb0 + 4 * s2];
        }
        __syncthreads();
        // panel top rows by LDS-DMA: one wave-instruction per row (64 lanes = the row's KBU
        // slots, never crossing into the pad); lanes past kbs / rows past w2 read row jb
#pragma unroll
        for (int c8 = 0; c8 < PW / NWU; ++c8) {
            const int c = wave * (PW / NWU) + c8;
            const cd* src = R + (size_t)jb * L + kb0;
            if (c < w2 && lane < kbs) src = R + (size_t)(jb + c) * L + kb0 + lane;
            __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)src,
                                             (__attribute__((address_space(3))) void*)(Bp + c * (KBU + 1)),
                                             16, 0, 0);
        }
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
        if (active) {
            for (int k0 = 0; k0 < kbs; k0 += 16) {
                cd an[4];
                const bool more = k0 + 16 < kbs;
#pragma unroll
                for (int s2 = 0; s2 < 4; ++s2) an[s2] = more ? arow[kb0 + k0 + 16 + 4 * s2] : czero();
#pragma unroll
                for (int s2 = 0; s2 < 4; ++s2) {
                    const cd v = av[s2];
#pragma unroll
                    for (int h = 0; h < 2; ++h) {
                        if (h >= nv) break;                  // wave-uniform
                        // C -= A conj(B)^T
                        csub_step<G3>(cre[h], cim[h], c2[h], v, Bp[(16 * h + li) * (KBU + 1) + k0 + 4 * s2 + lk]);
                    }
                }
#pragma unroll
                for (int s2 = 0; s2 < 4; ++s2) av[s2] = an[s2];
            }
        }
    }
    if (active) {
#pragma unroll
        for (int v = 0; v < 2; ++v) {
            if (v >= nv) break;
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                const int rr = row0 + lk + 4 * q, c = 16 * v + li;
                const cd o = csub_out<G3>(cre[v], cim[v], c2[v], q);
                if (rr < L && c < w2) R[(size_t)rr * L + jb + c] = o;
            }
        }
    }
}

// panel_update2_kernel (wide left-looking step): the updates of panels j AND j+1 by the columns
// [0, jb) in one launch -- for every trial gpt0 four-tile groups of panel j's rows and gpt1 of
// panel j+1's (rows from jb + 32, k < jb; the rank-32 remainder by panel j is the next factor
// launch's pre-update).  A trial's blocks are adjacent on one XCD, so the two column halves read
// each row segment of L[:, 0:jb] at about the same time: the second read is an L2 hit, and the
// left-looking re-reads from HBM halve (a 64-column panel's traffic with the 32-column panels'
// registers, occupancy and factor chain).
template <bool G3 = false>
__global__ __launch_bounds__(256) void panel_update2_kernel(MstepArgs a, int L, int jb, int ntile,
                                                            int gpt0, int gpt1, int skip) {
    __shared__ __attribute__((aligned(16))) cd Bp[PW * (KBU + 1)];
    const int gpt = gpt0 + gpt1;
    const int id = blockIdx.x, xcd = id & 7, slot = id >> 3;
    const int b = (slot / gpt) * 8 + xcd, g = slot - (slot / gpt) * gpt;
    if (b >= a.nbatch) return;
    if (a.done && a.done[b]) return;
    if (g < gpt0) panel_update_body<4, G3>(a, L, jb, jb, ntile, b, g, skip, Bp);
    else panel_update_body<4, G3>(a, L, jb + PW, jb, ntile - 2, b, g - gpt0, skip, Bp);
}

// 16 x 16 tile of R (rows row0.., columns c0.., w valid columns) into per-lane registers:
// lane holds entries e = lane + 64 h, row e >> 4, column e & 15
__device__ __forceinline__ void load_tile16(const cd* R, int L, int row0, int c0, int w, int lane,
                                            bool on, cd* v) {
#pragma unroll
    for (int h = 0; h < 4; ++h) {
        const int e = lane + 64 * h, rr = e >> 4, c = e & 15;
        v[h] = (on && row0 + rr < L && c < w) ? R[(size_t)(row0 + rr) * L + c0 + c] : czero();
    }
}

// TRSM of one 16-row tile (values in X, LDS) against the factored diagonal block of the
// sub-panel at column c0 (inverse Di): L = C D^{-H}, written to R; y rows updated with the
// sub-panel's y block yb.  Returns X[li][lk + 4q] in xv (the A-operand layout of k-step q).
// The y update Y_tile -= X Y_blk is two real MFMA GEMMs over the 16 columns of X with the
// right-hand sides embedded as 2*NR real columns (re | im): A = Re X, Im X (= xv as it
// comes out of the TRSM), B1 = [Re Y | Im Y], B2 = [-Im Y | Re Y]; lane (li, lk) ends with
// component (li < NR: re, else im) of right-hand side li mod NR for rows lk + 4q, and
// yd[q] holds the same component of those rows before the update (load_ycomp).  NR <= 8.
template <bool G3 = false>
__device__ __forceinline__ void trsm_tile16(cd* R, cd* y, const cd* Di, const cd* X, const cd* yb,
                                            int L, int NR, int row0, int c0, int w, int li,
                                            int lk, cd* xv, const double* yd, cd* ylds = nullptr) {
    d4v xre = {0.0, 0.0, 0.0, 0.0}, xim = {0.0, 0.0, 0.0, 0.0}, x2 = {0.0, 0.0, 0.0, 0.0};
#pragma unroll
    for (int s2 = 0; s2 < NB / 4; ++s2) {
        const cd d = Di[li * NB + 4 * s2 + lk];    // A[j][k] = conj(Di[j][4s+k])
        const cd c = X[li * NB + 4 * s2 + lk];     // B[k][i] = C[i][4s+k]
        // X^T = conj(Di) C^T:  re += dr cr + di ci ;  im += dr ci - di cr
        if constexpr (G3) {       // P1 = dr cr, P2 = di ci, P3 = (dr + di)(cr - ci): im = P1 - P2 - P3
            xre = __builtin_amdgcn_mfma_f64_16x16x4f64(d.x, c.x, xre, 0, 0, 0);
            x2 = __builtin_amdgcn_mfma_f64_16x16x4f64(d.y, c.y, x2, 0, 0, 0);
            xim = __builtin_amdgcn_mfma_f64_16x16x4f64(d.x + d.y, c.x - c.y, xim, 0, 0, 0);
        } else {
            xre = __builtin_amdgcn_mfma_f64_16x16x4f64(d.x, c.x, xre, 0, 0, 0);
            xre = __builtin_amdgcn_mfma_f64_16x16x4f64(d.y, c.y, xre, 0, 0, 0);
            xim = __builtin_amdgcn_mfma_f64_16x16x4f64(d.x, c.y, xim, 0, 0, 0);
            xim = __builtin_amdgcn_mfma_f64_16x16x4f64(-d.y, c.x, xim, 0, 0, 0);
        }
    }
    const bool live = row0 + li < L;
    cd* crow = R + (size_t)(live ? row0 + li : L - 1) * L + c0;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        const int j = lk + 4 * q;
        xv[q] = G3 ? cmk(xre[q] + x2[q], xre[q] - x2[q] - xim[q]) : cmk(xre[q], xim[q]);
        if (live && j < w) crow[j] = xv[q];
    }
    const bool isre = li < NR, on = li < 2 * NR;
    const int r = isre ? li : li - NR;
    // two accumulation chains of four MFMAs (Re X and Im X parts) instead of one of eight
    d4v u = {0.0, 0.0, 0.0, 0.0}, u2 = {0.0, 0.0, 0.0, 0.0};
#pragma unroll
    for (int s2 = 0; s2 < NB / 4; ++s2) {
        const cd v = on ? yb[(4 * s2 + lk) * NR + r] : czero();     // Y_blk[4s+lk][r]
        const double b1 = isre ? v.x : v.y, b2 = isre ? -v.y : v.x;
        u = __builtin_amdgcn_mfma_f64_16x16x4f64(xv[s2].x, b1, u, 0, 0, 0);
        u2 = __builtin_amdgcn_mfma_f64_16x16x4f64(xv[s2].y, b2, u2, 0, 0, 0);
    }
    u += u2;
    if (on) {
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            const int rr = lk + 4 * q;
            const double yn = yd[q] - u[q];
            if (row0 + rr < L) ((double*)(y + (size_t)(row0 + rr) * NR + r))[isre ? 0 : 1] = yn;
            // the updated rows also to LDS (zero past L) when the caller solves them next
            if (ylds) ((double*)(ylds + rr * NR + r))[isre ? 0 : 1] = row0 + rr < L ? yn : 0.0;
        }
    }
}

// the y rows of a 16-row tile for trsm_tile16: lane (li, lk) holds component li < NR (re) /
// NR <= li < 2 NR (im) of right-hand side li mod NR, rows lk + 4q
__device__ __forceinline__ void load_ycomp(const cd* y, int L, int NR, int row0, int li, int lk,
                                           bool on, double* yd) {
    const bool isre = li < NR;
    const int r = isre ? li : li - NR;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        const int rr = row0 + lk + 4 * q;
        yd[q] = (on && li < 2 * NR && rr < L) ? ((const double*)(y + (size_t)rr * NR + r))[isre ? 0 : 1]
                                              : 0.0;
    }
}

// panel_factor_kernel: one workgroup (4 waves) per trial, panel [jb, jb+32) as sub-panels
// A = [jb, jb+16) and B = [jb+16, jb+32):
//   wave 0: factor A's diagonal tile (factor_diag_lds), D_A^-1 y_A, TRSM of row tile 1
//           (X_A1, kept in LDS);                                                 barrier
//   wave 0: C_B1 -= X_A1 X_A1^H, factor it (B's diagonal tile), D_B^-1 y_B;
//   waves 1-3, row tiles tau >= 2: TRSM against D_A, then the in-panel rank-16 update
//           C_B,tau -= X_A,tau X_A1^H written back to R;                          barrier
//   all waves, tau >= 2: TRSM of C_B,tau against D_B.
// LDS of the factor body (cd entries): Xs (4 waves' 16 x 16 scratch), DiA, DiB, XA1, ybA, ybB
constexpr int kFacXs = 0, kFacDiA = 4 * NB * NB, kFacDiB = kFacDiA + NB * NB, kFacXA1 = kFacDiB + NB * NB,
              kFacYbA = kFacXA1 + NB * NB, kFacYbB = kFacYbA + NB * 8, kFacLds = kFacYbB + NB * 8;
template <bool G3 = false>
__device__ __forceinline__ void panel_preupdate(const MstepArgs& a, int L, int jb, int ntile, int b,
                                                cd* Lp);
template <bool G3 = false, bool CLK = false>
__device__ __forceinline__ void panel_factor_body(const MstepArgs& a, int L, int NR, int jb, int ntile,
                                                  int b, int skip, cd* sm, double* dinv, int& flag,
                                                  unsigned long long t_start = 0) {
    // skip: DIAGNOSTIC phase mask (timing only, results invalid): 2 diag factors, 8 trsm tiles
    cd* DiA = sm + kFacDiA;
    cd* DiB = sm + kFacDiB;
    cd* XA1 = sm + kFacXA1;
    cd* Xs = sm + kFacXs;
    cd* ybA = sm + kFacYbA;     // the sub-panels' y blocks after D^-1
    cd* ybB = sm + kFacYbB;
    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int li = lane & 15, lk = lane >> 4;
    const int w2 = (L - jb) < PW ? (L - jb) : PW;
    const int wA = w2 < NB ? w2 : NB, wB = w2 - NB;          // wB <= 0: no sub-panel B
    const int jbB = jb + NB;
    const double tol = a.tol[b];
    cd* R = a.R + (size_t)b * L * L;
    cd* y = a.rhs + (size_t)b * L * NR;
    cd* X = Xs + wave * NB * NB;
    const bool trsm = !(skip & 8);
    // DIAGNOSTIC (skip & 64, trial 0 only): per-phase s_memtime sums of waves 0 and 1 in
    // g_chol_clk[16 + 8 wave + phase] (timing only; results unchanged)
    const bool clk = CLK && b == 0 && wave < 2;
    unsigned long long tclk = clk ? (t_start ? t_start : __builtin_amdgcn_s_memtime()) : 0;
    auto stamp = [&](int ph) {
        if (clk && lane == 0) {
            const unsigned long long t2 = __builtin_amdgcn_s_memtime();
            g_chol_clk[16 + 8 * wave + ph] += t2 - tclk;
            tclk = t2;
        }
    };
    if (tid == 0) flag = 0;
    __syncthreads();
    stamp(0);
    cd xv[4];
    // waves 1-3: their first row tile (A part) and y rows are in flight while wave 0 factors
    cd cur[4];
    double ycur[4];
    if (wave != 0) {
        const int tau = 1 + wave;
        load_tile16(R, L, jb + tau * NB, jb, wA, lane, trsm && tau < ntile, cur);
        load_ycomp(y, L, NR, jb + tau * NB, li, lk, trsm && tau < ntile, ycur);
    }
    // wave 0's serial chain reads every global operand up front: B's diagonal tile (written
    // by no one in this launch) arrives by LDS-DMA in DiB (unused until factor B; no
    // registers held across factor A), y block A in ybA, before factor A starts
    if (wave == 0) {
        __builtin_amdgcn_s_setprio(3);                       // the serial chain issues first
        cd t1[4];
        double y1[4];
        load_tile16(R, L, jbB, jb, wA, lane, ntile > 1, t1);        // row tile 1, A part
        load_ycomp(y, L, NR, jbB, li, lk, ntile > 1, y1);
        if (wB > 0) {
#pragma unroll
            for (int h = 0; h < 4; ++h) {          // DiB[e] = R[jbB + e/16][jbB + e%16]
                const int e = lane + 64 * h, rr = e >> 4, c = e & 15;
                const cd* src = R + (size_t)(jbB + (rr < wB ? rr : 0)) * L + jbB + (c < wB ? c : 0);
                __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)src,
                                                 (__attribute__((address_space(3))) void*)(DiB + 64 * h),
                                                 16, 0, 0);
            }
        }
        for (int e = lane; e < NB * NR; e += 64) ybA[e] = (e < wA * NR) ? y[jb * NR + e] : czero();
        for (int e = lane; e < NB * NB; e += 64) {
            const int rr = e >> 4, c = e & 15;
            X[e] = (rr < wA && c <= rr) ? R[(size_t)(jb + rr) * L + jb + c] : czero();
        }
        wave_sync();
        stamp(1);
        if (!(skip & 2)) {
            factor_diag_lds(X, wA, lane, tol, a.solve_mode, DiA, dinv, &flag,
                            R + (size_t)jb * L + jb, L);
            forward_y_lds(DiA, ybA, y + jb * NR, wA, NR, lane);
        }
        wave_sync();
        stamp(2);
        if (ntile > 1 && trsm) {
#pragma unroll
            for (int h = 0; h < 4; ++h) X[lane + 64 * h] = t1[h];
            wave_sync();
            // row tile 1 = sub-panel B's rows: its updated y rows are staged raw in ybB
            trsm_tile16<G3>(R, y, DiA, X, ybA, L, NR, jbB, jb, wA, li, lk, xv, y1, ybB);
#pragma unroll
            for (int q = 0; q < 4; ++q) XA1[li * NB + lk + 4 * q] = xv[q];
        }
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");      // B's diagonal tile is in DiB
        stamp(3);
    }
    __syncthreads();
    stamp(4);
    if (wave == 0) {
        if (wB > 0) {
            // B's diagonal tile: C_B1 -= X_A1 X_A1^H, then factor
            d4v cre = {0.0, 0.0, 0.0, 0.0}, cim = {0.0, 0.0, 0.0, 0.0}, c2;
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                const int rr = lk + 4 * q;
                if (rr < wB && li < wB) {
                    const cd x = DiB[rr * NB + li];
                    cre[q] = x.x;
                    cim[q] = x.y;
                }
            }
            wave_sync();                                         // DiB is overwritten next
            csub_init<G3>(cre, cim, c2);
#pragma unroll
            for (int s2 = 0; s2 < 4; ++s2) csub_step<G3>(cre, cim, c2, xv[s2], XA1[li * NB + 4 * s2 + lk]);
#pragma unroll
            for (int q = 0; q < 4; ++q) X[(lk + 4 * q) * NB + li] = csub_out<G3>(cre, cim, c2, q);
            wave_sync();
            if (!(skip & 2)) {
                factor_diag_lds(X, wB, lane, tol, a.solve_mode, DiB, dinv, &flag,
                                R + (size_t)jbB * L + jbB, L);
                forward_y_lds(DiB, ybB, y + jbB * NR, wB, NR, lane);
            }
        }
    } else if (trsm) {
        // row tiles tau >= 2: TRSM against D_A, in-panel update of their B part
        int tau = 1 + wave;
        for (; tau < ntile; tau += 3) {
            const int row0 = jb + tau * NB;
#pragma unroll
            for (int h = 0; h < 4; ++h) X[lane + 64 * h] = cur[h];
            d4v cre = {0.0, 0.0, 0.0, 0.0}, cim = {0.0, 0.0, 0.0, 0.0}, c2;
            if (wB > 0) {
#pragma unroll
                for (int q = 0; q < 4; ++q) {
                    const int rr = row0 + lk + 4 * q;
                    if (rr < L && li < wB) {
                        const cd x = R[(size_t)rr * L + jbB + li];
                        cre[q] = x.x;
                        cim[q] = x.y;
                    }
                }
            }
            const double yv[4] = {ycur[0], ycur[1], ycur[2], ycur[3]};
            load_tile16(R, L, row0 + 3 * NB, jb, wA, lane, tau + 3 < ntile, cur);   // next
            load_ycomp(y, L, NR, row0 + 3 * NB, li, lk, tau + 3 < ntile, ycur);
            wave_sync();
            trsm_tile16<G3>(R, y, DiA, X, ybA, L, NR, row0, jb, wA, li, lk, xv, yv);
            if (wB > 0) {
                csub_init<G3>(cre, cim, c2);
#pragma unroll
                for (int s2 = 0; s2 < 4; ++s2) csub_step<G3>(cre, cim, c2, xv[s2], XA1[li * NB + 4 * s2 + lk]);
#pragma unroll
                for (int q = 0; q < 4; ++q) {
                    const int rr = row0 + lk + 4 * q;
                    if (rr < L && li < wB) R[(size_t)rr * L + jbB + li] = csub_out<G3>(cre, cim, c2, q);
                }
            }
            wave_sync();
        }
    }
    stamp(5);
    __syncthreads();
    stamp(6);
    if (wB > 0 && trsm) {
        // row tiles tau >= 2: TRSM of the updated B part against D_B
        int tau = 2 + wave;
        load_tile16(R, L, jb + tau * NB, jbB, wB, lane, tau < ntile, cur);
        load_ycomp(y, L, NR, jb + tau * NB, li, lk, tau < ntile, ycur);
        for (; tau < ntile; tau += 4) {
            const int row0 = jb + tau * NB;
#pragma unroll
            for (int h = 0; h < 4; ++h) X[lane + 64 * h] = cur[h];
            const double yv[4] = {ycur[0], ycur[1], ycur[2], ycur[3]};
            load_tile16(R, L, row0 + 4 * NB, jbB, wB, lane, tau + 4 < ntile, cur);
            load_ycomp(y, L, NR, row0 + 4 * NB, li, lk, tau + 4 < ntile, ycur);
            wave_sync();
            trsm_tile16<G3>(R, y, DiB, X, ybB, L, NR, row0, jbB, wB, li, lk, xv, yv);
            wave_sync();
        }
    }
    stamp(7);
    const int st = ((flag & 1) ? a.clamp_status : 0) | ((flag & 2) ? SBCE_STATUS_RANK : 0) |
                   ((skip & 31) ? SBCE_STATUS_DEBUG : 0);
    if (tid == 0 && st && a.status) atomicOr(&a.status[b], st);
}

// PRE (wide schedule, odd panels): the rank-32 update of the panel by the previous panel's
// columns [jb-32, jb) (the part panel_update2_kernel left) inside the factor launch, first
// (panel_preupdate), then the factor.
template <bool G3 = false, bool PRE = false, bool CLK = false>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(4)))
void panel_factor_kernel(MstepArgs a, int L, int NR, int jb, int ntile, int skip) {
    __shared__ __attribute__((aligned(16))) cd sm[kFacLds];
    __shared__ double dinv[NB];
    __shared__ int flag;
    const int b = blockIdx.x;
    if (a.done && a.done[b]) return;
    const unsigned long long t0 = CLK ? __builtin_amdgcn_s_memtime() : 0;   // diagnostic
    if (PRE && !(skip & 1)) panel_preupdate<G3>(a, L, jb, ntile, b, sm);
    panel_factor_body<G3, CLK>(a, L, NR, jb, ntile, b, skip, sm, dinv, flag, t0);
}

// ---------------------------------------------------------------- look-ahead panel step
// Rank-PW update of panel j (columns [jb, jb+32), every row tile) by panel j-1's columns
// [jb-32, jb), written back to R: the part of panel j's left-looking update that the
// look-ahead step could not make in the previous launch (panel j-1 was being factored there).
// Lp: PW * (PW + 1) LDS entries (panel j-1's rows jb .. jb+31, the shared B operand).
template <bool G3>
__device__ __forceinline__ void panel_preupdate(const MstepArgs& a, int L, int jb, int ntile, int b,
                                                cd* Lp) {
    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int li = lane & 15, lk = lane >> 4;
    const int w2 = (L - jb) < PW ? (L - jb) : PW;
    const int k0c = jb - PW;
    cd* R = a.R + (size_t)b * L * L;
    for (int e = tid; e < PW * PW; e += 256) {
        const int c = e >> 5, k = e & (PW - 1);
        Lp[c * (PW + 1) + k] = c < w2 ? R[(size_t)(jb + c) * L + k0c + k] : czero();
    }
    __syncthreads();
    for (int tau = wave; tau < ntile; tau += 4) {             // wave-uniform
        const int row0 = jb + tau * NB;
        int r = row0 + li;
        r = r < L ? r : L - 1;                                   // rows past L: harmless reads
        const cd* arow = R + (size_t)r * L + k0c + lk;
        cd av[4];
#pragma unroll
        for (int s2 = 0; s2 < 4; ++s2) av[s2] = arow[4 * s2];
        const int nv = tau == 0 ? 1 : 2;                         // tile 0's right half: upper triangle
        d4v cre[2], cim[2], c2[2];
#pragma unroll
        for (int v = 0; v < 2; ++v) {
            cre[v] = d4v{0.0, 0.0, 0.0, 0.0};
            cim[v] = d4v{0.0, 0.0, 0.0, 0.0};
            c2[v] = d4v{0.0, 0.0, 0.0, 0.0};
            if (v < nv) {
#pragma unroll
                for (int q = 0; q < 4; ++q) {
                    const int rr = row0 + lk + 4 * q, c = 16 * v + li;
                    if (rr < L && c < w2) {
                        const cd x = R[(size_t)rr * L + jb + c];
                        cre[v][q] = x.x;
                        cim[v][q] = x.y;
                    }
                }
            }
            csub_init<G3>(cre[v], cim[v], c2[v]);
        }
#pragma unroll 1
        for (int k0 = 0; k0 < PW; k0 += 16) {
            cd an[4];
#pragma unroll
            for (int s2 = 0; s2 < 4; ++s2) an[s2] = k0 == 0 ? arow[16 + 4 * s2] : czero();
#pragma unroll
            for (int s2 = 0; s2 < 4; ++s2) {
                const cd v = av[s2];
#pragma unroll
                for (int h = 0; h < 2; ++h) {
                    if (h >= nv) break;                          // wave-uniform
                    // C -= A conj(B)^T (three real MFMAs per complex product with G3)
                    csub_step<G3>(cre[h], cim[h], c2[h], v, Lp[(16 * h + li) * (PW + 1) + k0 + 4 * s2 + lk]);
                }
            }
#pragma unroll
            for (int s2 = 0; s2 < 4; ++s2) av[s2] = an[s2];
        }
#pragma unroll
        for (int v = 0; v < 2; ++v) {
            if (v >= nv) break;
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                const int rr = row0 + lk + 4 * q, c = 16 * v + li;
                if (rr < L && c < w2) R[(size_t)rr * L + jb + c] = csub_out<G3>(cre[v], cim[v], c2[v], q);
            }
        }
    }
    __syncthreads();
}

// ---------------------------------------------------------------- back substitution
// General blocked back substitution L^H x = y (any L <= 512, any NR; SBCE_BACKSUB=1 forces it
// for the shapes backsub4_kernel covers, as a cross-check), theta = conj(x).
__global__ __launch_bounds__(256) void backsub_kernel(MstepArgs a, int L, int NR, int skip) {
    extern __shared__ __attribute__((aligned(16))) char smem[];
    cd* y = reinterpret_cast<cd*>(smem);
    const int b = blockIdx.x;
    if (a.done && a.done[b]) return;
    const int tid = threadIdx.x, lane = tid & 63, nth = blockDim.x;     // 2 nth >= L
    const int wave = tid >> 6;
    const cd* R = a.R + (size_t)b * L * L;
    const cd* yg = a.rhs + (size_t)b * L * NR;
    for (int e = tid; e < L * NR; e += nth) y[e] = yg[e];
    __syncthreads();
    back_substitute_pf<2>(R, y, L, NR, tid, nth, lane, wave, (skip & 16) ? (L + NB - 1) / NB : 0, L,
                          y + L * NR);
    cd* th = a.theta + (size_t)b * L * NR;
    for (int e = tid; e < L * NR; e += nth) th[e] = cconj(y[e]);
}

// Back substitution block step shared by backsub4_kernel: thread tid owns row k = tid < 256 of
// y in registers; every wave solves the block x = D^{-H} z itself (lane c*NR + r: output (c, r))
// into a wave-private LDS copy, so the update of the wave's own rows needs no workgroup barrier;
// the owners of the next block's rows then publish them, every thread publishes its entry of the
// next diagonal block (L_cc, conj(Di[c2][c]) above the diagonal), both double-buffered in LDS,
// and the workgroup synchronises once per block.
struct Bs3Buf {
    cd lv[NB];         // L[k0 + cc][tid], this thread's update column
    cd dd;             // entry (tid >> 4, tid & 15) of the diagonal block
};
__device__ __forceinline__ void bs3_load(const cd* R, int L, int kb, int tid, Bs3Buf& bf) {
    const int k0 = kb * NB, w = (L - k0) < NB ? (L - k0) : NB;
    const int c = tid >> 4, c2 = tid & 15;
    bf.dd = (kb >= 0 && c < w && c2 >= c && c2 < w) ? R[(size_t)(k0 + c) * L + k0 + c2] : czero();
#pragma unroll
    for (int cc = 0; cc < NB; ++cc)
        bf.lv[cc] = (kb >= 0 && tid < k0 && cc < w) ? R[(size_t)(k0 + cc) * L + tid] : czero();
}
template <int NR>
__device__ __forceinline__ void bs3_step(int kb, int L, int tid, int lane, int wave, int c, int r,
                                         const Bs3Buf& bf, const cd& dnext, cd (&yr)[NR],
                                         cd (*zb)[NB * NR], cd (*db)[NB * NB], cd (*xw)[NB * NR],
                                         cd* th) {
    const int k0 = kb * NB, w = (L - k0) < NB ? (L - k0) : NB;
    const cd* z = zb[kb & 1];
    const cd* d = db[kb & 1] + c * NB;         // row c: L_cc, then conj(Di[c2][c]) for c2 > c
    cd x = czero();
    if (c < w) {
        const double lcc = d[c].x;
        x = lcc > 0.0 ? cscale(z[c * NR + r], 1.0 / lcc) : czero();
        for (int c2 = c + 1; c2 < w; ++c2) x = cfma(x, d[c2], z[c2 * NR + r]);
    }
    if (lane < NB * NR) xw[wave][lane] = x;
    if (wave == 0 && c < w) th[(size_t)(k0 + c) * NR + r] = cconj(x);
    wave_sync();
    if (tid < k0) {
#pragma unroll
        for (int cc = 0; cc < NB; ++cc)
#pragma unroll
            for (int q = 0; q < NR; ++q) {           // y -= x conj(l): four FMAs
                const cd xv = xw[wave][cc * NR + q];
                yr[q] = cfmac(yr[q], cmk(-xv.x, -xv.y), bf.lv[cc]);
            }
    }
    if (kb > 0) {                              // publish the next block's rows and diagonal block
        if (tid >= k0 - NB && tid < k0) {
#pragma unroll
            for (int q = 0; q < NR; ++q) zb[(kb - 1) & 1][(tid - (k0 - NB)) * NR + q] = yr[q];
        }
        db[(kb - 1) & 1][tid] = dnext;
    }
    __syncthreads();
}

// The same one-barrier block step with the factor entries loaded ONE step ahead into a single
// buffer (issued as soon as the update has consumed the current one, the next diagonal-block
// entry at the start of the step): ~100 VGPRs instead of backsub3's 192, so four trials'
// workgroups are resident per CU (one round over ~1000 trials instead of two).
template <int NR>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(4)))
void backsub4_kernel(MstepArgs a, int L) {
    __shared__ cd zb[2][NB * NR];              // the current / next block's z rows
    __shared__ cd db[2][NB * NB];              // the current / next diagonal block
    __shared__ cd xw[4][NB * NR];              // per-wave block solution
    const int b = blockIdx.x;
    if (a.done && a.done[b]) return;
    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const cd* R = a.R + (size_t)b * L * L;
    const cd* yg = a.rhs + (size_t)b * L * NR;
    cd* th = a.theta + (size_t)b * L * NR;
    const int nblk = (L + NB - 1) / NB;
    const int c = lane / NR, r = lane - (lane / NR) * NR;     // block-solve output of this lane
    const int dc = tid >> 4, dc2 = tid & 15;                  // this thread's diagonal-block entry
    cd yr[NR];                                                 // row k = tid of y
#pragma unroll
    for (int q = 0; q < NR; ++q) yr[q] = tid < L ? yg[(size_t)tid * NR + q] : czero();
    Bs3Buf bf;
    bs3_load(R, L, nblk - 1, tid, bf);
    {
        // the last block's rows (k0 may be 256: no owner thread) straight from the input
        const int k0 = (nblk - 1) * NB, w = L - k0;
        if (tid < w * NR) zb[(nblk - 1) & 1][tid] = yg[(size_t)k0 * NR + tid];
        db[(nblk - 1) & 1][tid] = bf.dd;
    }
    __syncthreads();
    for (int kb = nblk - 1; kb >= 0; --kb) {
        const int k0 = kb * NB, w = (L - k0) < NB ? (L - k0) : NB;
        cd dnext = czero();                    // entry of the next diagonal block (k0 - 16 ..)
        if (kb > 0 && dc2 >= dc) dnext = R[(size_t)(k0 - NB + dc) * L + k0 - NB + dc2];
        const cd* z = zb[kb & 1];
        const cd* d = db[kb & 1] + c * NB;     // row c: L_cc, then conj(Di[c2][c]) for c2 > c
        cd x = czero();
        if (c < w) {
            const double lcc = d[c].x;
            x = lcc > 0.0 ? cscale(z[c * NR + r], 1.0 / lcc) : czero();
            for (int c2 = c + 1; c2 < w; ++c2) x = cfma(x, d[c2], z[c2 * NR + r]);
        }
        if (lane < NB * NR) xw[wave][lane] = x;
        if (wave == 0 && c < w) th[(size_t)(k0 + c) * NR + r] = cconj(x);
        wave_sync();
        if (tid < k0) {
#pragma unroll
            for (int cc = 0; cc < NB; ++cc)
#pragma unroll
                for (int q = 0; q < NR; ++q) {       // y -= x conj(l): four FMAs
                    const cd xv = xw[wave][cc * NR + q];
                    yr[q] = cfmac(yr[q], cmk(-xv.x, -xv.y), bf.lv[cc]);
                }
        }
        if (kb > 0) {
            // next block's update columns into the same registers (rows tid < k0 - 16 only)
#pragma unroll
            for (int cc = 0; cc < NB; ++cc)
                bf.lv[cc] = (tid < k0 - NB) ? R[(size_t)(k0 - NB + cc) * L + tid] : czero();
            // publish the next block's rows and diagonal block
            if (tid >= k0 - NB && tid < k0) {
#pragma unroll
                for (int q = 0; q < NR; ++q) zb[(kb - 1) & 1][(tid - (k0 - NB)) * NR + q] = yr[q];
            }
            db[(kb - 1) & 1][tid] = dnext;
        }
        __syncthreads();
    }
}

// DIAGNOSTIC launch timing (sbce_debug_chol_timing): HIP events around the wide schedule's
// update / factor / back-substitution launches of the next M-step(s) on the launch stream
struct CholTimer {
    bool on = false, made = false;
    int n = 0;
    hipEvent_t ev[512];
    int kind[256];
};
CholTimer g_ct;
void ct_begin(hipStream_t s, int kind) {
    if (g_ct.on && g_ct.n + 2 <= 512) { g_ct.kind[g_ct.n / 2] = kind; (void)hipEventRecord(g_ct.ev[g_ct.n++], s); }
}
void ct_end(hipStream_t s) {
    if (g_ct.on && (g_ct.n & 1)) (void)hipEventRecord(g_ct.ev[g_ct.n++], s);
}

hipError_t launch_chol_batched(const Problem& pb, const MstepArgs& a, hipStream_t s) {
    const int skip = g_chol_skip;                   // diagnostic only (see kernels)
    hipError_t e = launch_diag_tol(pb, a, s);
    if (e != hipSuccess) return e;
    const int npan = (pb.L + PW - 1) / PW;
    // the wide schedule: even panels j >= 2 update panels j and j+1 by [0, jb) in one launch
    // (panel_update2_kernel), odd panels are pre-updated by panel j-1 inside their factor launch:
    // half the left-looking HBM re-reads of one update launch per panel
    const bool g3 = g_debug.cplx3 && (a.solve_mode == SBCE_SOLVE_CHOL || a.solve_mode == kSolveClampHpd);
    for (int j = 0; j < npan; ++j) {
        const int jb = j * PW;
        const int rem = (pb.L - jb + NB - 1) / NB;
        if (j >= 2 && !(j & 1)) {
            ct_begin(s, 0);
            const int gpt0 = (rem + 3) / 4;
            const int gpt1 = j + 1 < npan ? (rem - 2 + 3) / 4 : 0;
            const long nblk = 8L * ((pb.B + 7) / 8) * (gpt0 + gpt1);
            if (g3)
                hipLaunchKernelGGL(panel_update2_kernel<true>, dim3((unsigned)nblk), dim3(256), 0, s, a, pb.L,
                                   jb, rem, gpt0, gpt1, skip);
            else
                hipLaunchKernelGGL(panel_update2_kernel<false>, dim3((unsigned)nblk), dim3(256), 0, s, a, pb.L,
                                   jb, rem, gpt0, gpt1, skip);
            ct_end(s);
        }
        const bool pre = (j & 1) != 0;
        ct_begin(s, 1);
        if (g3 && pre && (skip & 64))               // DIAGNOSTIC phase clocks (tools/chol_clock.py)
            hipLaunchKernelGGL((panel_factor_kernel<true, true, true>), dim3(pb.B), dim3(256), 0, s, a, pb.L,
                               pb.NR, jb, rem, skip);
        else if (g3 && (skip & 64))
            hipLaunchKernelGGL((panel_factor_kernel<true, false, true>), dim3(pb.B), dim3(256), 0, s, a, pb.L,
                               pb.NR, jb, rem, skip);
        else if (g3 && pre)
            hipLaunchKernelGGL((panel_factor_kernel<true, true>), dim3(pb.B), dim3(256), 0, s, a, pb.L, pb.NR,
                               jb, rem, skip);
        else if (g3)
            hipLaunchKernelGGL((panel_factor_kernel<true, false>), dim3(pb.B), dim3(256), 0, s, a, pb.L,
                               pb.NR, jb, rem, skip);
        else if (pre)
            hipLaunchKernelGGL((panel_factor_kernel<false, true>), dim3(pb.B), dim3(256), 0, s, a, pb.L,
                               pb.NR, jb, rem, skip);
        else
            hipLaunchKernelGGL((panel_factor_kernel<false, false>), dim3(pb.B), dim3(256), 0, s, a, pb.L,
                               pb.NR, jb, rem, skip);
        ct_end(s);
        if ((e = hipGetLastError()) != hipSuccess) return e;
    }
    // default (L <= 272, NR <= 4): the one-buffer one-barrier kernel; otherwise, or with
    // SBCE_BACKSUB=1 (cross-check), the general kernel
    if (pb.L <= 272 && pb.NR <= 4 && !g_debug.backsub_general && !(skip & 16)) {
        ct_begin(s, 2);
        switch (pb.NR) {
            case 1: hipLaunchKernelGGL(backsub4_kernel<1>, dim3(pb.B), dim3(256), 0, s, a, pb.L); break;
            case 2: hipLaunchKernelGGL(backsub4_kernel<2>, dim3(pb.B), dim3(256), 0, s, a, pb.L); break;
            case 3: hipLaunchKernelGGL(backsub4_kernel<3>, dim3(pb.B), dim3(256), 0, s, a, pb.L); break;
            default: hipLaunchKernelGGL(backsub4_kernel<4>, dim3(pb.B), dim3(256), 0, s, a, pb.L); break;
        }
        ct_end(s);
        return hipGetLastError();
    }
    hipLaunchKernelGGL(backsub_kernel, dim3(pb.B), dim3(256),
                       ((size_t)pb.L * pb.NR + NB * NB) * sizeof(cd), s,
                       a, pb.L, pb.NR, skip);
    return hipGetLastError();
}

template <int RPT, bool YLDS>
hipError_t launch_rpt(const Problem& pb, const MstepArgs& a, int nth, size_t lds, hipStream_t s) {
    const int skip = g_chol_skip;                   // diagnostic only (see kernel)
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

}  // namespace

// mode 1: time the launches of the following M-steps (events created once); mode 0: after the
// caller synchronised, out6 = {update ms, factor ms, back substitution ms, and their launch
// counts}, then timing is switched off
hipError_t chol_debug_timing(int mode, double* out6) {
    if (mode == 1) {
        if (!g_ct.made) {
            for (int i = 0; i < 512; ++i)
                if (hipEventCreate(&g_ct.ev[i]) != hipSuccess) return hipErrorInvalidValue;
            g_ct.made = true;
        }
        g_ct.n = 0;
        g_ct.on = true;
        return hipSuccess;
    }
    g_ct.on = false;
    if (!out6) return hipErrorInvalidValue;
    for (int k = 0; k < 6; ++k) out6[k] = 0.0;
    for (int i = 0; i + 1 < g_ct.n; i += 2) {
        float ms = 0.0f;
        if (hipEventElapsedTime(&ms, g_ct.ev[i], g_ct.ev[i + 1]) != hipSuccess) return hipErrorInvalidValue;
        const int k = g_ct.kind[i / 2];
        out6[k] += ms;
        out6[3 + k] += 1.0;
    }
    return hipSuccess;
}

hipError_t chol_debug_clock(unsigned long long* out) {
    return hipMemcpyFromSymbol(out, HIP_SYMBOL(g_chol_clk), sizeof(g_chol_clk), 0,
                               hipMemcpyDeviceToHost);
}
#if SBCE_AB
void chol_debug_skip(int mask) { g_chol_skip = mask; }
#else
void chol_debug_skip(int) {}
#endif
int chol_debug_skip_mask() { return g_chol_skip; }
hipError_t chol_debug_clock_reset() {
    static const unsigned long long z[32] = {0};
    return hipMemcpyToSymbol(HIP_SYMBOL(g_chol_clk), z, sizeof(z), 0, hipMemcpyHostToDevice);
}

// Every path launches some grid with the batch in grid y (the tiled large-L and min-norm
// factorisations, pilot_rhs_kernel, the small-L R build), so batch <= 65535 for every shape.
bool chol_supported(const Problem& pb) {
    return pb.L >= 1 && pb.L <= kMaxL && pb.B <= 65535;
}

// Factor the w x w diagonal tile at (k0, k0) of every trial's R in place (large-L path).
hipError_t launch_chol_tile(const Problem& pb, const MstepArgs& a, int k0, int w, const int32_t* ext,
                            hipStream_t s) {
    const int ntile = (w + NB - 1) / NB;             // <= 4 -> one 16-row tile per wave
    CholGeom geo;
    geo.ld = pb.L; geo.off = k0; geo.stride = (size_t)pb.L * pb.L; geo.tolp = a.tol; geo.ext = ext;
    const size_t lds = (size_t)(NB * (128 + 1) + NB * NB + ntile * NB * NB) * sizeof(cd) +
                       18 * sizeof(double);
    hipLaunchKernelGGL((chol_mfma_kernel<1, false, 4, 128, false>), dim3(pb.B), dim3(64 * ntile),
                       lds, s, a, w, pb.NR, 0, geo);
    return hipGetLastError();
}

hipError_t launch_chol_solve(const Problem& pb, const MstepArgs& a, hipStream_t s) {
    if (!chol_supported(pb)) return hipErrorInvalidValue;
    if (a.solve_mode == SBCE_SOLVE_MINNORM) return launch_minnorm(pb, a, s);
    const bool force_valu = g_debug.chol_valu;       // SBCE_CHOL_IMPL=valu: VALU cross-check
    if (pb.L > kLargeL && !(force_valu && pb.L <= 1024)) return launch_chol_large(pb, a, s);
    const size_t ybytes = (size_t)pb.L * pb.NR * sizeof(cd);
    if (!force_valu) return launch_chol_batched(pb, a, s);   // batched panel launches
    int nth = (pb.L + 63) / 64 * 64;
    if (nth > 512) nth = 512;
    const int rpt = (pb.L + nth - 1) / nth;
    const size_t base = (size_t)(NB * KC + 2 * NB * NB) * sizeof(cd) + (NB + 18) * sizeof(double);
    if (ybytes <= 48 * 1024) return launch_y<true>(pb, a, nth, rpt, base + ybytes, s);
    return launch_y<false>(pb, a, nth, rpt, base, s);
}

}  // namespace sbce
