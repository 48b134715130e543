// Small-L M-step (L = (N+1) n_tx <= 64, n_tx not in {4, 8}): the whole M-step of one trial in ONE
// workgroup -- R and B^H built, factored and solved in registers, theta written.
//
// Reference: the M-step of "Proposed method/all_detectorsvsTd.py" (its five EMs, :62-96 etc.:
// A = sum Z^H Z, b = sum Z^H y, np.linalg.solve) at BASELINE cfg 5's 2 x 2, N_RIS = 15 shape
// (L = 32), in the reduced form of mstep.hip (R X = B^H, commutation_matrix.py:3-8).
//
// The batched path (rbuild_kernel, rhs_dma_kernel, diag_tol_kernel, panel_factor_kernel,
// backsub4_kernel) spends five launches and four HBM round trips of R per iteration on a
// 32 x 32 system, each launch a few microseconds of latency-bound work per trial.  Here each
// thread owns a fixed set of R's entries and of B^H's from the build to the solve:
//   1. every entry accumulated in rbuild_kernel's / rhs_kernel's operation order (pilot terms,
//      then the data symbols in order; the symbols staged in LDS) -> bitwise their R and B^H;
//   2. tol = 1e-14 max diag R (diag_tol_kernel); right-looking Cholesky with the forward
//      substitution fused: per column ONE barrier, column c and y_c exchanged through a
//      double-buffered LDS vector, every other update on the owner's registers;
//   3. back substitution L^H x = y the same way (row c of L and x_c exchanged); theta = conj(x).
// Pivot rule and status bits are the batched path's (chol.hip factor_diag): a pivot that is not
// above tol is flagged (clamp_status) and its direction dropped (l_cc = 0, its unknowns 0) under
// SBCE_SOLVE_CHOL and CHOL_DROP alike (include/sbce.h).
#include <type_traits>

#include "sbce_internal.h"

namespace sbce {

namespace {

constexpr int kSmallMaxL = 64;
constexpr int kSmallThreads = 256;
constexpr int kStageCd = 2048;                // staged symbols: <= 32 KB of complex doubles
constexpr int kStageMf = 1024;                // the MFMA build's symbol chunks

// ---- MFMA build (P <= 16: every (i, j) block of R is ONE 16 x 16 complex tile) ----
// R_ij[p][q] = sum_t a_t[p] conj(b_t[q]) with a = psi_t[p] S_t[i][j] (data) or u_t[p n_tx + i]
// (pilots), b = psi_t[q] (data) or u_t[q n_tx + j] (pilots): four real v_mfma_f64_16x16x4f64 per
// block and k-step of 4 symbols, lane (li, lk) feeding symbol t0 + lk at index li of both operands
// (the symbols staged in LDS by chunks, all loads of a chunk in flight at once).  B^H rides along
// as an (L x T) x (T x n_rx) product on row tiles of 16.  The NT(NT+1)/2 blocks and NT row tiles
// are spread over the 4 waves.  Results to LDS (R: [L][LD], B^H: [L][NR]) over the staging area.
typedef double d4v __attribute__((ext_vector_type(4)));

__device__ __forceinline__ void cmfma(d4v& cre, d4v& cim, cd x, cd y) {   // C += x * y
    cre = __builtin_amdgcn_mfma_f64_16x16x4f64(x.x, y.x, cre, 0, 0, 0);
    cre = __builtin_amdgcn_mfma_f64_16x16x4f64(-x.y, y.y, cre, 0, 0, 0);
    cim = __builtin_amdgcn_mfma_f64_16x16x4f64(x.x, y.y, cim, 0, 0, 0);
    cim = __builtin_amdgcn_mfma_f64_16x16x4f64(x.y, y.x, cim, 0, 0, 0);
}

template <int N>
__device__ __forceinline__ cd pick(const cd (&v)[N], int i) {   // v[i] without dynamic indexing
    cd r = v[0];
#pragma unroll
    for (int k = 1; k < N; ++k) r = csel(i == k, v[k], r);
    return r;
}

template <int NT, int NR>
__device__ __forceinline__ void mfma_build(const MstepArgs& a, int b, int P, int Tp, int Td, int L,
                                           int LD, cd* stg, int sg, int tid) {
    constexpr int NBLK = NT * (NT + 1) / 2, LT = NT, NIT = NBLK + LT, IPW = (NIT + 3) / 4;
    constexpr int MS = NT + NT * NT;
    const int lane = tid & 63, wave = tid >> 6, li = lane & 15, lk = lane >> 4;
    int bi[IPW], bj[IPW], tq[IPW];                    // item: block (bi, bj) or B^H row tile tq
    d4v cre[IPW], cim[IPW];
#pragma unroll
    for (int s = 0; s < IPW; ++s) {
        const int it = wave + 4 * s;
        bi[s] = 0; bj[s] = 0; tq[s] = -1;
        if (it < NBLK) {
            int i = 0;
            while ((i + 1) * (i + 2) / 2 <= it) ++i;
            bi[s] = i;
            bj[s] = it - i * (i + 1) / 2;
        } else {
            tq[s] = it - NBLK;                       // >= LT: no item
        }
        cre[s] = d4v{0.0, 0.0, 0.0, 0.0};
        cim[s] = cre[s];
    }
    // pilots, TPC symbols (a multiple of 4) per LDS chunk: u_p [TPC][L], y_p [TPC][NR]
    {
        int TPC = (sg / (L + NR)) & ~3;
        if (TPC < 4) TPC = 4;
        const cd* up = a.up + (size_t)b * Tp * L;
        const cd* yp = a.yp + (size_t)b * Tp * NR;
        cd* su = stg;
        cd* sp = stg + TPC * L;
        for (int c0 = 0; c0 < Tp; c0 += TPC) {
            const int tc = (Tp - c0) < TPC ? (Tp - c0) : TPC;
            __syncthreads();
            for (int e = tid; e < tc * L; e += kSmallThreads) su[e] = up[(size_t)c0 * L + e];
            for (int e = tid; e < tc * NR; e += kSmallThreads) sp[e] = yp[(size_t)c0 * NR + e];
            __syncthreads();
            for (int t0 = 0; t0 < tc; t0 += 4) {
                const int t = t0 + lk;
                const bool on = t < tc;
                cd u[NT];
#pragma unroll
                for (int i = 0; i < NT; ++i) u[i] = (on && li < P) ? su[t * L + li * NT + i] : czero();
                const cd yc = (on && li < NR) ? cconj(sp[t * NR + li]) : czero();
#pragma unroll
                for (int s = 0; s < IPW; ++s) {
                    if (tq[s] < 0) {
                        cmfma(cre[s], cim[s], pick(u, bi[s]), cconj(pick(u, bj[s])));
                    } else if (tq[s] < LT) {
                        const int l = 16 * tq[s] + li;
                        cmfma(cre[s], cim[s], (on && l < L) ? su[t * L + l] : czero(), yc);
                    }
                }
            }
        }
    }
    // data symbols, TC (a multiple of 4) per LDS chunk: psi [TC][P], moments [TC][MS], y_d [TC][NR]
    {
        int TC = (sg / (P + MS + NR)) & ~3;
        if (TC < 4) TC = 4;
        const cd* ps = a.psid + (size_t)b * Td * P;
        const cd* mom = a.mom + (size_t)b * Td * MS;
        const cd* yd = a.yd + (size_t)b * Td * NR;
        cd* s_ps = stg;
        cd* s_m = s_ps + TC * P;
        cd* s_y = s_m + TC * MS;
        for (int c0 = 0; c0 < Td; c0 += TC) {
            const int tc = (Td - c0) < TC ? (Td - c0) : TC;
            __syncthreads();
            for (int e = tid; e < tc * P; e += kSmallThreads) s_ps[e] = ps[(size_t)c0 * P + e];
            for (int e = tid; e < tc * MS; e += kSmallThreads) s_m[e] = mom[(size_t)c0 * MS + e];
            for (int e = tid; e < tc * NR; e += kSmallThreads) s_y[e] = yd[(size_t)c0 * NR + e];
            __syncthreads();
            for (int t0 = 0; t0 < tc; t0 += 4) {
                const int t = t0 + lk;
                const bool on = t < tc;
                const cd psi = (on && li < P) ? s_ps[t * P + li] : czero();
                const cd yc = (on && li < NR) ? cconj(s_y[t * NR + li]) : czero();
                cd sv[MS];
#pragma unroll
                for (int e = 0; e < MS; ++e) sv[e] = on ? s_m[t * MS + e] : czero();
#pragma unroll
                for (int s = 0; s < IPW; ++s) {
                    if (tq[s] < 0) {
                        cmfma(cre[s], cim[s], cmul(psi, pick(sv, NT + bi[s] * NT + bj[s])), cconj(psi));
                    } else if (tq[s] < LT) {
                        const int l = 16 * tq[s] + li;
                        const int pl = l / NT, al = l - pl * NT;
                        const cd pv = (on && l < L) ? s_ps[t * P + pl] : czero();
                        cmfma(cre[s], cim[s], cmul(pv, pick(sv, al)), yc);
                    }
                }
            }
        }
    }
    __syncthreads();                                 // every wave is done with the staged symbols
    cd* sR = stg;
    cd* sY = stg + L * LD;
    // lane holds column li, rows lk + 4v of each of its tiles
#pragma unroll
    for (int s = 0; s < IPW; ++s) {
#pragma unroll
        for (int v = 0; v < 4; ++v) {
            const int p = lk + 4 * v;
            const cd c = cmk(cre[s][v], cim[s][v]);
            if (tq[s] < 0) {
                if (p < P && li < P) {
                    sR[(p * NT + bi[s]) * LD + li * NT + bj[s]] = c;
                    if (bi[s] != bj[s]) sR[(li * NT + bj[s]) * LD + p * NT + bi[s]] = cconj(c);
                }
            } else if (tq[s] < LT) {
                const int l = 16 * tq[s] + p;
                if (l < L && li < NR) sY[l * NR + li] = c;
            }
        }
    }
}

// Thread (ti, tj) = (tid / 16, tid % 16) owns the R elements (ti + 16 k1, tj + 16 k2), k1, k2 <
// KB = ceil(L / 16), in registers from the build to the end of the solve; B^H / y entry
// e = tid + 256 k (row e / NR, column e % NR) likewise.  Only column c (forward) or row c (back
// substitution) of L and y_c / x_c cross threads, through a double-buffered LDS vector: one
// barrier per column.
template <int NR, int KB, int MNT>
__device__ __forceinline__ void mstep_small_body(const MstepArgs& a, int NT, int P, int Tp, int Td,
                                                 int L, int write_sys, int stop, int sg) {
    const int b = blockIdx.x;
    if (a.done && a.done[b]) return;
    constexpr int YK = (64 * NR + kSmallThreads - 1) / kSmallThreads;
    extern __shared__ __attribute__((aligned(16))) char smem[];
    cd* stg = reinterpret_cast<cd*>(smem);           // [sg] staged symbols / the MFMA build's R, B^H
    cd* xb = stg + sg;                               // [2][64 + 8] column / row + y_c exchange
    double* dinv = reinterpret_cast<double*>(xb + 2 * (64 + 8));   // [64] 1 / l_cc (0: dropped)
    double* red = dinv + 64;                                      // [4]
    const int tid = threadIdx.x, ti = tid >> 4, tj = tid & 15;
    const int lane = tid & 63, wave = tid >> 6;
    const int MS = NT + NT * NT;

    // ---- 1. R and B^H in registers --------------------------------------------------------------
    // element (i, j) is accumulated as rbuild_kernel's block pair (p, q), p >= q, entry (ia, ja):
    // swapped (and conjugated at the end) when i's block is above j's
    cd A[KB][KB];
    int rr[KB][KB], cc[KB][KB];
    int prr[KB][KB], pcc[KB][KB], sidx[KB][KB];   // rbuild's block pair and S_t entry
    bool need[KB][KB], swp[KB][KB];
#pragma unroll
    for (int k1 = 0; k1 < KB; ++k1)
#pragma unroll
        for (int k2 = 0; k2 < KB; ++k2) {
            const int i = ti + 16 * k1, j = tj + 16 * k2;
            const bool valid = i < L && j < L;
            swp[k1][k2] = valid && (i / NT) < (j / NT);
            need[k1][k2] = valid && (i >= j || write_sys);
            rr[k1][k2] = swp[k1][k2] ? j : i;
            cc[k1][k2] = swp[k1][k2] ? i : j;
            prr[k1][k2] = rr[k1][k2] / NT;
            pcc[k1][k2] = cc[k1][k2] / NT;
            sidx[k1][k2] = NT + (rr[k1][k2] - prr[k1][k2] * NT) * NT + (cc[k1][k2] - pcc[k1][k2] * NT);
            A[k1][k2] = czero();
        }
    cd Y[YK];
    int yl[YK], ypl[YK], yal[YK], yrr[YK];            // row, its block and stream, column
#pragma unroll
    for (int k = 0; k < YK; ++k) {
        yl[k] = (tid + kSmallThreads * k) / NR;
        yrr[k] = tid + kSmallThreads * k - yl[k] * NR;
        ypl[k] = yl[k] / NT;
        yal[k] = yl[k] - ypl[k] * NT;
        Y[k] = czero();
    }

    if constexpr (MNT > 0) {
        const int LD = L + 1;
        mfma_build<MNT, NR>(a, b, P, Tp, Td, L, LD, stg, sg, tid);
        __syncthreads();
#pragma unroll
        for (int k1 = 0; k1 < KB; ++k1)
#pragma unroll
            for (int k2 = 0; k2 < KB; ++k2)
                if (need[k1][k2]) A[k1][k2] = stg[(ti + 16 * k1) * LD + tj + 16 * k2];
#pragma unroll
        for (int k = 0; k < YK; ++k)
            if (yl[k] < L) Y[k] = stg[L * LD + tid + kSmallThreads * k];
    } else {
        // pilots, TPC symbols at a time: u_p [TPC][L], y_p [TPC][NR]
        {
            const int TPC = sg / (L + NR) > 0 ? sg / (L + NR) : 1;
            const cd* up = a.up + (size_t)b * Tp * L;
            const cd* yp = a.yp + (size_t)b * Tp * NR;
            cd* su = stg;
            cd* sp = stg + TPC * L;
            for (int t0 = 0; t0 < Tp; t0 += TPC) {
                const int tc = (Tp - t0) < TPC ? (Tp - t0) : TPC;
                __syncthreads();
                for (int e = tid; e < tc * L; e += kSmallThreads) su[e] = up[(size_t)t0 * L + e];
                for (int e = tid; e < tc * NR; e += kSmallThreads) sp[e] = yp[(size_t)t0 * NR + e];
                __syncthreads();
                for (int tt = 0; tt < (stop == 3 ? 0 : tc); ++tt) {
    #pragma unroll
                    for (int k1 = 0; k1 < KB; ++k1)
    #pragma unroll
                        for (int k2 = 0; k2 < KB; ++k2)
                            if (need[k1][k2])
                                A[k1][k2] = cfmac(A[k1][k2], su[tt * L + rr[k1][k2]], su[tt * L + cc[k1][k2]]);
    #pragma unroll
                    for (int k = 0; k < YK; ++k)
                        if (yl[k] < L) Y[k] = cfmac(Y[k], su[tt * L + yl[k]], sp[tt * NR + yrr[k]]);
                }
            }
        }
        // data symbols, TC at a time: psi [TC][P], moments [TC][MS], y_d [TC][NR]
        {
            const int TC = sg / (P + MS + NR) > 0 ? sg / (P + MS + NR) : 1;
            const cd* ps = a.psid + (size_t)b * Td * P;
            const cd* mom = a.mom + (size_t)b * Td * MS;
            const cd* yd = a.yd + (size_t)b * Td * NR;
            cd* s_ps = stg;
            cd* s_m = s_ps + TC * P;
            cd* s_y = s_m + TC * MS;
            for (int t0 = 0; t0 < Td; t0 += TC) {
                const int tc = (Td - t0) < TC ? (Td - t0) : TC;
                __syncthreads();
                for (int e = tid; e < tc * P; e += kSmallThreads) s_ps[e] = ps[(size_t)t0 * P + e];
                for (int e = tid; e < tc * MS; e += kSmallThreads) s_m[e] = mom[(size_t)t0 * MS + e];
                for (int e = tid; e < tc * NR; e += kSmallThreads) s_y[e] = yd[(size_t)t0 * NR + e];
                __syncthreads();
                for (int tt = 0; tt < (stop == 3 ? 0 : tc); ++tt) {
    #pragma unroll
                    for (int k1 = 0; k1 < KB; ++k1)
    #pragma unroll
                        for (int k2 = 0; k2 < KB; ++k2)
                            if (need[k1][k2]) {
                                const cd w = cmulc(s_ps[tt * P + prr[k1][k2]], s_ps[tt * P + pcc[k1][k2]]);
                                A[k1][k2] = cfma(A[k1][k2], w, s_m[tt * MS + sidx[k1][k2]]);
                            }
    #pragma unroll
                    for (int k = 0; k < YK; ++k)
                        if (yl[k] < L) {
                            const cd w = cmul(s_ps[tt * P + ypl[k]], s_m[tt * MS + yal[k]]);
                            Y[k] = cfmac(Y[k], w, s_y[tt * NR + yrr[k]]);
                        }
                }
            }
        }
    #pragma unroll
        for (int k1 = 0; k1 < KB; ++k1)
    #pragma unroll
            for (int k2 = 0; k2 < KB; ++k2)
                if (swp[k1][k2]) A[k1][k2] = cconj(A[k1][k2]);
    }
    if (write_sys) {                                 // sbce_mstep's r_out / rhs_out
        cd* R = a.R + (size_t)b * L * L;
#pragma unroll
        for (int k1 = 0; k1 < KB; ++k1)
#pragma unroll
            for (int k2 = 0; k2 < KB; ++k2)
                if (need[k1][k2]) R[(size_t)(ti + 16 * k1) * L + tj + 16 * k2] = A[k1][k2];
        cd* rh = a.rhs + (size_t)b * L * NR;
#pragma unroll
        for (int k = 0; k < YK; ++k)
            if (yl[k] < L) rh[tid + kSmallThreads * k] = Y[k];
    }
    if (stop == 1 || stop == 3) return;              // DIAGNOSTIC phase timing (results invalid)

    // ---- 2. tol = 1e-14 max diag R (diag_tol_kernel); Cholesky + forward substitution ------------
    double mx = 0.0;
#pragma unroll
    for (int k = 0; k < KB; ++k)
        if (ti == tj && ti + 16 * k < L) mx = fmax(mx, A[k][k].x);
    for (int off = 32; off >= 1; off >>= 1) mx = fmax(mx, __shfl_xor(mx, off));
    if (lane == 0) red[wave] = mx;
    __syncthreads();
    const double tol = 1e-14 * fmax(fmax(red[0], red[1]), fmax(red[2], red[3]));
    bool anybad = false;
#pragma unroll
    for (int kc = 0; kc < KB; ++kc) {
        for (int cl = 0; cl < 16; ++cl) {
            const int c = 16 * kc + cl;
            if (c >= L) break;
            cd* col = xb + (c & 1) * (64 + 8);
            if (tj == cl) {                          // column c (rows >= c), fully updated
#pragma unroll
                for (int k1 = 0; k1 < KB; ++k1) {
                    const int i = ti + 16 * k1;
                    if (i >= c && i < L) col[i] = A[k1][kc];
                }
            }
#pragma unroll
            for (int k = 0; k < YK; ++k)
                if (yl[k] == c) col[64 + (tid + kSmallThreads * k - c * NR)] = Y[k];
            __syncthreads();
            const double dia = col[c].x;
            const bool bad = !(dia > tol);
            const bool drop = bad;                   // every public mode drops (sbce.h)
            // pivot and its inverse as the batched panel factor forms them (v_rsq_f64 seed, two
            // Newton steps: ~5 dependent ops on the column chain instead of sqrt + division)
            const double pv = bad ? tol : dia;
            const double rs = fast_rsqrt64(pv);
            const double piv = pv * rs;
            const double inv = drop ? 0.0 : rs;
            anybad |= bad;
            if (tid == 0) dinv[c] = inv;
            if (tj == cl) {
#pragma unroll
                for (int k1 = 0; k1 < KB; ++k1) {
                    const int i = ti + 16 * k1;
                    if (i == c) A[k1][kc] = cmk(drop ? 0.0 : piv, 0.0);
                    else if (i > c && i < L) A[k1][kc] = cscale(A[k1][kc], inv);
                }
            }
            cd li[KB], lj[KB];
#pragma unroll
            for (int k = 0; k < KB; ++k) {
                li[k] = cscale(col[(ti + 16 * k) & 63], inv);
                lj[k] = cscale(col[(tj + 16 * k) & 63], inv);
            }
#pragma unroll
            for (int k1 = 0; k1 < KB; ++k1)
#pragma unroll
                for (int k2 = 0; k2 < KB; ++k2) {
                    const int i = ti + 16 * k1, j = tj + 16 * k2;
                    if (j > c && j <= i && i < L) A[k1][k2] = csub(A[k1][k2], cmulc(li[k1], lj[k2]));
                }
#pragma unroll
            for (int k = 0; k < YK; ++k) {
                const int r = tid + kSmallThreads * k - yl[k] * NR;
                if (yl[k] == c) {
                    Y[k] = cscale(Y[k], inv);
                } else if (yl[k] > c && yl[k] < L) {
                    Y[k] = csub(Y[k], cmul(cscale(col[yl[k]], inv), cscale(col[64 + r], inv)));
                }
            }
        }
    }
    if (stop == 2) return;
    // the last forward column's dinv[L-1] and row buffer are read by other waves below
    __syncthreads();

    // ---- 3. back substitution L^H x = y (y_i -= x_c conj(l_ci)), theta = conj(x) ------------------
#pragma unroll
    for (int kc = KB - 1; kc >= 0; --kc) {
        for (int cl = 15; cl >= 0; --cl) {
            const int c = 16 * kc + cl;
            if (c >= L) continue;
            cd* row = xb + (c & 1) * (64 + 8);
            if (ti == cl) {                          // row c of L left of the diagonal
#pragma unroll
                for (int k2 = 0; k2 < KB; ++k2) {
                    const int j = tj + 16 * k2;
                    if (j < c) row[j] = A[kc][k2];
                }
            }
            const double iv = dinv[c];
#pragma unroll
            for (int k = 0; k < YK; ++k)
                if (yl[k] == c) {
                    Y[k] = cscale(Y[k], iv);
                    row[64 + (tid + kSmallThreads * k - c * NR)] = Y[k];
                }
            __syncthreads();
#pragma unroll
            for (int k = 0; k < YK; ++k) {
                const int r = tid + kSmallThreads * k - yl[k] * NR;
                if (yl[k] < c) Y[k] = csub(Y[k], cmulc(row[64 + r], row[yl[k]]));
            }
        }
    }
    cd* th = a.theta + (size_t)b * L * NR;
#pragma unroll
    for (int k = 0; k < YK; ++k)
        if (yl[k] < L) th[tid + kSmallThreads * k] = cconj(Y[k]);
    if (tid == 0 && a.status && anybad) a.status[b] |= a.clamp_status;
}

template <int NR, int KB, int MNT>
__global__ __launch_bounds__(kSmallThreads) void mstep_small_kernel(MstepArgs a, int NT, int P,
                                                                    int Tp, int Td, int L,
                                                                    int write_sys, int stop, int sg) {
    mstep_small_body<NR, KB, MNT>(a, NT, P, Tp, Td, L, write_sys, stop, sg);
}
// n_tx <= 2 MFMA build (BASELINE cfg 5: L = 32, 1280 trials) held to 96 VGPRs (no spills) and
// ~21 KB of LDS: five workgroups per CU, so 1280 trials run in one round instead of two
template <int NR, int KB, int MNT>
__global__ __launch_bounds__(kSmallThreads) __attribute__((amdgpu_waves_per_eu(5))) void
mstep_small5_kernel(MstepArgs a, int NT, int P, int Tp, int Td, int L, int write_sys, int stop, int sg) {
    mstep_small_body<NR, KB, MNT>(a, NT, P, Tp, Td, L, write_sys, stop, sg);
}

// ---- n_tx <= 2, P <= 16, n_rx <= 4 (L <= 32: BASELINE cfg 5), round 6 ---------------------------
// The kernel above spends its time in two places (cfg 5, 1280 trials, five workgroups per CU):
// wave 0 carries two of the five MFMA items (the (0,0) block and a B^H row tile, whose 16 x 16
// tile uses 2 of its 16 columns), so SIMD 0 runs 8 of the 20 MFMAs of every k-step; and the
// factorisation / back substitution take one 256-thread barrier per column (64 barriers).  Here
// two launches:
//   build   (mstep_small2_build_kernel, 4 waves per trial, five trials per CU) wave w < NBLK
//           builds block w of R (the (0,0), (1,0), (1,1) blocks) over ALL symbols, wave NBLK
//           B^H = sum_t (psi_t (x) m_t) y_t^H as one more 16 x (NT NR) MFMA product (the pilots in
//           NT passes, their u_t not being a product); complex products by three real MFMAs
//           (Gauss: P1 = sum xr yr, P2 = sum xi yi, P3 = sum (xr + xi)(yr + yi); re = P1 - P2,
//           im = P3 - P1 - P2); each wave streams its operands from global memory with the raw
//           values of the next k-steps in flight (a staging of the symbols in LDS by 16-symbol
//           chunks, one barrier per chunk, measured slower: 113.6 vs 98.8 us at T_d = 120);
//           R (full) and B^H to the workspace, no barrier;
//   solve   (mstep_small3_solve_kernel below by default -- 4-column panels, MFMA trailing
//           updates; this column-by-column mstep_small2_solve_kernel with SBCE_SMALL_SOLVE=col in
//           the A/B build)
//           (mstep_small2_solve_kernel, ONE wave per trial, no occupancy cap: the row registers,
//           the column values and the right-hand sides stay in VGPRs -- at the build's 96-VGPR
//           cap they went to scratch, one memory round trip per column) right-looking Cholesky
//           with the forward substitution fused, lane (r, h) holding row r's columns 2e + h, a
//           rolled loop over column pairs whose current column is register slot 0, the pivot by
//           v_readlane, the scaled column published through a double-buffered LDS vector and
//           read back in one batch (a branch per slot put every read's latency on the chain), y_c
//           by v_readlane; back substitution with L's rows from LDS; theta = conj(x).
// The oracle early stop (|‖theta‖ - ‖h‖| < 1, early_stop_kernel) is folded into the solve's
// epilogue when a.h_true is set.  Pivot rule and status as factor_diag (a pivot not above 1e-14
// max diag R is flagged and dropped).
// right-hand side h + 2k of a lane's half h: the entry of v without a lane-dependent index
template <int NR>
__device__ __forceinline__ cd rhs_pick(const cd (&v)[NR], int h, int k) {
    const cd v0 = (2 * k < NR) ? v[(2 * k) < NR ? 2 * k : 0] : czero();
    const cd v1 = (2 * k + 1 < NR) ? v[(2 * k + 1) < NR ? 2 * k + 1 : 0] : czero();
    return csel(h != 0, v1, v0);
}

// DIAGNOSTIC (SBCE_SMALL_STOP=4, results unchanged): s_memtime stamps of trial 0's solve wave --
// [0] start, [1] loads done, [2] tol, [3 + k] column pair k factored, [40] factor done, [41] back
// substitution done (tools/small_clock.py)
__device__ unsigned long long g_small_clk[48];

template <int NT, int NR>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(5))) void
mstep_small2_build_kernel(MstepArgs a, int P, int Tp, int Td, int L) {
    const int b = blockIdx.x;
    if (a.done && a.done[b]) return;
    constexpr int NBLK = NT * (NT + 1) / 2;
    constexpr int MS = NT + NT * NT;
    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int T = Tp + Td;
    const cd* up = a.up + (size_t)b * Tp * L;
    const cd* yp = a.yp + (size_t)b * Tp * NR;
    const cd* ps = a.psid + (size_t)b * Td * P;
    const cd* mom = a.mom + (size_t)b * Td * MS;
    const cd* yd = a.yd + (size_t)b * Td * NR;
    cd* R = a.R + (size_t)b * L * L;
    cd* rh = a.rhs + (size_t)b * L * NR;
    const int role = (wave + b) & 3;                 // rotates the roles over the SIMDs
    const int li = lane & 15, lk = lane >> 4;
    const bool lon = li < P;
    // this wave's product: block (bi, bj) of R (role < NBLK) or B^H (role NBLK, bh)
    const bool bh = role == NBLK;
    const int bi = role >= 1 ? 1 : 0, bj = role == 2 ? 1 : 0;
    const int ca = li / NR, cr = li - ca * NR;      // B^H: column (a, r) of the product
    const bool con = li < NT * NR;
    const int VP = bh ? NT * Tp : Tp;                // virtual symbols: pilot slots, then data
    const int V = VP + Td;
    d4v p1 = {0.0, 0.0, 0.0, 0.0}, p2 = p1, p3 = p1;
    auto mfma3 = [&](cd x, cd y) {
        p1 = __builtin_amdgcn_mfma_f64_16x16x4f64(x.x, y.x, p1, 0, 0, 0);
        p2 = __builtin_amdgcn_mfma_f64_16x16x4f64(x.y, y.y, p2, 0, 0, 0);
        p3 = __builtin_amdgcn_mfma_f64_16x16x4f64(x.x + x.y, y.x + y.y, p3, 0, 0, 0);
    };
    {
        // Each role streams its operands: the pilots, then the data symbols, each with the raw
        // values of the next KD k-steps in flight in registers; loads never branch (indices
        // clamped, invalid lanes / symbols zeroed by select), addresses advance by increments
        const int lc = lon ? li : 0;
        if (role < NBLK) {
            // block (bi, bj) of R: A = u_t[p NT + bi] / psi_t[p] S_t[bi][bj],
            //                      B = conj(u_t[q NT + bj]) / conj(psi_t[q])
            constexpr int KD = 3;
            cd ra[KD], rc[KD];
            {   // pilots
                const cd* pa = up + lc * NT + bi;
                const cd* pb = up + lc * NT + bj;
                auto raw = [&](int t, cd& x, cd& y) {
                    const int tt = t < Tp ? t : (Tp > 0 ? Tp - 1 : 0);
                    const bool ok = lon && t < Tp;
                    const cd u1 = Tp > 0 ? pa[(size_t)tt * L] : czero();
                    const cd u2 = Tp > 0 ? pb[(size_t)tt * L] : czero();
                    x = csel(ok, u1, czero());
                    y = csel(ok, u2, czero());
                };
#pragma unroll
                for (int d = 0; d < KD; ++d) raw(4 * d + lk, ra[d], rc[d]);
                for (int t0 = 0; t0 < Tp; t0 += 4 * KD) {
#pragma unroll
                    for (int d = 0; d < KD; ++d) {
                        const cd x = ra[d], y = cconj(rc[d]);
                        raw(t0 + 4 * (KD + d) + lk, ra[d], rc[d]);
                        mfma3(x, y);
                    }
                }
            }
            {   // data
                const cd* pp = ps + lc;
                const cd* pm = mom + NT + bi * NT + bj;
                auto raw = [&](int t, cd& x, cd& y) {
                    const int tt = t < Td ? t : Td - 1;
                    const bool ok = lon && t < Td;
                    x = csel(ok, pp[(size_t)tt * P], czero());
                    y = pm[(size_t)tt * MS];
                };
#pragma unroll
                for (int d = 0; d < KD; ++d) raw(4 * d + lk, ra[d], rc[d]);
                for (int t0 = 0; t0 < Td; t0 += 4 * KD) {
#pragma unroll
                    for (int d = 0; d < KD; ++d) {
                        const cd x = cmul(ra[d], rc[d]), y = cconj(ra[d]);
                        raw(t0 + 4 * (KD + d) + lk, ra[d], rc[d]);
                        mfma3(x, y);
                    }
                }
            }
        } else if (bh) {
            // B^H[(p, a)][r] (column a NR + r of a 16 x (NT NR) product): A = psi_t[p] / u_t[p NT +
            // ap] (one pilot pass per stream ap), B = m_t[a] conj(y_t[r]) / conj(y_p,t[r]) in the
            // columns of a = ap
            constexpr int KD = 2;
            const int cc = con ? ca : 0, rc2 = con ? cr : 0;
            cd ra[KD], rm[KD], ry[KD];
            for (int ap = 0; ap < NT; ++ap) {        // pilots
                const cd* pa = up + lc * NT + ap;
                const cd* py = yp + rc2;
                const bool col_on = con && ca == ap;
                auto raw = [&](int t, cd& x, cd& m, cd& y) {
                    const int tt = t < Tp ? t : (Tp > 0 ? Tp - 1 : 0);
                    const bool ok = t < Tp;
                    const cd u = Tp > 0 ? pa[(size_t)tt * L] : czero();
                    const cd yv = Tp > 0 ? py[(size_t)tt * NR] : czero();
                    x = csel(ok && lon, u, czero());
                    m = cmk(ok && col_on ? 1.0 : 0.0, 0.0);
                    y = yv;
                };
#pragma unroll
                for (int d = 0; d < KD; ++d) raw(4 * d + lk, ra[d], rm[d], ry[d]);
                for (int t0 = 0; t0 < Tp; t0 += 4 * KD) {
#pragma unroll
                    for (int d = 0; d < KD; ++d) {
                        const cd x = ra[d], y = cmulc(rm[d], ry[d]);
                        raw(t0 + 4 * (KD + d) + lk, ra[d], rm[d], ry[d]);
                        mfma3(x, y);
                    }
                }
            }
            {   // data
                const cd* pp = ps + lc;
                const cd* pm = mom + cc;
                const cd* py = yd + rc2;
                auto raw = [&](int t, cd& x, cd& m, cd& y) {
                    const int tt = t < Td ? t : Td - 1;
                    const bool ok = t < Td;
                    x = csel(ok && lon, pp[(size_t)tt * P], czero());
                    m = csel(ok && con, pm[(size_t)tt * MS], czero());
                    y = py[(size_t)tt * NR];
                };
#pragma unroll
                for (int d = 0; d < KD; ++d) raw(4 * d + lk, ra[d], rm[d], ry[d]);
                for (int t0 = 0; t0 < Td; t0 += 4 * KD) {
#pragma unroll
                    for (int d = 0; d < KD; ++d) {
                        const cd x = ra[d], y = cmulc(rm[d], ry[d]);
                        raw(t0 + 4 * (KD + d) + lk, ra[d], rm[d], ry[d]);
                        mfma3(x, y);
                    }
                }
            }
        }
    }
#pragma unroll
    for (int v = 0; v < 4; ++v) {                    // lane holds C[lk + 4v][li]
        const int p = lk + 4 * v, q = li;
        const cd c = cmk(p1[v] - p2[v], p3[v] - p1[v] - p2[v]);
        if (role < NBLK && p < P && q < P) {
            R[(size_t)(p * NT + bi) * L + q * NT + bj] = c;
            if (bi != bj) R[(size_t)(q * NT + bj) * L + p * NT + bi] = cconj(c);
        } else if (bh && p < P && con) {
            rh[(p * NT + ca) * NR + cr] = c;
        }
    }
}

template <int NR>
__global__ __launch_bounds__(64) void mstep_small2_solve_kernel(MstepArgs a, int L, int stop) {
    const int b = blockIdx.x;
    // the next E-step's list counters (its first kernel runs after this launch: stream order)
    if (a.zero_cnt && b == 0 && threadIdx.x < 5) a.zero_cnt[threadIdx.x] = 0;
    if (a.done && a.done[b]) return;
    const unsigned long long clk0 = __builtin_amdgcn_s_memtime();
    constexpr int LDR = 33;
    __shared__ cd sL[32 * LDR];                      // L's rows for the back substitution
    __shared__ cd colb[2][64];                       // column c (rows 0..31; 32..63 padding)
    __shared__ double dinv[32];
    const int lane = threadIdx.x;
    const bool clk = stop == 4 && b == 0 && lane == 0;
    const cd* Rg = a.R + (size_t)b * L * L;
    const cd* rh = a.rhs + (size_t)b * L * NR;
    // ---- lane (r, h): row r, columns 2e + h -----------------------------------------------------
    const int r = lane & 31, h = lane >> 5;
    const bool rin = r < L;
    cd A[16];
#pragma unroll
    for (int e = 0; e < 16; ++e) {
        const int j = 2 * e + h;
        A[e] = (rin && j <= r) ? Rg[(size_t)r * L + j] : czero();
    }
    cd Y[2];
#pragma unroll
    for (int k = 0; k < 2; ++k) {
        const int rr = h + 2 * k;
        Y[k] = (rin && rr < NR) ? rh[r * NR + rr] : czero();
    }
    double dg = 0.0;                                 // the diagonal, on lane (r, r & 1)
#pragma unroll
    for (int e = 0; e < 16; ++e) dg = (rin && 2 * e + h == r) ? A[e].x : dg;
    if (clk) {
        g_small_clk[0] = clk0;
        g_small_clk[1] = __builtin_amdgcn_s_memtime();
    }
    const double tol = 1e-14 * wave_max_dpp(dg);
    bool anybad = false;
    if (clk) g_small_clk[2] = __builtin_amdgcn_s_memtime();
    colb[0][lane] = czero();                         // the padding rows stay finite
    colb[1][lane] = czero();
    // The trailing update touches every slot of every lane (no per-slot predicate): the slots
    // past a row's diagonal and the rows at or above the current column only ever hold products
    // of bounded factor entries, and nothing reads them -- pivots come from the diagonal slot,
    // the published column from rows below it, L's stored rows from slots on or below the
    // diagonal.  Only slot 0 is excluded where it holds a finished column.  ~4 FMAs per slot
    // instead of ~14 instructions.
#pragma unroll 1
    for (int k = 0; 2 * k < L; ++k) {
#pragma unroll
        for (int hc = 0; hc < 2; ++hc) {
            const int c = 2 * k + hc;
            if (c >= L) break;                       // wave-uniform
            const double d = lane_d(A[0].x, c + 32 * hc);
            const bool bad = !(d > tol);
            anybad |= bad;
            const double pv = bad ? tol : d;
            const double rs = fast_rsqrt64(pv);
            const double inv = bad ? 0.0 : rs;       // dropped direction (sbce.h SBCE_SOLVE_CHOL)
            cd* col = colb[hc];
            if (h == hc && r >= c) {
                const cd v = r == c ? cmk(bad ? 0.0 : pv * rs, 0.0) : cscale(A[0], inv);
                A[0] = v;
                if (r > c) col[r] = v;
            }
            if (lane == 0) dinv[c] = inv;
            if (r == c) {
                Y[0] = cscale(Y[0], inv);
                Y[1] = cscale(Y[1], inv);
            }
            cd yc[NR];
#pragma unroll
            for (int rr = 0; rr < NR; ++rr)
                yc[rr] = cmk(lane_d(Y[rr >> 1].x, c + 32 * (rr & 1)), lane_d(Y[rr >> 1].y, c + 32 * (rr & 1)));
            wave_sync();
            const cd lr = col[r];                    // rows <= c: stale, only garbage slots use it
            const cd* cb = col + 2 * k + h;          // slot e <-> column 2 (k + e) + h
            // slots past 15 - k hold columns >= 32, past every row: the update runs over the first
            // 16 / 12 / 8 / 4 slots (a wave-uniform choice of four static slot ranges)
            auto upd = [&](auto ns) {
                constexpr int N = decltype(ns)::value;
                cd cv[N];
#pragma unroll
                for (int e = 0; e < N; ++e) cv[e] = cb[2 * e];
#pragma unroll
                for (int e = 0; e < N; ++e) {
                    // slot 0 is column 2k + h: the current column (h == hc) or, at hc = 1, the
                    // finished column 2k of half 0 -- only at hc = 0 does half 1's slot 0 trail
                    if (e == 0 && !(hc == 0 && h == 1)) continue;
                    // A -= lr conj(cv): four FMAs
                    A[e].x = fma(-lr.x, cv[e].x, A[e].x);
                    A[e].x = fma(-lr.y, cv[e].y, A[e].x);
                    A[e].y = fma(-lr.y, cv[e].x, A[e].y);
                    A[e].y = fma(lr.x, cv[e].y, A[e].y);
                }
            };
            const int emax = 15 - k;
            if (emax >= 12) upd(std::integral_constant<int, 16>());
            else if (emax >= 8) upd(std::integral_constant<int, 12>());
            else if (emax >= 4) upd(std::integral_constant<int, 8>());
            else upd(std::integral_constant<int, 4>());
            if (rin && r > c) {
#pragma unroll
                for (int q = 0; q < 2; ++q) {
                    const int rr = h + 2 * q;
                    if (rr < NR) Y[q] = csub(Y[q], cmul(lr, rhs_pick(yc, h, q)));
                }
            }
        }
        if (clk) g_small_clk[3 + k] = __builtin_amdgcn_s_memtime();
        if (rin && 2 * k + h <= r) sL[r * LDR + 2 * k + h] = A[0];
#pragma unroll
        for (int e = 0; e < 15; ++e) A[e] = A[e + 1];
    }
    if (clk) g_small_clk[40] = __builtin_amdgcn_s_memtime();
    // ---- back substitution L^H x = y: x_c = y_c / l_cc, then y_r -= conj(L[c][r]) x_c, r < c ----
    wave_sync();
    // the next column's 1 / l_cc and L row are read one column ahead (off the x_c chain)
    double iv_n = dinv[L - 1];
    cd lcr_n = sL[(L - 1) * LDR + (r & 31)];
#pragma unroll 1
    for (int c = L - 1; c >= 0; --c) {
        const double iv = iv_n;
        const cd lcr = lcr_n;
        const int cp = c > 0 ? c - 1 : 0;
        iv_n = dinv[cp];
        lcr_n = sL[cp * LDR + (r & 31)];
        if (r == c) {
            Y[0] = cscale(Y[0], iv);
            Y[1] = cscale(Y[1], iv);
        }
        cd xc[NR];
#pragma unroll
        for (int rr = 0; rr < NR; ++rr)
            xc[rr] = cmk(lane_d(Y[rr >> 1].x, c + 32 * (rr & 1)), lane_d(Y[rr >> 1].y, c + 32 * (rr & 1)));
#pragma unroll
        for (int q = 0; q < 2; ++q) {
            const int rr = h + 2 * q;
            if (rr < NR) Y[q] = csel(r < c, csub(Y[q], cmulc(rhs_pick(xc, h, q), lcr)), Y[q]);
        }
    }
    if (clk) g_small_clk[41] = __builtin_amdgcn_s_memtime();
    cd* th = a.theta + (size_t)b * L * NR;
    double nt = 0.0;
#pragma unroll
    for (int k = 0; k < 2; ++k) {
        const int rr = h + 2 * k;
        if (rin && rr < NR) {
            th[r * NR + rr] = cconj(Y[k]);
            nt += cabs2(Y[k]);
        }
    }
    if (a.h_true) {                                  // the oracle early stop (early_stop_kernel)
        const int K = L * NR;
        double nh = 0.0;
        for (int e = lane; e < K; e += 64) nh += cabs2(a.h_true[(size_t)b * K + e]);
        nt = wave_sum_dpp(nt);
        nh = wave_sum_dpp(nh);
        if (lane == 0) {
            if (a.iters_done) a.iters_done[b] = a.it + 1;
            if (a.it != 0 && fabs(sqrt(nt) - sqrt(nh)) < 1.0) a.done_w[b] = 1;
        }
    }
    if (lane == 0 && a.status && anybad) a.status[b] |= a.clamp_status;
}

// Blocked variant of the solve (round 6, the default): the column kernel above issues ~250
// instructions per column (64 FMAs of trailing update + the slot bookkeeping) and is issue-bound
// at ~1250 cycles a column.  Here the trailing matrix lives in MFMA accumulator layout -- the
// lower 16 x 16 tiles (0,0), (1,0), (1,1) of R, lane (li, lk) holding C[lk + 4v][li] -- and the
// factorisation goes by panels of 4 columns:
//   1. the panel's 4 columns leave the accumulators through LDS (P[row][j]) and land one row
//      per lane (rows on lanes 0..31, mirrored on 32..63, which carry the other right-hand
//      sides: lane (r, h) holds y's components h, h + 2 of row r);
//   2. 4 columns factored there: pivot by v_readlane, l_{rc} = a_{rc} / sqrt(d), the panel's
//      later columns updated with l_{c+j,c} by v_readlane, y forward-substituted (y_c by
//      v_readlane); L's rows to LDS (sL) for the back substitution;
//   3. the trailing tiles updated by the panel: C -= L_p L_p^H as four real
//      v_mfma_f64_16x16x4f64 per tile (k = the panel's 4 columns), operands from LDS.
// Entries above the trailing part (finished rows / columns) take garbage updates that nothing
// reads, as in the column kernel.  Pivot rule, dropped directions, status, the early stop, the
// back substitution and theta are the column kernel's.
template <int NR>
__global__ __launch_bounds__(64) void mstep_small3_solve_kernel(MstepArgs a, int L, int stop) {
    const int b = blockIdx.x;
    if (a.zero_cnt && b == 0 && threadIdx.x < 5) a.zero_cnt[threadIdx.x] = 0;
    if (a.done && a.done[b]) return;
    const unsigned long long clk0 = __builtin_amdgcn_s_memtime();
    constexpr int LDR = 33;
    __shared__ cd sL[32 * LDR];                      // L's rows for the back substitution
    __shared__ cd P[32 * 4];                         // the panel, row-major
    __shared__ double dinv[32];
    const int lane = threadIdx.x;
    const bool clk = stop == 4 && b == 0 && lane == 0;
    const cd* Rg = a.R + (size_t)b * L * L;
    const cd* rh = a.rhs + (size_t)b * L * NR;
    const int li = lane & 15, lk = lane >> 4;
    // ---- trailing matrix: tiles (0,0), (1,0), (1,1) as [re, im] accumulators --------------------
    d4v cre[3], cim[3];
#pragma unroll
    for (int t = 0; t < 3; ++t) {
        const int ti = t == 0 ? 0 : 1, tj = t == 2 ? 1 : 0;
#pragma unroll
        for (int v = 0; v < 4; ++v) {
            const int rr = 16 * ti + lk + 4 * v, cc = 16 * tj + li;
            const cd x = (rr < L && cc < L) ? Rg[(size_t)rr * L + cc] : czero();
            cre[t][v] = x.x;
            cim[t][v] = x.y;
        }
    }
    // ---- lane (r, h): row r of the panel, y components h, h + 2 ----------------------------------
    const int r = lane & 31, h = lane >> 5;
    const bool rin = r < L;
    cd Y[2];
#pragma unroll
    for (int k = 0; k < 2; ++k) {
        const int rr = h + 2 * k;
        Y[k] = (rin && rr < NR) ? rh[r * NR + rr] : czero();
    }
    // tol = 1e-14 max diag R: the diagonal sits in tiles 0 and 2 at lane li = lk + 4v
    double dg = 0.0;
#pragma unroll
    for (int v = 0; v < 4; ++v) {
        const bool on = li == lk + 4 * v;
        dg = fmax(dg, on && lk + 4 * v < L ? cre[0][v] : 0.0);
        dg = fmax(dg, on && 16 + lk + 4 * v < L ? cre[2][v] : 0.0);
    }
    if (clk) {
        g_small_clk[0] = clk0;
        g_small_clk[1] = __builtin_amdgcn_s_memtime();
    }
    const double tol = 1e-14 * wave_max_dpp(dg);
    bool anybad = false;
    if (clk) g_small_clk[2] = __builtin_amdgcn_s_memtime();
#pragma unroll 1
    for (int p = 0; 4 * p < L; ++p) {
        const int c0 = 4 * p;
        const bool lo = c0 < 16;                     // wave-uniform: the panel's tile column
        const int lc0 = c0 & 15;
        // 1. the panel's columns out of the accumulators: lanes li in [lc0, lc0 + 4)
        if (li >= lc0 && li < lc0 + 4) {
            const int j = li - lc0;
#pragma unroll
            for (int v = 0; v < 4; ++v) {
                const int rr = lk + 4 * v;
                if (lo) {
                    P[rr * 4 + j] = cmk(cre[0][v], cim[0][v]);
                    P[(16 + rr) * 4 + j] = cmk(cre[1][v], cim[1][v]);
                } else {
                    P[(16 + rr) * 4 + j] = cmk(cre[2][v], cim[2][v]);
                }
            }
        }
        wave_sync();
        cd pv[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) pv[j] = P[r * 4 + j];
        // 2. factor the panel's columns (rows >= c meaningful), forward substitution
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const int c = c0 + j;
            if (c < L) {                             // wave-uniform
            const double d = lane_d(pv[j].x, c);
            const bool bad = !(d > tol);
            anybad |= bad;
            const double pvt = bad ? tol : d;
            const double rs = fast_rsqrt64(pvt);
            const double inv = bad ? 0.0 : rs;       // dropped direction (sbce.h SBCE_SOLVE_CHOL)
            pv[j] = r == c ? cmk(bad ? 0.0 : pvt * rs, 0.0) : cscale(pv[j], inv);
            if (lane == 0) dinv[c] = inv;
            if (r == c) {
                Y[0] = cscale(Y[0], inv);
                Y[1] = cscale(Y[1], inv);
            }
            cd yc[NR];
#pragma unroll
            for (int rr = 0; rr < NR; ++rr)
                yc[rr] = cmk(lane_d(Y[rr >> 1].x, c + 32 * (rr & 1)), lane_d(Y[rr >> 1].y, c + 32 * (rr & 1)));
            if (rin && r > c) {
#pragma unroll
                for (int q = 0; q < 2; ++q) {
                    const int rr = h + 2 * q;
                    if (rr < NR) Y[q] = csub(Y[q], cmul(pv[j], rhs_pick(yc, h, q)));
                }
            }
            // the panel's later columns: a_{r,c'} -= l_{r,c} conj(l_{c',c})
#pragma unroll
            for (int j2 = j + 1; j2 < 4; ++j2) {
                const cd cv = cmk(lane_d(pv[j].x, c0 + j2), lane_d(pv[j].y, c0 + j2));
                pv[j2].x = fma(-pv[j].x, cv.x, pv[j2].x);
                pv[j2].x = fma(-pv[j].y, cv.y, pv[j2].x);
                pv[j2].y = fma(-pv[j].y, cv.x, pv[j2].y);
                pv[j2].y = fma(pv[j].x, cv.y, pv[j2].y);
            }
            }
        }
        if (clk) g_small_clk[3 + p] = __builtin_amdgcn_s_memtime();
        // L's rows for the back substitution; the panel (rows >= c0, zero above) for the MFMAs
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const int c = c0 + j;
            if (h == 0 && rin && c < L && r >= c) sL[r * LDR + c] = pv[j];
        }
        if (4 * (p + 1) >= L) break;                 // wave-uniform: no trailing part left
        wave_sync();
        if (h == 0) {
#pragma unroll
            for (int j = 0; j < 4; ++j) P[r * 4 + j] = r >= c0 + j ? pv[j] : czero();
        }
        wave_sync();
        // 3. trailing tiles -= L_p L_p^H: lane (li, lk) feeds L_p[16 t + li][lk] to both operands
        const cd x0 = P[li * 4 + lk], x1 = P[(16 + li) * 4 + lk];
        auto upd = [&](int t, cd xa, cd xb) {
            cre[t] = __builtin_amdgcn_mfma_f64_16x16x4f64(-xa.x, xb.x, cre[t], 0, 0, 0);
            cre[t] = __builtin_amdgcn_mfma_f64_16x16x4f64(-xa.y, xb.y, cre[t], 0, 0, 0);
            cim[t] = __builtin_amdgcn_mfma_f64_16x16x4f64(-xa.y, xb.x, cim[t], 0, 0, 0);
            cim[t] = __builtin_amdgcn_mfma_f64_16x16x4f64(xa.x, xb.y, cim[t], 0, 0, 0);
        };
        if (lo) {
            upd(0, x0, x0);
            upd(1, x1, x0);
        }
        upd(2, x1, x1);
        wave_sync();                                 // P is rewritten by the next panel
    }
    if (clk) g_small_clk[40] = __builtin_amdgcn_s_memtime();
    // ---- back substitution L^H x = y (the column kernel's) -----------------------------------------
    wave_sync();
    double iv_n = dinv[L - 1];
    cd lcr_n = sL[(L - 1) * LDR + (r & 31)];
#pragma unroll 1
    for (int c = L - 1; c >= 0; --c) {
        const double iv = iv_n;
        const cd lcr = lcr_n;
        const int cp = c > 0 ? c - 1 : 0;
        iv_n = dinv[cp];
        lcr_n = sL[cp * LDR + (r & 31)];
        if (r == c) {
            Y[0] = cscale(Y[0], iv);
            Y[1] = cscale(Y[1], iv);
        }
        cd xc[NR];
#pragma unroll
        for (int rr = 0; rr < NR; ++rr)
            xc[rr] = cmk(lane_d(Y[rr >> 1].x, c + 32 * (rr & 1)), lane_d(Y[rr >> 1].y, c + 32 * (rr & 1)));
#pragma unroll
        for (int q = 0; q < 2; ++q) {
            const int rr = h + 2 * q;
            if (rr < NR) Y[q] = csel(r < c, csub(Y[q], cmulc(rhs_pick(xc, h, q), lcr)), Y[q]);
        }
    }
    if (clk) g_small_clk[41] = __builtin_amdgcn_s_memtime();
    cd* th = a.theta + (size_t)b * L * NR;
    double nt = 0.0;
#pragma unroll
    for (int k = 0; k < 2; ++k) {
        const int rr = h + 2 * k;
        if (rin && rr < NR) {
            th[r * NR + rr] = cconj(Y[k]);
            nt += cabs2(Y[k]);
        }
    }
    if (a.h_true) {                                  // the oracle early stop (early_stop_kernel)
        const int K = L * NR;
        double nh = 0.0;
        for (int e = lane; e < K; e += 64) nh += cabs2(a.h_true[(size_t)b * K + e]);
        nt = wave_sum_dpp(nt);
        nh = wave_sum_dpp(nh);
        if (lane == 0) {
            if (a.iters_done) a.iters_done[b] = a.it + 1;
            if (a.it != 0 && fabs(sqrt(nt) - sqrt(nh)) < 1.0) a.done_w[b] = 1;
        }
    }
    if (lane == 0 && a.status && anybad) a.status[b] |= a.clamp_status;
}

template <int KB, int MNT>
hipError_t launch_nr(const Problem& pb, const MstepArgs& a, size_t lds, int write_sys, int sg,
                     hipStream_t s) {
    switch (pb.NR) {
#define SBCE_MS(n) case n: \
    if constexpr (MNT == 2 && n <= 4) \
        hipLaunchKernelGGL((mstep_small5_kernel<n, KB, MNT>), dim3(pb.B), dim3(kSmallThreads), lds, s, a, pb.NT, pb.P, pb.Tp, pb.Td, pb.L, write_sys, g_debug.small_stop, sg); \
    else \
        hipLaunchKernelGGL((mstep_small_kernel<n, KB, MNT>), dim3(pb.B), dim3(kSmallThreads), lds, s, a, pb.NT, pb.P, pb.Tp, pb.Td, pb.L, write_sys, g_debug.small_stop, sg); \
    break;
        SBCE_MS(1) SBCE_MS(2) SBCE_MS(3) SBCE_MS(4) SBCE_MS(5) SBCE_MS(6) SBCE_MS(7) SBCE_MS(8)
#undef SBCE_MS
        default: return hipErrorInvalidValue;
    }
    return hipGetLastError();
}

}  // namespace

// the round-6 kernel (mstep_small2_kernel): n_tx <= 2, P <= 16, n_rx <= 4
bool mstep_small2_selected(const Problem& pb) {
    return pb.P <= 16 && pb.NT <= 2 && pb.NR <= 4 && pb.L <= 32 && !g_debug.small_valu &&
           g_debug.small_stop != 3 && !g_debug.small_v1;
}

hipError_t small_debug_clock(unsigned long long* out48) {
    return hipMemcpyFromSymbol(out48, HIP_SYMBOL(g_small_clk), sizeof(g_small_clk), 0,
                               hipMemcpyDeviceToHost);
}

bool mstep_small_supported(const Problem& pb, int solve_mode) {
    return !g_debug.mstep_nosmall && !g_debug.chol_valu && chol_debug_skip_mask() == 0 &&
           (solve_mode == SBCE_SOLVE_CHOL || solve_mode == SBCE_SOLVE_CHOL_DROP) &&
           pb.L >= 1 && pb.L <= kSmallMaxL && pb.NR >= 1 && pb.NR <= 8 &&
           !rbuild_herm_supported(pb);
}

hipError_t launch_mstep_small(const Problem& pb, const MstepArgs& a, bool write_sys, hipStream_t s) {
    const int w = write_sys ? 1 : 0;
    if (mstep_small2_selected(pb)) {
        // build (R and B^H to the workspace), then the one-wave solve; the early stop (a.h_true)
        // rides in the solve launch
        MstepArgs ab = a;
        switch (pb.NT * 8 + pb.NR) {
#define SBCE_MS2(nt, nr) case nt * 8 + nr: \
    hipLaunchKernelGGL((mstep_small2_build_kernel<nt, nr>), dim3(pb.B), dim3(256), 0, s, ab, pb.P, pb.Tp, pb.Td, pb.L); \
    break;
            SBCE_MS2(1, 1) SBCE_MS2(1, 2) SBCE_MS2(1, 3) SBCE_MS2(1, 4)
            SBCE_MS2(2, 1) SBCE_MS2(2, 2) SBCE_MS2(2, 3) SBCE_MS2(2, 4)
#undef SBCE_MS2
            default: return hipErrorInvalidValue;
        }
        if (g_debug.small_stop == 1) return hipGetLastError();      // DIAGNOSTIC: build only
        switch (pb.NR) {
#define SBCE_MS2S(nr) case nr: \
    if (g_debug.small_col) \
        hipLaunchKernelGGL((mstep_small2_solve_kernel<nr>), dim3(pb.B), dim3(64), 0, s, a, pb.L, g_debug.small_stop); \
    else \
        hipLaunchKernelGGL((mstep_small3_solve_kernel<nr>), dim3(pb.B), dim3(64), 0, s, a, pb.L, g_debug.small_stop); \
    break;
            SBCE_MS2S(1) SBCE_MS2S(2) SBCE_MS2S(3) SBCE_MS2S(4)
#undef SBCE_MS2S
            default: return hipErrorInvalidValue;
        }
        return hipGetLastError();
    }
    const int KB = (pb.L + 15) / 16;
    // P <= 16 (BASELINE cfg 5): the MFMA build, R and B^H through LDS; else the VALU build
    const bool mf = pb.P <= 16 && pb.NT <= 3 && !g_debug.small_valu && g_debug.small_stop == 0;
    // the MFMA build's staging area also holds its R / B^H result; its symbol chunks are kept to
    // 1024 complex values (five workgroups per CU at cfg 5)
    int sg = mf ? kStageMf : kStageCd;
    if (mf && pb.L * (pb.L + 1) + pb.L * pb.NR > sg) sg = pb.L * (pb.L + 1) + pb.L * pb.NR;
    const size_t lds = ((size_t)sg + 2 * (64 + 8)) * sizeof(cd) + (64 + 4) * sizeof(double);
    if (mf) {
        switch (pb.NT * 8 + KB) {
            case 1 * 8 + 1: return launch_nr<1, 1>(pb, a, lds, w, sg, s);
            case 2 * 8 + 1: return launch_nr<1, 2>(pb, a, lds, w, sg, s);
            case 2 * 8 + 2: return launch_nr<2, 2>(pb, a, lds, w, sg, s);
            case 3 * 8 + 1: return launch_nr<1, 3>(pb, a, lds, w, sg, s);
            case 3 * 8 + 2: return launch_nr<2, 3>(pb, a, lds, w, sg, s);
            case 3 * 8 + 3: return launch_nr<3, 3>(pb, a, lds, w, sg, s);
        }
        return hipErrorInvalidValue;
    }
    switch (KB) {
        case 1: return launch_nr<1, 0>(pb, a, lds, w, sg, s);
        case 2: return launch_nr<2, 0>(pb, a, lds, w, sg, s);
        case 3: return launch_nr<3, 0>(pb, a, lds, w, sg, s);
        case 4: return launch_nr<4, 0>(pb, a, lds, w, sg, s);
    }
    return hipErrorInvalidValue;
}

}  // namespace sbce
