// Batched Hermitian solve of the reduced M-step system  R X = B^H  (one trial per
// workgroup), replacing np.linalg.solve ("Proposed method/Proposed_method_NMSEvsTp.py":80,
// LAPACK zgesv on the K x K system) by a Cholesky factorisation of the L x L
// Hermitian R (commutation_matrix.py:3-8 identity, SURVEY.md §8 preamble).
//
// Design (gfx950): left-looking blocked Cholesky, panel width NB = 16, with the
// panel REGISTER-resident: thread t owns panel rows t, t+nth, ... (RPT rows), so
//   * the left-looking update  A[i, jb:jb+16] -= L[i, 0:jb] L[jb:jb+16, 0:jb]^H
//     streams the thread's own row of L (contiguous) against a 16 x KC top block
//     staged in LDS (broadcast reads);
//   * the 16 x 16 diagonal block is factored by ONE wave in LDS (wave-level
//     syncs only), which also forward-solves the 16-row block of y = L^{-1} B^H;
//   * every other panel row does its own 16-wide triangular solve and its
//     y update in registers (no barriers);
// so a panel costs 2 barriers per KC-chunk of the update plus 3, instead of
// 2 per column.  The back substitution L^H x = y is blocked by 16 the same way.
// Pivots <= 1e-14 * max(diag R) are flagged (status bit 0); solve_mode DROP
// zeroes that direction, CHOL clamps the pivot to the tolerance.
#include <stdlib.h>

#include "sbce_internal.h"

namespace sbce {

namespace {

constexpr int NB = 16;   // panel width (columns)
constexpr int KC = 32;   // k-chunk of the left-looking update

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

    // ---- tolerance from max diag(R); y = B^H ----
    double mx = 0.0;
    for (int i = tid; i < L; i += nth) mx = fmax(mx, R[(size_t)i * L + i].x);
    for (int off = 32; off >= 1; off >>= 1) mx = fmax(mx, shfl_xor_d(mx, off));
    if (lane == 0) red[wave] = mx;
    if (YLDS) {
        const cd* rhs = a.rhs + (size_t)b * L * NR;
        for (int e = tid; e < L * NR; e += nth) y[e] = rhs[e];
    }
    if (tid == 0) *flag = 0;
    __syncthreads();
    double tol = 0.0;
    for (int w = 0; w < (nth >> 6); ++w) tol = fmax(tol, red[w]);
    tol *= 1e-14;

    // ================= factorisation + fused forward substitution =================
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
        // ---- diagonal block: factored in wave-0 REGISTERS (lane r < w holds row r, in place) ----
        if (wave == 0 && !(skip & 2)) {
            cd* dr = row[0];
            const bool mine = lane < w;
            cd* colbuf = Di;      // scratch until the inverse is built
#pragma unroll
            for (int c = 0; c < NB; ++c) {
                if (c < w) {
                    if (lane == c) colbuf[NB] = dr[c];
                    wave_sync();
                    const double dia = colbuf[NB].x;
                    const bool bad = !(dia > tol);
                    const bool drop = bad && a.solve_mode == SBCE_SOLVE_CHOL_DROP;
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
                if (c2 > c && c2 < w) R[(size_t)(jb + c) * L + jb + c2] = cconj(Di[c2 * NB + c]);
            }
        }
        if (wave == 0 && !(skip & 4)) {
            // forward-solve the y block in parallel: y_blk <- Di y_blk  (w*NR <= 128 outputs)
            const int e0 = lane, e1 = lane + 64;
            cd t0 = czero(), t1 = czero();
            if (e0 < w * NR) {
                const int c = e0 / NR, r = e0 - c * NR;
                for (int c2 = 0; c2 <= c; ++c2) t0 = cfma(t0, Di[c * NB + c2], y[(jb + c2) * NR + r]);
            }
            if (e1 < w * NR) {
                const int c = e1 / NR, r = e1 - c * NR;
                for (int c2 = 0; c2 <= c; ++c2) t1 = cfma(t1, Di[c * NB + c2], y[(jb + c2) * NR + r]);
            }
            wave_sync();
            if (e0 < w * NR) y[jb * NR + e0] = t0;
            if (e1 < w * NR) y[jb * NR + e1] = t1;
        }
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

    // ================= blocked back substitution  L^H x = y =================
    const int nblk = (L + NB - 1) / NB;
    for (int kb = nblk - 1; kb >= ((skip & 16) ? nblk : 0); --kb) {
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

}  // namespace

bool chol_supported(const Problem& pb) { return pb.L >= 1 && pb.L <= 1024; }

hipError_t launch_chol_solve(const Problem& pb, const MstepArgs& a, hipStream_t s) {
    if (!chol_supported(pb)) return hipErrorInvalidValue;
    int nth = (pb.L + 63) / 64 * 64;
    if (nth > 512) nth = 512;
    const int rpt = (pb.L + nth - 1) / nth;
    const size_t base = (size_t)(NB * KC + 2 * NB * NB) * sizeof(cd) + (NB + 18) * sizeof(double);
    const size_t ybytes = (size_t)pb.L * pb.NR * sizeof(cd);
    if (ybytes <= 48 * 1024) return launch_y<true>(pb, a, nth, rpt, base + ybytes, s);
    return launch_y<false>(pb, a, nth, rpt, base, s);
}

}  // namespace sbce
