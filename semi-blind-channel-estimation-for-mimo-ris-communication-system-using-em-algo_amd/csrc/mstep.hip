// M-step kernels: reduced normal equations + batched Hermitian solve.
//
// Reference: "Proposed method/Proposed_method_NMSEvsTp.py":70-80 accumulates the
// K x K system  sum beta Z^H Z,  sum beta Z^H y  (K = (N+1) n_tx n_rx) and calls
// np.linalg.solve (LAPACK zgesv).  With Z = u^T (x) I_{n_rx} the commutation
// identity ("Proposed method/commutation_matrix.py":3-8) gives
// Z^H Z = conj(u u^H) (x) I, so the system is block-diagonal in the receive
// antenna: H_c R = B with the L x L Hermitian
//   R = sum_p u_p u_p^H + sum_t (psi_t psi_t^H) (x) S_t
// and B^H = sum_p u_p y_p^H + sum_t (psi_t (x) m_t) y_t^H  (L x n_rx).
// The pilot terms are rebuilt every iteration by the reference (:72-74); here
// they are summed in the same pass as the data terms (never stored).
#include <stdlib.h>

#include "sbce_internal.h"

namespace sbce {

namespace {

// ------------------------------------------------------------------ R build
// One thread per block pair (p >= q) of one trial; the NT x NT block of R at
// rows p*NT.., cols q*NT.. and its Hermitian mirror.  S_t is wave-uniform.
template <int NT>
__global__ __launch_bounds__(256) void rbuild_kernel(MstepArgs a, int B, int P, int Tp, int Td,
                                                     int L) {
    const int b = blockIdx.y;
    if ((a.done && a.done[b]) || (a.gate && !a.gate[b])) return;
    const int npairs = P * (P + 1) / 2;
    const int pi = blockIdx.x * blockDim.x + threadIdx.x;
    if (pi >= npairs) return;
    int p = (int)((sqrt(8.0 * pi + 1.0) - 1.0) * 0.5);
    while ((p + 1) * (p + 2) / 2 <= pi) ++p;
    while (p * (p + 1) / 2 > pi) --p;
    const int q = pi - p * (p + 1) / 2;
    constexpr int MS = NT + NT * NT;

    cd acc[NT][NT];
#pragma unroll
    for (int i = 0; i < NT; ++i)
#pragma unroll
        for (int j = 0; j < NT; ++j) acc[i][j] = czero();

    const cd* up = a.up + (size_t)b * Tp * L;
    for (int tp = 0; tp < Tp; ++tp) {
        cd ua[NT], ub[NT];
#pragma unroll
        for (int i = 0; i < NT; ++i) { ua[i] = up[tp * L + p * NT + i]; ub[i] = up[tp * L + q * NT + i]; }
#pragma unroll
        for (int i = 0; i < NT; ++i)
#pragma unroll
            for (int j = 0; j < NT; ++j) acc[i][j] = cfmac(acc[i][j], ua[i], ub[j]);
    }
    const cd* ps = a.psid + (size_t)b * Td * P;
    const cd* mom = a.mom + (size_t)b * Td * MS;
    for (int t = 0; t < Td; ++t) {
        const cd w = cmulc(ps[t * P + p], ps[t * P + q]);
        const cd* St = mom + t * MS + NT;
#pragma unroll
        for (int i = 0; i < NT; ++i)
#pragma unroll
            for (int j = 0; j < NT; ++j) acc[i][j] = cfma(acc[i][j], w, St[i * NT + j]);
    }
    cd* R = a.R + (size_t)b * L * L;
#pragma unroll
    for (int i = 0; i < NT; ++i)
#pragma unroll
        for (int j = 0; j < NT; ++j) {
            R[(size_t)(p * NT + i) * L + q * NT + j] = acc[i][j];
            if (p != q) R[(size_t)(q * NT + j) * L + p * NT + i] = cconj(acc[i][j]);
        }
}

// Wide variant for NT = 5..8 (PM E-step shapes): one thread per (block pair, row i)
// keeps NT accumulators instead of NT^2.
template <int NT>
__global__ __launch_bounds__(256) void rbuild_wide_kernel(MstepArgs a, int B, int P, int Tp,
                                                          int Td, int L) {
    const int b = blockIdx.y;
    if ((a.done && a.done[b]) || (a.gate && !a.gate[b])) return;
    const int npairs = P * (P + 1) / 2;
    const int gid = blockIdx.x * blockDim.x + threadIdx.x;
    const int pi = gid / NT, i = gid - pi * NT;
    if (pi >= npairs) return;
    int p = (int)((sqrt(8.0 * pi + 1.0) - 1.0) * 0.5);
    while ((p + 1) * (p + 2) / 2 <= pi) ++p;
    while (p * (p + 1) / 2 > pi) --p;
    const int q = pi - p * (p + 1) / 2;
    constexpr int MS = NT + NT * NT;

    cd acc[NT];
#pragma unroll
    for (int j = 0; j < NT; ++j) acc[j] = czero();
    const cd* up = a.up + (size_t)b * Tp * L;
    for (int tp = 0; tp < Tp; ++tp) {
        const cd ua = up[tp * L + p * NT + i];
#pragma unroll
        for (int j = 0; j < NT; ++j) acc[j] = cfmac(acc[j], ua, up[tp * L + q * NT + j]);
    }
    const cd* ps = a.psid + (size_t)b * Td * P;
    const cd* mom = a.mom + (size_t)b * Td * MS;
    for (int t = 0; t < Td; ++t) {
        const cd w = cmulc(ps[t * P + p], ps[t * P + q]);
        const cd* St = mom + t * MS + NT + i * NT;
#pragma unroll
        for (int j = 0; j < NT; ++j) acc[j] = cfma(acc[j], w, St[j]);
    }
    cd* R = a.R + (size_t)b * L * L;
#pragma unroll
    for (int j = 0; j < NT; ++j) {
        R[(size_t)(p * NT + i) * L + q * NT + j] = acc[j];
        if (p != q) R[(size_t)(q * NT + j) * L + p * NT + i] = cconj(acc[j]);
    }
}

// ------------------------------------------------------------------ B^H build
// One thread per row l = p*NT + a of one trial (L x NR right-hand sides).
template <int NR>
__global__ __launch_bounds__(256) void rhs_kernel(MstepArgs a, int B, int P, int NT, int Tp,
                                                  int Td, int L) {
    const int b = blockIdx.y;
    if (a.done && a.done[b]) return;
    const int l = blockIdx.x * blockDim.x + threadIdx.x;
    if (l >= L) return;
    const int p = l / NT, ai = l - p * NT;
    const int MS = NT + NT * NT;
    cd acc[NR];
#pragma unroll
    for (int r = 0; r < NR; ++r) acc[r] = czero();
    const cd* up = a.up + (size_t)b * Tp * L;
    const cd* yp = a.yp + (size_t)b * Tp * NR;
    for (int tp = 0; tp < Tp; ++tp) {
        const cd u = up[tp * L + l];
#pragma unroll
        for (int r = 0; r < NR; ++r) acc[r] = cfmac(acc[r], u, yp[tp * NR + r]);
    }
    const cd* ps = a.psid + (size_t)b * Td * P;
    const cd* mom = a.mom + (size_t)b * Td * MS;
    const cd* yd = a.yd + (size_t)b * Td * NR;
    for (int t = 0; t < Td; ++t) {
        const cd w = cmul(ps[t * P + p], mom[t * MS + ai]);
#pragma unroll
        for (int r = 0; r < NR; ++r) acc[r] = cfmac(acc[r], w, yd[t * NR + r]);
    }
    cd* rhs = a.rhs + ((size_t)b * L + l) * NR;
#pragma unroll
    for (int r = 0; r < NR; ++r) rhs[r] = acc[r];
}

// L <= 512: one block per trial, one thread per row l; the phases, moments and observations
// of TCR symbols at a time are staged in LDS (coalesced), so the symbol loop reads LDS only.
template <int NR>
__global__ __launch_bounds__(512) void rhs_lds_kernel(MstepArgs a, int P, int NT, int Tp, int Td,
                                                      int L, int TCR) {
    extern __shared__ __attribute__((aligned(16))) char smem[];
    cd* s_ps = reinterpret_cast<cd*>(smem);          // [TCR][P]
    cd* s_m = s_ps + TCR * P;                        // [TCR][NT]
    cd* s_y = s_m + TCR * NT;                        // [TCR][NR]
    const int b = blockIdx.x;
    if (a.done && a.done[b]) return;
    const int tid = threadIdx.x, nth = blockDim.x;
    const bool live = tid < L;
    const int l = live ? tid : L - 1;
    const int p = l / NT, ai = l - p * NT;
    const int MS = NT + NT * NT;
    cd acc[NR];
#pragma unroll
    for (int r = 0; r < NR; ++r) acc[r] = czero();
    const cd* up = a.up + (size_t)b * Tp * L;
    const cd* yp = a.yp + (size_t)b * Tp * NR;
    for (int tp = 0; tp < Tp; ++tp) {
        const cd u = up[tp * L + l];
#pragma unroll
        for (int r = 0; r < NR; ++r) acc[r] = cfmac(acc[r], u, yp[tp * NR + r]);
    }
    const cd* ps = a.psid + (size_t)b * Td * P;
    const cd* mom = a.mom + (size_t)b * Td * MS;
    const cd* yd = a.yd + (size_t)b * Td * NR;
    for (int t0 = 0; t0 < Td; t0 += TCR) {
        const int tc = (Td - t0) < TCR ? (Td - t0) : TCR;
        __syncthreads();
        for (int e = tid; e < tc * P; e += nth) s_ps[e] = ps[(size_t)t0 * P + e];
        for (int e = tid; e < tc * NT; e += nth) {
            const int tt = e / NT;
            s_m[e] = mom[(size_t)(t0 + tt) * MS + (e - tt * NT)];
        }
        for (int e = tid; e < tc * NR; e += nth) s_y[e] = yd[(size_t)t0 * NR + e];
        __syncthreads();
        for (int tt = 0; tt < tc; ++tt) {
            const cd w = cmul(s_ps[tt * P + p], s_m[tt * NT + ai]);
#pragma unroll
            for (int r = 0; r < NR; ++r) acc[r] = cfmac(acc[r], w, s_y[tt * NR + r]);
        }
    }
    if (live) {
        cd* rhs = a.rhs + ((size_t)b * L + l) * NR;
#pragma unroll
        for (int r = 0; r < NR; ++r) rhs[r] = acc[r];
    }
}

// The same with the symbol chunks double-buffered by LDS-DMA (global_load_lds, no staging
// registers): chunk c + 1's phases, moments and observations are in flight while chunk c is
// accumulated, one workgroup barrier per chunk (rhs_lds_kernel waits on each chunk's global
// loads with the whole block idle).  Lanes past a partial last chunk re-read its last element.
template <int NR>
__global__ __launch_bounds__(512) void rhs_dma_kernel(MstepArgs a, int P, int NT, int Tp, int Td,
                                                      int L, int TCR) {
    extern __shared__ __attribute__((aligned(16))) char smem[];
    const int CH = TCR * (P + NT + NR);              // cd per chunk buffer: [TCR][P] [TCR][NT] [TCR][NR]
    const int b = blockIdx.x;
    if (a.done && a.done[b]) return;
    const int tid = threadIdx.x, nth = blockDim.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6), nw = nth >> 6;
    const bool live = tid < L;
    const int l = live ? tid : L - 1;
    const int p = l / NT, ai = l - p * NT;
    const int MS = NT + NT * NT;
    const cd* ps = a.psid + (size_t)b * Td * P;
    const cd* mom = a.mom + (size_t)b * Td * MS;
    const cd* yd = a.yd + (size_t)b * Td * NR;
    auto stage = [&](int t0, cd* dst) {
        const int tc = (Td - t0) < TCR ? (Td - t0) : TCR;
        cd* d_m = dst + TCR * P;
        cd* d_y = d_m + TCR * NT;
        for (int e0 = wave * 64; e0 < TCR * P; e0 += nw * 64) {
            const int e = e0 + lane, ec = e < tc * P ? e : tc * P - 1;
            if (e < TCR * P)
                __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)(ps + (size_t)t0 * P + ec),
                                                 (__attribute__((address_space(3))) void*)(dst + e0), 16, 0, 0);
        }
        for (int e0 = wave * 64; e0 < TCR * NT; e0 += nw * 64) {
            const int e = e0 + lane, tt = e / NT, tcl = tt < tc ? tt : tc - 1;
            if (e < TCR * NT)
                __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)(mom + (size_t)(t0 + tcl) * MS + (e - tt * NT)),
                                                 (__attribute__((address_space(3))) void*)(d_m + e0), 16, 0, 0);
        }
        for (int e0 = wave * 64; e0 < TCR * NR; e0 += nw * 64) {
            const int e = e0 + lane, ec = e < tc * NR ? e : tc * NR - 1;
            if (e < TCR * NR)
                __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)(yd + (size_t)t0 * NR + ec),
                                                 (__attribute__((address_space(3))) void*)(d_y + e0), 16, 0, 0);
        }
    };
    cd* buf = reinterpret_cast<cd*>(smem);
    if (Td > 0) stage(0, buf);                       // first chunk in flight during the pilot sums
    cd acc[NR];
#pragma unroll
    for (int r = 0; r < NR; ++r) acc[r] = czero();
    if (a.prhs && Tp > 0) {                          // pilot part kept once per run
        const cd* pr = a.prhs + ((size_t)b * L + l) * NR;
#pragma unroll
        for (int r = 0; r < NR; ++r) acc[r] = pr[r];
    } else {
        const cd* up = a.up + (size_t)b * Tp * L;
        const cd* yp = a.yp + (size_t)b * Tp * NR;
        for (int tp = 0; tp < Tp; ++tp) {
            const cd u = up[tp * L + l];
#pragma unroll
            for (int r = 0; r < NR; ++r) acc[r] = cfmac(acc[r], u, yp[tp * NR + r]);
        }
    }
    int c = 0;
    for (int t0 = 0; t0 < Td; t0 += TCR, ++c) {
        const int tc = (Td - t0) < TCR ? (Td - t0) : TCR;
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");    // this wave's DMAs of chunk c
        __syncthreads();                                     // everyone's; chunk c - 1 consumed
        if (t0 + TCR < Td) stage(t0 + TCR, buf + ((c + 1) & 1) * CH);
        const cd* s_ps = buf + (c & 1) * CH;
        const cd* s_m = s_ps + TCR * P;
        const cd* s_y = s_m + TCR * NT;
        for (int tt = 0; tt < tc; ++tt) {
            const cd w = cmul(s_ps[tt * P + p], s_m[tt * NT + ai]);
#pragma unroll
            for (int r = 0; r < NR; ++r) acc[r] = cfmac(acc[r], w, s_y[tt * NR + r]);
        }
    }
    if (live) {
        cd* rhs = a.rhs + ((size_t)b * L + l) * NR;
#pragma unroll
        for (int r = 0; r < NR; ++r) rhs[r] = acc[r];
    }
}

// ------------------------------------------------------------------ small per-trial kernels
__device__ double block_sum(double v, double* sh) {
    for (int off = 32; off >= 1; off >>= 1) v += __shfl_xor(v, off);
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    __syncthreads();
    if (lane == 0) sh[wave] = v;
    __syncthreads();
    double s = 0.0;
    for (int w = 0; w < (int)(blockDim.x >> 6); ++w) s += sh[w];
    return s;
}

__global__ __launch_bounds__(256) void nmse_kernel(const cd* theta, const cd* h, double* out, int K) {
    __shared__ double sh[4];
    const int b = blockIdx.x;
    double num = 0.0, den = 0.0;
    for (int e = threadIdx.x; e < K; e += blockDim.x) {
        const cd hv = h[(size_t)b * K + e];
        num += cabs2(csub(theta[(size_t)b * K + e], hv));
        den += cabs2(hv);
    }
    num = block_sum(num, sh);
    den = block_sum(den, sh);
    if (threadIdx.x == 0) out[b] = num / den;
}

// Gaussian prior, n_rx = 1 ("Proposed method/MIMO_Gaussian_proposed.py":73-76): the
// reference's covar adds the scalar ||mu_t||^2 = ||psi_t||^2 ||m_t||^2 to every entry of A,
// i.e. R += c 1 1^T with c = sum_t ||psi_t||^2 ||m_t||^2 (one block per trial).
__global__ __launch_bounds__(256) void gauss_rank1_kernel(MstepArgs a, int Td, int P, int NT,
                                                          int L) {
    __shared__ double sh[4];
    const int b = blockIdx.x;
    if (a.done && a.done[b]) return;
    const int MS = NT + NT * NT;
    double c = 0.0;
    for (int t = threadIdx.x; t < Td; t += blockDim.x) {
        const cd* ps = a.psid + ((size_t)b * Td + t) * P;
        const cd* m = a.mom + ((size_t)b * Td + t) * MS;
        double np2 = 0.0, nm2 = 0.0;
        for (int p = 0; p < P; ++p) np2 += cabs2(ps[p]);
        for (int q = 0; q < NT; ++q) nm2 += cabs2(m[q]);
        c = fma(np2, nm2, c);
    }
    c = block_sum(c, sh);
    cd* R = a.R + (size_t)b * L * L;
    for (int e = threadIdx.x; e < L * L; e += blockDim.x) R[e].x += c;
}

// H_l of "Proposed method/MIMO_Gaussian_proposed.py":77-85 from the reduced estimate
// (include/sbce.h, sbce_gauss_expand): block (r, b) writes row r of trial b.
__global__ __launch_bounds__(256) void gauss_expand_kernel(const cd* theta, cd* out, int Lr,
                                                           int NR) {
    __shared__ double sh[4];
    const int r = blockIdx.x, b = blockIdx.y;
    const cd* th = theta + (size_t)b * Lr * NR;
    const long Q = (long)Lr * NR * NR;
    cd* o = out + ((size_t)b * NR + r) * Q;
    if (NR == 1) {
        for (int c = threadIdx.x; c < Lr; c += blockDim.x) o[c] = th[c];
        return;
    }
    double sx = 0.0, sy = 0.0;
    for (int c = threadIdx.x; c < Lr; c += blockDim.x) { sx += th[c * NR + r].x; sy += th[c * NR + r].y; }
    sx = block_sum(sx, sh);
    sy = block_sum(sy, sh);
    const double inv_n = 1.0 / NR;
    const double g = -1.0 / ((double)Lr * (double)(NR * NR - NR));
    const cd off = cmk(sx * g, sy * g);
    for (long e = threadIdx.x; e < Q; e += blockDim.x) {
        const int c = (int)(e / (NR * NR)), i = (int)(e - (long)c * NR * NR);
        const bool diag = (i / NR) == (i % NR);
        o[e] = diag ? cscale(th[c * NR + r], inv_n) : off;
    }
}

// Superimposed pilots ("Parallel/ParallelProtocol_Tp.py":63-86): hypotheses x_j + x_p,t.
// The E-step runs on y'_t = y_t - H_t x_p,t (thread per (symbol, receive antenna)) and
// the moments of x_j + x_p,t follow by the shift m' = m + x_p,
// S' = S + m x_p^H + x_p m^H + x_p x_p^H (thread per symbol).
__global__ __launch_bounds__(256) void sup_shift_y_kernel(const cd* yd, const cd* psid,
                                                          const cd* theta, const cd* xsup,
                                                          cd* yout, const int32_t* done, long n,
                                                          int Td, int P, int NT, int NR) {
    const long e = (long)blockIdx.x * blockDim.x + threadIdx.x;
    if (e >= n) return;
    const long sym = e / NR;
    const int r = (int)(e - sym * NR);
    const int b = (int)(sym / Td);
    if (done && done[b]) return;
    const cd* th = theta + (size_t)b * P * NT * NR;
    const cd* ps = psid + (size_t)sym * P;
    const cd* xp = xsup + (size_t)sym * NT;
    cd acc = yd[e];
    for (int p = 0; p < P; ++p) {
        cd hx = czero();
        for (int a = 0; a < NT; ++a) hx = cfma(hx, th[(p * NT + a) * NR + r], xp[a]);
        acc = csub(acc, cmul(ps[p], hx));
    }
    yout[e] = acc;
}

__global__ __launch_bounds__(256) void sup_shift_mom_kernel(cd* mom, const cd* xsup,
                                                            const int32_t* done, long nsym,
                                                            int Td, int NT) {
    const long sym = (long)blockIdx.x * blockDim.x + threadIdx.x;
    if (sym >= nsym) return;
    if (done && done[sym / Td]) return;
    cd* mo = mom + (size_t)sym * (NT + NT * NT);
    const cd* xp = xsup + (size_t)sym * NT;
    for (int i = 0; i < NT; ++i)
        for (int j = 0; j < NT; ++j) {
            cd v = mo[NT + i * NT + j];
            v = cadd(v, cmulc(mo[i], xp[j]));
            v = cadd(v, cmulc(xp[i], mo[j]));
            v = cadd(v, cmulc(xp[i], xp[j]));
            mo[NT + i * NT + j] = v;
        }
    for (int i = 0; i < NT; ++i) mo[i] = cadd(mo[i], xp[i]);
}

// Last-iteration hard decisions (PMd/SER/log_max_SER.py:77-78): for the hard E-step modes
// m_t IS the decided hypothesis (weight 1), so x_dest[b][t] = m_t of the final E-step.
__global__ __launch_bounds__(256) void decisions_kernel(const cd* mom, cd* xdest, long n, int NT) {
    const long e = (long)blockIdx.x * blockDim.x + threadIdx.x;
    if (e >= n) return;
    const long t = e / NT;
    xdest[e] = mom[t * (NT + NT * NT) + (e - t * NT)];
}

// Per-trial SER of the decisions (PMd/SER/log_max_SER.py:162):
//   out[b][0] = count_nonzero(array(X_d) - array(X_dest)) / (T_d n_tx) with the script's
//               shapes (T_d, n_tx, 1) - (T_d, 1, n_tx): every (a, a') pair of a symbol is
//               compared (the reference's broadcast), so it is not 0 for exact decisions;
//   out[b][1] = the element-wise symbol error rate.
__global__ __launch_bounds__(256) void ser_kernel(const cd* xdest, const cd* xtrue, double* out,
                                                  int Td, int NT) {
    __shared__ double sh[4];
    const int b = blockIdx.x;
    double pairs = 0.0, elem = 0.0;
    const cd* xd = xdest + (size_t)b * Td * NT;
    const cd* xt = xtrue + (size_t)b * Td * NT;
    for (int e = threadIdx.x; e < Td * NT * NT; e += blockDim.x) {
        const int t = e / (NT * NT), r = e - t * NT * NT, a = r / NT, a2 = r - a * NT;
        const cd u = xt[t * NT + a], v = xd[t * NT + a2];
        const bool ne = u.x != v.x || u.y != v.y;
        pairs += ne ? 1.0 : 0.0;
        if (a == a2) elem += ne ? 1.0 : 0.0;
    }
    pairs = block_sum(pairs, sh);
    elem = block_sum(elem, sh);
    if (threadIdx.x == 0) {
        out[2 * b] = pairs / ((double)Td * NT);
        out[2 * b + 1] = elem / ((double)Td * NT);
    }
}

// LLF of "Proposed method/IterationsvsLLF.py":49-50,76:
//   -T_d n_tx ln M - (T_d+T_p) ln(pi varn^2) - (||Y_p - Z_p th|| + ||Y_d - Z_d th||)/varn^2
// with Z_d built from the TRUE symbols (genie) and UNsquared norms.
__global__ __launch_bounds__(256) void llf_kernel(const cd* theta, const cd* yp, const cd* up,
                                                  const cd* yd, const cd* psid, const cd* xd,
                                                  double* llf, const int32_t* done, int P, int NT,
                                                  int NR, int Tp, int Td, int M, double varn,
                                                  const double* varn_t, int iters, int it) {
    __shared__ double sh[4];
    const int b = blockIdx.x;
    if (done && done[b]) return;
    if (varn_t) varn = varn_t[b];                    // per-trial noise variance (ABI 6)
    const int L = P * NT;
    const cd* th = theta + (size_t)b * L * NR;
    double sp = 0.0, sd = 0.0;
    for (int e = threadIdx.x; e < Tp * NR; e += blockDim.x) {
        const int tp = e / NR, r = e % NR;
        cd acc = yp[((size_t)b * Tp + tp) * NR + r];
        const cd* u = up + ((size_t)b * Tp + tp) * L;
        for (int l = 0; l < L; ++l) acc = csub(acc, cmul(th[l * NR + r], u[l]));
        sp += cabs2(acc);
    }
    for (int e = threadIdx.x; e < Td * NR; e += blockDim.x) {
        const int t = e / NR, r = e % NR;
        cd acc = yd[((size_t)b * Td + t) * NR + r];
        const cd* ps = psid + ((size_t)b * Td + t) * P;
        const cd* x = xd + ((size_t)b * Td + t) * NT;
        for (int p = 0; p < P; ++p) {
            cd hx = czero();
            for (int ai = 0; ai < NT; ++ai) hx = cfma(hx, th[(p * NT + ai) * NR + r], x[ai]);
            acc = csub(acc, cmul(ps[p], hx));
        }
        sd += cabs2(acc);
    }
    sp = block_sum(sp, sh);
    sd = block_sum(sd, sh);
    if (threadIdx.x == 0) {
        const double v2 = varn * varn;
        llf[(size_t)b * iters + it] = -(double)Td * NT * log((double)M) -
                                      (double)(Td + Tp) * log(M_PI * v2) - sqrt(sp) / v2 -
                                      sqrt(sd) / v2;
    }
}

// Oracle early stop of "Proposed method/PM.py":110-112:
//   if |‖theta‖ - ‖h‖| < 1 and l != 0: break
__global__ __launch_bounds__(256) void early_stop_kernel(const cd* theta, const cd* h, int32_t* done,
                                                         int32_t* iters_done, int K, int it) {
    __shared__ double sh[4];
    const int b = blockIdx.x;
    if (done[b]) return;
    double nt = 0.0, nh = 0.0;
    for (int e = threadIdx.x; e < K; e += blockDim.x) {
        nt += cabs2(theta[(size_t)b * K + e]);
        nh += cabs2(h[(size_t)b * K + e]);
    }
    nt = block_sum(nt, sh);
    nh = block_sum(nh, sh);
    if (threadIdx.x == 0) {
        if (iters_done) iters_done[b] = it + 1;
        if (it != 0 && fabs(sqrt(nt) - sqrt(nh)) < 1.0) done[b] = 1;
    }
}

}  // namespace

hipError_t launch_mstep_build(const Problem& pb, const MstepArgs& a0, hipStream_t s,
                              bool pilots_factored) {
    const int npairs = pb.P * (pb.P + 1) / 2;
    MstepArgs a = a0;
    // NT in {4, 8}: MFMA build from Kronecker-factored pilots (mstep_large.hip; the factors
    // depend on u_p only, so an EM run computes them once), then the VALU build below
    // re-runs only the trials whose u_p is not a Kronecker product
    const bool herm = rbuild_herm_supported(pb);
    if (herm) {
        hipError_t e0 = pilots_factored ? hipSuccess : launch_pilot_factor(pb, a, s);
        if (e0 == hipSuccess) e0 = launch_rbuild_herm(pb, a, s);
        if (e0 != hipSuccess) return e0;
        a.gate = a.pflag;
    }
    dim3 g1((npairs + 255) / 256, pb.B);
    switch (pb.NT) {
        case 1: hipLaunchKernelGGL(rbuild_kernel<1>, g1, dim3(256), 0, s, a, pb.B, pb.P, pb.Tp, pb.Td, pb.L); break;
        case 2: hipLaunchKernelGGL(rbuild_kernel<2>, g1, dim3(256), 0, s, a, pb.B, pb.P, pb.Tp, pb.Td, pb.L); break;
        case 3: hipLaunchKernelGGL(rbuild_kernel<3>, g1, dim3(256), 0, s, a, pb.B, pb.P, pb.Tp, pb.Td, pb.L); break;
        case 4: hipLaunchKernelGGL(rbuild_kernel<4>, g1, dim3(256), 0, s, a, pb.B, pb.P, pb.Tp, pb.Td, pb.L); break;
#define SBCE_RW(n) case n: hipLaunchKernelGGL(rbuild_wide_kernel<n>, dim3((npairs * n + 255) / 256, pb.B), dim3(256), 0, s, a, pb.B, pb.P, pb.Tp, pb.Td, pb.L); break;
        SBCE_RW(5) SBCE_RW(6) SBCE_RW(7) SBCE_RW(8)
#undef SBCE_RW
        default: return hipErrorInvalidValue;
    }
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
    if (pb.L <= 512) {
        const int nth = (pb.L + 63) / 64 * 64;
        const int tcr = pb.P <= 128 ? 16 : 4;             // <= 33 KB of phases per chunk
        const size_t lds = (size_t)tcr * (pb.P + pb.NT + pb.NR) * sizeof(cd);
        // LDS-DMA double-buffered chunks when two buffers fit 64 KB (cfg1: 37 KB), else the
        // single-buffer kernel
        if (2 * lds <= 64 * 1024) {
            switch (pb.NR) {
#define SBCE_RHSD(n) case n: hipLaunchKernelGGL(rhs_dma_kernel<n>, dim3(pb.B), dim3(nth), 2 * lds, s, a, pb.P, pb.NT, pb.Tp, pb.Td, pb.L, tcr); break;
                SBCE_RHSD(1) SBCE_RHSD(2) SBCE_RHSD(3) SBCE_RHSD(4) SBCE_RHSD(5) SBCE_RHSD(6) SBCE_RHSD(7) SBCE_RHSD(8)
#undef SBCE_RHSD
                default: return hipErrorInvalidValue;
            }
            return hipGetLastError();
        }
        switch (pb.NR) {
#define SBCE_RHSL(n) case n: hipLaunchKernelGGL(rhs_lds_kernel<n>, dim3(pb.B), dim3(nth), lds, s, a, pb.P, pb.NT, pb.Tp, pb.Td, pb.L, tcr); break;
            SBCE_RHSL(1) SBCE_RHSL(2) SBCE_RHSL(3) SBCE_RHSL(4) SBCE_RHSL(5) SBCE_RHSL(6) SBCE_RHSL(7) SBCE_RHSL(8)
#undef SBCE_RHSL
            default: return hipErrorInvalidValue;
        }
        return hipGetLastError();
    }
    dim3 g2((pb.L + 255) / 256, pb.B);
    switch (pb.NR) {
#define SBCE_RHS(n) case n: hipLaunchKernelGGL(rhs_kernel<n>, g2, dim3(256), 0, s, a, pb.B, pb.P, pb.NT, pb.Tp, pb.Td, pb.L); break;
        SBCE_RHS(1) SBCE_RHS(2) SBCE_RHS(3) SBCE_RHS(4) SBCE_RHS(5) SBCE_RHS(6) SBCE_RHS(7) SBCE_RHS(8)
#undef SBCE_RHS
        default: return hipErrorInvalidValue;
    }
    return hipGetLastError();
}

hipError_t launch_gauss_rank1(const Problem& pb, const MstepArgs& a, hipStream_t s) {
    hipLaunchKernelGGL(gauss_rank1_kernel, dim3(pb.B), dim3(256), 0, s, a, pb.Td, pb.P, pb.NT, pb.L);
    return hipGetLastError();
}

hipError_t launch_gauss_expand(const Problem& pb, const cd* theta, cd* out, hipStream_t s) {
    hipLaunchKernelGGL(gauss_expand_kernel, dim3(pb.NR, pb.B), dim3(256), 0, s, theta, out, pb.L,
                       pb.NR);
    return hipGetLastError();
}

hipError_t launch_nmse(const Problem& pb, const cd* theta, const cd* h, double* out, hipStream_t s) {
    hipLaunchKernelGGL(nmse_kernel, dim3(pb.B), dim3(256), 0, s, theta, h, out, pb.K);
    return hipGetLastError();
}

hipError_t launch_sup_shift_y(const Problem& pb, const cd* yd, const cd* psid, const cd* theta,
                              const cd* xsup, cd* yout, const int32_t* done, hipStream_t s) {
    const long n = (long)pb.B * pb.Td * pb.NR;
    if (n == 0) return hipSuccess;
    hipLaunchKernelGGL(sup_shift_y_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, yd,
                       psid, theta, xsup, yout, done, n, pb.Td, pb.P, pb.NT, pb.NR);
    return hipGetLastError();
}

hipError_t launch_sup_shift_mom(const Problem& pb, cd* mom, const cd* xsup, const int32_t* done,
                                hipStream_t s) {
    const long n = (long)pb.B * pb.Td;
    if (n == 0) return hipSuccess;
    hipLaunchKernelGGL(sup_shift_mom_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s,
                       mom, xsup, done, n, pb.Td, pb.NT);
    return hipGetLastError();
}

hipError_t launch_decisions(const Problem& pb, const cd* mom, cd* xdest, hipStream_t s) {
    const long n = (long)pb.B * pb.Td * pb.NT;
    if (n == 0) return hipSuccess;
    hipLaunchKernelGGL(decisions_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, mom,
                       xdest, n, pb.NT);
    return hipGetLastError();
}

hipError_t launch_ser(const Problem& pb, const cd* xdest, const cd* xtrue, double* out,
                      hipStream_t s) {
    hipLaunchKernelGGL(ser_kernel, dim3(pb.B), dim3(256), 0, s, xdest, xtrue, out, pb.Td, pb.NT);
    return hipGetLastError();
}

hipError_t launch_llf(const Problem& pb, const cd* theta, const cd* yp, const cd* up, const cd* yd,
                      const cd* psid, const cd* xd, double* llf, int iters, int it,
                      const int32_t* done, const double* varn_t, hipStream_t s) {
    hipLaunchKernelGGL(llf_kernel, dim3(pb.B), dim3(256), 0, s, theta, yp, up, yd, psid, xd, llf, done,
                       pb.P, pb.NT, pb.NR, pb.Tp, pb.Td, pb.M, pb.varn, varn_t, iters, it);
    return hipGetLastError();
}

namespace {
__global__ __launch_bounds__(256) void em_init_kernel(int B, int32_t* done, int32_t* status, int sv,
                                                      int32_t* cnt) {
    const int i = blockIdx.x * 256 + threadIdx.x;
    if (i < B) {
        done[i] = 0;
        if (status) status[i] = sv;
    }
    if (cnt && i < 5) cnt[i] = 0;
}
}  // namespace

hipError_t launch_em_init(int B, int32_t* done, int32_t* status, int sv, int32_t* cnt, hipStream_t s) {
    hipLaunchKernelGGL(em_init_kernel, dim3((B + 255) / 256 > 0 ? (B + 255) / 256 : 1), dim3(256), 0,
                       s, B, done, status, sv, cnt);
    return hipGetLastError();
}

hipError_t launch_early_stop(const Problem& pb, const cd* theta, const cd* h, int32_t* done,
                             int32_t* iters_done, int it, hipStream_t s) {
    hipLaunchKernelGGL(early_stop_kernel, dim3(pb.B), dim3(256), 0, s, theta, h, done, iters_done,
                       pb.K, it);
    return hipGetLastError();
}

}  // namespace sbce
