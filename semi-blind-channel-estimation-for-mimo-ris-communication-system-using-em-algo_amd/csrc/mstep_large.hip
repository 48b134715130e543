// Large-L M-step (L > 512: BASELINE cfg 2, L = 2056, and cfg 4, L = 4100).
//
// The same reduced normal equations as mstep.hip / chol.hip (R X = B^H, theta = conj(X),
// "Proposed method/Proposed_method_NMSEvsTp.py":70-80 + commutation_matrix.py:3-8), at a
// size where one trial's R (67.6 MB at cfg 2, 269 MB at cfg 4) no longer fits a single
// workgroup's working set, so both the build and the factorisation are tiled in 64 x 64
// blocks and spread over the whole chip:
//
//   pilot_factor_kernel  u_p[t] = psi_p[t] (x) x_p[t] (PMd/PM.py:119-130) is factored back
//                        into (psi', x'), so the pilot term of R has the data term's form
//                        (psi psi^H) (x) (x x^H) and is built by the same MFMA kernel;
//   rbuild_tile_kernel   R[(p,a),(q,b)] = sum_t psi[t][p] conj(psi[t][q]) S_t[a][b] as a
//                        GEMM over t with M = (p,q) pairs, N = (a,b): the A operand is
//                        generated from psi in LDS, the B operand is S_t; 64 x 64 tiles of
//                        the lower block triangle only (the factorisation never reads the
//                        strict upper triangle);
//   blocked right-looking Cholesky, NB = 64, per column block k:
//     chol_mfma_kernel<SOLVE=false>  factors the 64 x 64 diagonal tile in place (chol.hip);
//     tile_inverse_kernel            W = L_kk^{-1} (64 x 64, workspace);
//     tile_gemm_kernel<TRSM>         L_ik = A_ik W^H             (i > k);
//     tile_gemm_kernel<HERK>         A_ij -= L_ik L_jk^H          (i >= j > k);
//   trisolve_kernel      forward L y = B^H and back L^H x = y, blocked by 16 with the
//                        diagonal inverses kept in R's strict upper 16 x 16 blocks.
#include "sbce_internal.h"

namespace sbce {

namespace {

typedef double d4v __attribute__((ext_vector_type(4)));
constexpr int TB = 64;      // tile of the blocked factorisation and of the R build
constexpr int KS = 16;      // k-chunk staged in LDS by the tile GEMM

__device__ __forceinline__ d4v mfma4(double a, double b, d4v c) {
    return __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c, 0, 0, 0);
}

// ---------------------------------------------------------------- pilot factorisation
// One wave per (pilot symbol, trial).  l* = argmax |u_l|; x'[a] = u[p* NT + a],
// psi'[p] = u[p NT + a*] / u[l*]  =>  psi' (x) x' = u for an exact Kronecker product
// (the common scale cancels in (psi psi^H) (x) (x x^H)).  A residual above 1e-10 |u[l*]|
// sets status bit SBCE_STATUS_PILOT (the large-L build assumes Kronecker pilots).
__global__ __launch_bounds__(64) void pilot_factor_kernel(MstepArgs a, int P, int NT, int Tp,
                                                          int L) {
    const int tp = blockIdx.x, b = blockIdx.y, lane = threadIdx.x;
    const cd* u = a.up + ((size_t)b * Tp + tp) * L;
    double best = -1.0;
    int bi = 0;
    for (int l = lane; l < L; l += 64) {
        const double m = cabs2(u[l]);
        if (m > best) { best = m; bi = l; }
    }
    for (int off = 32; off >= 1; off >>= 1) {
        const double ob = __shfl_xor(best, off);
        const int oi = __shfl_xor(bi, off);
        if (ob > best || (ob == best && oi < bi)) { best = ob; bi = oi; }
    }
    const int ps = bi / NT, as = bi - ps * NT;
    const cd piv = u[bi];
    const double den = cabs2(piv);
    const cd ipiv = den > 0.0 ? cmk(piv.x / den, -piv.y / den) : czero();
    cd* psi = a.ppsi + ((size_t)b * Tp + tp) * P;
    cd* S = a.pS + ((size_t)b * Tp + tp) * NT * NT;
    for (int p = lane; p < P; p += 64) psi[p] = cmul(u[p * NT + as], ipiv);
    for (int e = lane; e < NT * NT; e += 64) {
        const int i = e / NT, j = e - i * NT;
        S[e] = cmulc(u[ps * NT + i], u[ps * NT + j]);
    }
    double res = 0.0;
    for (int l = lane; l < L; l += 64) {
        const int p = l / NT, i = l - p * NT;
        const cd v = cmul(cmul(u[p * NT + as], ipiv), u[ps * NT + i]);
        res = fmax(res, cabs2(csub(u[l], v)));
    }
    for (int off = 32; off >= 1; off >>= 1) res = fmax(res, __shfl_xor(res, off));
    if (lane == 0 && a.status && res > 1e-20 * den) atomicOr(&a.status[b], SBCE_STATUS_PILOT);
}

// ---------------------------------------------------------------- R build (MFMA)
// Block = 64 x 64 tile (ti >= tj) of R for one trial: pairs p in [ti PB, ti PB + PB),
// q in [tj PB, ..), PB = 64 / NT.  4 waves; wave w owns TP pair tiles x TA ab tiles of the
// 16 x 16 MFMA grid (NT = 8: 1 x 4, NT = 4: 4 x 1).  Per 4 symbols: TP operands
// psi_p conj(psi_q) (A), TA operands S_t[ab] (B), 16 chained MFMAs.
template <int NT>
__global__ __launch_bounds__(256) void rbuild_tile_kernel(MstepArgs a, int P, int Tp, int Td,
                                                          int L, int ntr) {
    constexpr int PB = TB / NT;                 // p (and q) values per tile side
    constexpr int NAB = NT * NT;
    constexpr int TA = NAB / 16;                // ab tiles per wave
    constexpr int TP = 4 / TA;                  // pair tiles per wave
    constexpr int TC = 16;                      // symbols per LDS chunk
    constexpr int MS = NT + NT * NT;
    static_assert(NAB % 16 == 0 && TP * TA == 4, "rbuild_tile: NT in {4, 8}");
    __shared__ cd s_pp[TC][PB], s_pq[TC][PB];
    __shared__ cd s_S[TC][NAB];
    const int b = blockIdx.y;
    if (a.done && a.done[b]) return;
    // lower-triangular tile index -> (ti, tj)
    const int tix = blockIdx.x;
    int ti = (int)((sqrt(8.0 * tix + 1.0) - 1.0) * 0.5);
    while ((ti + 1) * (ti + 2) / 2 <= tix) ++ti;
    while (ti * (ti + 1) / 2 > tix) --ti;
    const int tj = tix - ti * (ti + 1) / 2;
    const int p0 = ti * PB, q0 = tj * PB;
    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int li = lane & 15, lk = lane >> 4;

    d4v cre[TP][TA], cim[TP][TA];
#pragma unroll
    for (int u = 0; u < TP; ++u)
#pragma unroll
        for (int v = 0; v < TA; ++v) {
            cre[u][v] = d4v{0.0, 0.0, 0.0, 0.0};
            cim[u][v] = d4v{0.0, 0.0, 0.0, 0.0};
        }
    // pair of A-operand row i in pair tile u of this wave: pair index (wave*TP + u)*16 + i
    int pp[TP], pq[TP];
#pragma unroll
    for (int u = 0; u < TP; ++u) {
        const int pi = (wave * TP + u) * 16 + li;
        pp[u] = pi / PB;
        pq[u] = pi - pp[u] * PB;
    }
    const cd* psd = a.psid + (size_t)b * Td * P;
    const cd* mom = a.mom + (size_t)b * Td * MS;
    const cd* psp = a.ppsi + (size_t)b * Tp * P;
    const cd* pS = a.pS + (size_t)b * Tp * NAB;
    const int T = Td + Tp;
    for (int t0 = 0; t0 < T; t0 += TC) {
        __syncthreads();
        for (int e = tid; e < TC * PB; e += 256) {
            const int tt = e / PB, k = e - tt * PB, t = t0 + tt;
            cd vp = czero(), vq = czero();
            if (t < Td) {
                if (p0 + k < P) vp = psd[(size_t)t * P + p0 + k];
                if (q0 + k < P) vq = psd[(size_t)t * P + q0 + k];
            } else if (t < T) {
                if (p0 + k < P) vp = psp[(size_t)(t - Td) * P + p0 + k];
                if (q0 + k < P) vq = psp[(size_t)(t - Td) * P + q0 + k];
            }
            s_pp[tt][k] = vp;
            s_pq[tt][k] = vq;
        }
        for (int e = tid; e < TC * NAB; e += 256) {
            const int tt = e / NAB, k = e - tt * NAB, t = t0 + tt;
            cd v = czero();
            if (t < Td) v = mom[(size_t)t * MS + NT + k];
            else if (t < T) v = pS[(size_t)(t - Td) * NAB + k];
            s_S[tt][k] = v;
        }
        __syncthreads();
#pragma unroll
        for (int s = 0; s < TC / 4; ++s) {
            const int tt = 4 * s + lk;
            cd av[TP], bv[TA];
#pragma unroll
            for (int u = 0; u < TP; ++u) av[u] = cmulc(s_pp[tt][pp[u]], s_pq[tt][pq[u]]);
#pragma unroll
            for (int v = 0; v < TA; ++v) bv[v] = s_S[tt][16 * v + li];
#pragma unroll
            for (int u = 0; u < TP; ++u)
#pragma unroll
                for (int v = 0; v < TA; ++v) {
                    // C += A B (complex): re += ar br - ai bi ; im += ar bi + ai br
                    cre[u][v] = mfma4(av[u].x, bv[v].x, cre[u][v]);
                    cre[u][v] = mfma4(-av[u].y, bv[v].y, cre[u][v]);
                    cim[u][v] = mfma4(av[u].x, bv[v].y, cim[u][v]);
                    cim[u][v] = mfma4(av[u].y, bv[v].x, cim[u][v]);
                }
        }
    }
    // write: C row = pair (lk + 4q) of the pair tile, column = ab (li) of the ab tile
    cd* R = a.R + (size_t)b * L * L;
#pragma unroll
    for (int u = 0; u < TP; ++u)
#pragma unroll
        for (int v = 0; v < TA; ++v)
#pragma unroll
            for (int q4 = 0; q4 < 4; ++q4) {
                const int pi = (wave * TP + u) * 16 + lk + 4 * q4;
                const int p = p0 + pi / PB, q = q0 + pi % PB;
                const int ab = 16 * v + li, ai = ab / NT, bi = ab - ai * NT;
                if (p < P && q < P)
                    R[(size_t)(p * NT + ai) * L + q * NT + bi] = cmk(cre[u][v][q4], cim[u][v][q4]);
            }
    (void)ntr;
}

// ---------------------------------------------------------------- tolerance
// tol[b] = 1e-14 max_i Re R[i][i] of the freshly built R (chol.hip's pivot threshold).
__global__ __launch_bounds__(256) void diag_tol_kernel(MstepArgs a, int L) {
    const int b = blockIdx.x;
    const cd* R = a.R + (size_t)b * L * L;
    __shared__ double red[4];
    double m = 0.0;
    for (int i = threadIdx.x; i < L; i += 256) m = fmax(m, R[(size_t)i * L + i].x);
    for (int off = 32; off >= 1; off >>= 1) m = fmax(m, __shfl_xor(m, off));
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = m;
    __syncthreads();
    if (threadIdx.x == 0) a.tol[b] = 1e-14 * fmax(fmax(red[0], red[1]), fmax(red[2], red[3]));
}

// ---------------------------------------------------------------- W = L_kk^{-1}
// One wave per trial: lane j forward-substitutes column j of the inverse of the factored
// w x w diagonal tile (uniform loads of L, column in LDS).  Dropped pivots (0) give 0.
__global__ __launch_bounds__(64) void tile_inverse_kernel(MstepArgs a, int L, int k0, int w) {
    const int b = blockIdx.x;
    if (a.done && a.done[b]) return;
    extern __shared__ __attribute__((aligned(16))) char smem[];
    cd(*col)[TB] = reinterpret_cast<cd(*)[TB]>(smem);       // [TB][TB], 64 KB
    const cd* Lk = a.R + (size_t)b * L * L + (size_t)k0 * L + k0;
    const int j = threadIdx.x;
    for (int r = 0; r < w; ++r) {
        const cd* lr = Lk + (size_t)r * L;
        cd acc = cmk(r == j ? 1.0 : 0.0, 0.0);
        for (int m = j; m < r; ++m) acc = csub(acc, cmul(lr[m], col[m][j]));
        const double d = lr[r].x;
        col[r][j] = (j <= r && d > 0.0) ? cscale(acc, 1.0 / d) : czero();
    }
    cd* W = a.winv + (size_t)b * TB * TB;
    for (int r = 0; r < TB; ++r) W[r * TB + j] = (r < w && j < w) ? col[r][j] : czero();
}

// ---------------------------------------------------------------- tile GEMM
// C[r][c] = init + sgn sum_k A[r][k] conj(B[c][k]) on a 64 x 64 tile, K = 64.
//   TRSM (HERK = false): tile (i, k), C = A_ik W^H written in place (init 0);
//   HERK (HERK = true):  tile (i, j), C = A_ij - L_ik L_jk^H.
// 4 waves, wave w owns the 32 x 32 quadrant (w >> 1, w & 1) = 2 x 2 MFMA tiles.
template <bool HERK>
__global__ __launch_bounds__(256) void tile_gemm_kernel(MstepArgs a, int L, int kb) {
    __shared__ cd As[TB][KS + 1], Bs[TB][KS + 1];
    const int b = blockIdx.y;
    if (a.done && a.done[b]) return;
    int ti, tj;
    if (HERK) {
        const int tix = blockIdx.x;
        int x = (int)((sqrt(8.0 * tix + 1.0) - 1.0) * 0.5);
        while ((x + 1) * (x + 2) / 2 <= tix) ++x;
        while (x * (x + 1) / 2 > tix) --x;
        ti = kb + 1 + x;
        tj = kb + 1 + (tix - x * (x + 1) / 2);
    } else {
        ti = kb + 1 + blockIdx.x;
        tj = kb;
    }
    cd* R = a.R + (size_t)b * L * L;
    const int r0 = ti * TB, c0 = tj * TB, k0 = kb * TB;
    const cd* Arow = R + (size_t)r0 * L + k0;                          // A[r][k]
    const cd* Brow = HERK ? R + (size_t)c0 * L + k0 : a.winv + (size_t)b * TB * TB;
    const int ldb = HERK ? L : TB;
    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int li = lane & 15, lk = lane >> 4;
    const int wr = (wave >> 1) * 32, wc = (wave & 1) * 32;
    const int kmax = (L - k0) < TB ? (L - k0) : TB;

    d4v cre[2][2], cim[2][2];
#pragma unroll
    for (int u = 0; u < 2; ++u)
#pragma unroll
        for (int v = 0; v < 2; ++v) {
            cre[u][v] = d4v{0.0, 0.0, 0.0, 0.0};
            cim[u][v] = d4v{0.0, 0.0, 0.0, 0.0};
            if (HERK) {
#pragma unroll
                for (int q = 0; q < 4; ++q) {
                    const int r = r0 + wr + 16 * u + lk + 4 * q, c = c0 + wc + 16 * v + li;
                    if (r < L && c < L) {
                        const cd x = R[(size_t)r * L + c];
                        cre[u][v][q] = x.x;
                        cim[u][v][q] = x.y;
                    }
                }
            }
        }
    const double sg = HERK ? -1.0 : 1.0;
    for (int kc = 0; kc < TB; kc += KS) {
        __syncthreads();
        for (int e = tid; e < TB * KS; e += 256) {
            const int r = e / KS, k = e - r * KS;
            const bool kin = kc + k < kmax;
            As[r][k] = (kin && r0 + r < L) ? Arow[(size_t)r * L + kc + k] : czero();
            Bs[r][k] = (kin && (HERK ? c0 + r < L : true)) ? Brow[(size_t)r * ldb + kc + k] : czero();
        }
        __syncthreads();
#pragma unroll
        for (int s = 0; s < KS / 4; ++s) {
            cd av[2], bv[2];
#pragma unroll
            for (int u = 0; u < 2; ++u) av[u] = As[wr + 16 * u + li][4 * s + lk];
#pragma unroll
            for (int v = 0; v < 2; ++v) bv[v] = Bs[wc + 16 * v + li][4 * s + lk];
#pragma unroll
            for (int u = 0; u < 2; ++u)
#pragma unroll
                for (int v = 0; v < 2; ++v) {
                    // C += sg A conj(B)^T:  re += ar br + ai bi ; im += ai br - ar bi
                    cre[u][v] = mfma4(sg * av[u].x, bv[v].x, cre[u][v]);
                    cre[u][v] = mfma4(sg * av[u].y, bv[v].y, cre[u][v]);
                    cim[u][v] = mfma4(sg * av[u].y, bv[v].x, cim[u][v]);
                    cim[u][v] = mfma4(-sg * av[u].x, bv[v].y, cim[u][v]);
                }
        }
    }
    __syncthreads();   // TRSM writes in place over its own A operand
#pragma unroll
    for (int u = 0; u < 2; ++u)
#pragma unroll
        for (int v = 0; v < 2; ++v)
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                const int r = r0 + wr + 16 * u + lk + 4 * q, c = c0 + wc + 16 * v + li;
                if (r < L && c < L && (HERK || c < k0 + kmax))
                    R[(size_t)r * L + c] = cmk(cre[u][v][q], cim[u][v][q]);
            }
}

// ---------------------------------------------------------------- triangular solves
// One workgroup (256 threads = 16 rows x 16 k-lanes) per trial.  Forward L y = B^H and
// back L^H x = y blocked by 16; the 16 x 16 diagonal blocks are applied through their
// inverses: Di[c][c] = 1 / L[c][c], Di[c2][c] = conj(R[c][c2]) (c2 > c, chol.hip).
// y lives in the rhs buffer (L x NR, too large for LDS at cfg 2); theta = conj(x).
__global__ __launch_bounds__(256) void trisolve_kernel(MstepArgs a, int L, int NR) {
    const int b = blockIdx.x;
    if (a.done && a.done[b]) return;
    __shared__ cd z[16][8];
    __shared__ cd Dl[16][17];
    const cd* R = a.R + (size_t)b * L * L;
    cd* y = a.rhs + (size_t)b * L * NR;
    const int tid = threadIdx.x, rr = tid >> 4, kl = tid & 15;
    const int nblk = (L + 15) / 16;
    // ---- forward ----
    for (int bk = 0; bk < nblk; ++bk) {
        const int k0 = bk * 16, w = (L - k0) < 16 ? (L - k0) : 16;
        cd acc[8];
#pragma unroll
        for (int r = 0; r < 8; ++r) acc[r] = czero();
        if (rr < w) {
            const cd* row = R + (size_t)(k0 + rr) * L;
            for (int k = kl; k < k0; k += 16) {
                const cd l = row[k];
#pragma unroll
                for (int r = 0; r < 8; ++r)
                    if (r < NR) acc[r] = cfma(acc[r], l, y[(size_t)k * NR + r]);
            }
        }
#pragma unroll
        for (int r = 0; r < 8; ++r) {
            for (int off = 8; off >= 1; off >>= 1) {
                acc[r].x += __shfl_xor(acc[r].x, off);
                acc[r].y += __shfl_xor(acc[r].y, off);
            }
        }
        // Di of this block (lower): diag 1/L[c][c], strict lower conj(R[c][c2]) transposed
        {
            const int c = tid >> 4, c2 = tid & 15;
            cd v = czero();
            if (c < w && c2 < w) {
                if (c2 == c) {
                    const double d = R[(size_t)(k0 + c) * L + k0 + c].x;
                    v = cmk(d > 0.0 ? 1.0 / d : 0.0, 0.0);
                } else if (c2 < c) {
                    v = cconj(R[(size_t)(k0 + c2) * L + k0 + c]);
                }
            }
            Dl[c][c2] = v;
        }
        if (kl == 0 && rr < w) {
#pragma unroll
            for (int r = 0; r < 8; ++r)
                if (r < NR) z[rr][r] = csub(y[(size_t)(k0 + rr) * NR + r], acc[r]);
        }
        __syncthreads();
        if (tid < w * NR) {
            const int c = tid / NR, r = tid - c * NR;
            cd s = czero();
            for (int c2 = 0; c2 <= c; ++c2) s = cfma(s, Dl[c][c2], z[c2][r]);
            y[(size_t)(k0 + c) * NR + r] = s;
        }
        __syncthreads();
    }
    // ---- back: x_b = Di_b^H (y_b - sum_{m > b} L[m][b]^H x_m) ----
    for (int bk = nblk - 1; bk >= 0; --bk) {
        const int k0 = bk * 16, w = (L - k0) < 16 ? (L - k0) : 16;
        const int c = rr;                                   // column of this block
        cd acc[8];
#pragma unroll
        for (int r = 0; r < 8; ++r) acc[r] = czero();
        if (c < w) {
            for (int m = k0 + 16 + kl; m < L; m += 16) {
                const cd l = R[(size_t)m * L + k0 + c];
#pragma unroll
                for (int r = 0; r < 8; ++r)
                    if (r < NR) acc[r] = cfmac(acc[r], y[(size_t)m * NR + r], l);
            }
        }
#pragma unroll
        for (int r = 0; r < 8; ++r) {
            for (int off = 8; off >= 1; off >>= 1) {
                acc[r].x += __shfl_xor(acc[r].x, off);
                acc[r].y += __shfl_xor(acc[r].y, off);
            }
        }
        {
            const int cc = tid >> 4, c2 = tid & 15;
            cd v = czero();
            if (cc < w && c2 < w) {
                if (c2 == cc) {
                    const double d = R[(size_t)(k0 + cc) * L + k0 + cc].x;
                    v = cmk(d > 0.0 ? 1.0 / d : 0.0, 0.0);
                } else if (c2 < cc) {
                    v = cconj(R[(size_t)(k0 + c2) * L + k0 + cc]);
                }
            }
            Dl[cc][c2] = v;                                 // Di[cc][c2]
        }
        if (kl == 0 && c < w) {
#pragma unroll
            for (int r = 0; r < 8; ++r)
                if (r < NR) z[c][r] = csub(y[(size_t)(k0 + c) * NR + r], acc[r]);
        }
        __syncthreads();
        if (tid < w * NR) {
            const int c1 = tid / NR, r = tid - c1 * NR;
            cd s = czero();                                 // x[c1] = sum_{c2 >= c1} conj(Di[c2][c1]) z[c2]
            for (int c2 = c1; c2 < w; ++c2) s = cfmac(s, z[c2][r], Dl[c2][c1]);
            y[(size_t)(k0 + c1) * NR + r] = s;
        }
        __syncthreads();
    }
    cd* th = a.theta + (size_t)b * L * NR;
    for (int e = tid; e < L * NR; e += 256) th[e] = cconj(y[e]);
}

}  // namespace

bool rbuild_tile_supported(const Problem& pb) { return pb.NT == 4 || pb.NT == 8; }

hipError_t launch_pilot_factor(const Problem& pb, const MstepArgs& a, hipStream_t s) {
    if (pb.Tp == 0 || pb.B == 0) return hipSuccess;
    hipLaunchKernelGGL(pilot_factor_kernel, dim3(pb.Tp, pb.B), dim3(64), 0, s, a, pb.P, pb.NT,
                       pb.Tp, pb.L);
    return hipGetLastError();
}

hipError_t launch_rbuild_tiles(const Problem& pb, const MstepArgs& a, hipStream_t s) {
    const int ntr = (pb.L + TB - 1) / TB;
    const dim3 g(ntr * (ntr + 1) / 2, pb.B);
    if (pb.NT == 8)
        hipLaunchKernelGGL(rbuild_tile_kernel<8>, g, dim3(256), 0, s, a, pb.P, pb.Tp, pb.Td, pb.L,
                           ntr);
    else if (pb.NT == 4)
        hipLaunchKernelGGL(rbuild_tile_kernel<4>, g, dim3(256), 0, s, a, pb.P, pb.Tp, pb.Td, pb.L,
                           ntr);
    else
        return hipErrorInvalidValue;
    return hipGetLastError();
}

hipError_t launch_chol_large(const Problem& pb, const MstepArgs& a, hipStream_t s) {
    if (pb.NR > 8) return hipErrorInvalidValue;
    hipLaunchKernelGGL(diag_tol_kernel, dim3(pb.B), dim3(256), 0, s, a, pb.L);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
    const int nb = (pb.L + TB - 1) / TB;
    for (int k = 0; k < nb; ++k) {
        const int k0 = k * TB, w = (pb.L - k0) < TB ? (pb.L - k0) : TB;
        if ((e = launch_chol_tile(pb, a, k0, w, s)) != hipSuccess) return e;
        const int below = nb - k - 1;
        if (below == 0) break;
        hipLaunchKernelGGL(tile_inverse_kernel, dim3(pb.B), dim3(64), TB * TB * sizeof(cd), s, a,
                           pb.L, k0, w);
        hipLaunchKernelGGL(tile_gemm_kernel<false>, dim3(below, pb.B), dim3(256), 0, s, a, pb.L, k);
        hipLaunchKernelGGL(tile_gemm_kernel<true>, dim3(below * (below + 1) / 2, pb.B), dim3(256),
                           0, s, a, pb.L, k);
        if ((e = hipGetLastError()) != hipSuccess) return e;
    }
    hipLaunchKernelGGL(trisolve_kernel, dim3(pb.B), dim3(256), 0, s, a, pb.L, pb.NR);
    return hipGetLastError();
}

}  // namespace sbce
