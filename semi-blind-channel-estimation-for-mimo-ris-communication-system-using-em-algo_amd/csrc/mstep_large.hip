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
//   forward L y = B^H fused: tile_inverse_kernel applies W to y_k, each TRSM tile block
//   subtracts L_ik y_k from its rows; back L^H x = y by column blocks from the last:
//   backdiag_kernel (diagonal tile, 16-blocks through the inverses kept in R's strict upper
//   16 x 16 blocks) then backupd_kernel (all earlier row blocks in parallel).
#include <stdlib.h>

#include "sbce_internal.h"

namespace sbce {

namespace {

typedef double d4v __attribute__((ext_vector_type(4)));
constexpr int TB = 64;      // tile of the blocked factorisation and of the R build
constexpr int KS = 16;      // k-chunk staged in LDS by the tile GEMM
constexpr int kTileGroup = 4;   // column blocks per trailing update (tile_herk_kernel K <= 256)

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
    if (lane == 0 && res > 1e-20 * den) {
        atomicOr(&a.pflag[b], 1);
        if (a.status) atomicOr(&a.status[b], SBCE_STATUS_PILOT);
    }
}

// Pilot part of B^H, once per run: prhs[b][l][r] = sum_tp u_p[tp][l] y_p[tp][r], one thread per
// (l, r), summed in tp order exactly as rhs_dma_kernel's own pilot loop (same bits).
__global__ __launch_bounds__(256) void pilot_rhs_kernel(MstepArgs a, int Tp, int L, int NR) {
    const int b = blockIdx.y;
    const int e = blockIdx.x * blockDim.x + threadIdx.x;
    if (e >= L * NR) return;
    const int l = e / NR, r = e - l * NR;
    const cd* up = a.up + (size_t)b * Tp * L;
    const cd* yp = a.yp + (size_t)b * Tp * NR;
    cd acc = czero();
    for (int tp = 0; tp < Tp; ++tp) acc = cfmac(acc, up[tp * L + l], yp[tp * NR + r]);
    a.prhs[((size_t)b * L + l) * NR + r] = acc;
}

// ---------------------------------------------------------------- R build (MFMA)
// R[(p,i),(q,j)] = sum_t psi_t[p] conj(psi_t[q]) S_t[i][j] over the pairs p >= q, with
// S_t Hermitian.  Writing w = psi_p conj(psi_q) = wr + i wi and S_ij = Sr + i Si (i < j):
//   R[(p,i),(q,j)] = (sum wr Sr - sum wi Si) + i (sum wr Si + sum wi Sr)
//   R[(p,j),(q,i)] = (sum wr Sr + sum wi Si) + i (sum wi Sr - sum wr Si)
//   R[(p,i),(q,i)] = sum wr S_ii + i sum wi S_ii
// so the whole build is two REAL GEMMs over t, [wr | wi] (pairs x T) times the NT^2 real
// columns of the Hermitian S (NT diagonal + NT(NT-1)/2 real + as many imaginary parts):
// half the MFMAs of the complex product of the full S.  Column tiles of 16: item c < 8
// of a tile is an off-diagonal (i,j) (column c = Re S_ij, c + 8 = Im S_ij) or a pair of
// diagonals (d0, d1) (column c = S_d0d0, c + 8 = S_d1d1); the epilogue combines columns
// c and c + 8 with one lane exchange.
//
// Block = 4 waves x TPW pair tiles of 16 consecutive pairs (p-major order, p >= q); the
// phases psi_t of the p and q the block needs (at most min(P, pairs + 1) values, in two
// index segments) and the real S columns are staged per TC-symbol chunk in LDS; per 4
// symbols a lane forms w for (its pair, its symbol) once and feeds 2 NT^2/16 MFMAs.
// Blocks of one trial are placed on one XCD (blockIdx % 8) so psi / S are L2 hits.
template <int NT>
__device__ __forceinline__ void herm_item(int item, int& i, int& j, bool& diag) {
    constexpr int NOFF = NT * (NT - 1) / 2;
    if (item >= NOFF) {
        diag = true;
        i = 2 * (item - NOFF);
        j = i + 1;
        return;
    }
    diag = false;
    int o = item;
    i = 0;
#pragma unroll
    for (int r = 0; r < NT - 1; ++r) {
        const int cnt = NT - 1 - r;
        if (o >= cnt && i == r) { o -= cnt; i = r + 1; }
    }
    j = i + 1 + o;
}

__device__ __forceinline__ void pair_of(int pi, int& p, int& q) {
    int x = (int)((sqrt(8.0 * pi + 1.0) - 1.0) * 0.5);
    while ((x + 1) * (x + 2) / 2 <= pi) ++x;
    while (x * (x + 1) / 2 > pi) --x;
    p = x;
    q = pi - x * (x + 1) / 2;
}

// STR > 0: compile-time LDS row stride (every block stages <= STR phases per symbol):
// the main loop's LDS reads take immediate offsets and the staging needs no index division.
// STR = 0: row stride = the block's phase count (any P).
template <int NT, int TPW, int TC, int STR>
__global__ __launch_bounds__(256) void rbuild_herm_kernel(MstepArgs a, int B, int P, int Tp,
                                                          int Td, int L, int G, int smax) {
    constexpr int NC = NT * NT;                 // real columns of the Hermitian S
    constexpr int NCT = NC / 16;                // 16-column MFMA tiles
    constexpr int PPB = 4 * TPW * 16;           // pairs per block
    constexpr int MS = NT + NT * NT;
    static_assert(NC % 16 == 0, "rbuild_herm: NT in {4, 8}");
    extern __shared__ __attribute__((aligned(16))) char smem[];
    cd* s_psi = reinterpret_cast<cd*>(smem);                    // [TC][STR or cnt] + 64 pad
    double* s_S = reinterpret_cast<double*>(s_psi + (STR > 0 ? TC * STR : TC * smax + 64));

    const int id = blockIdx.x, xcd = id & 7, slot = id >> 3;
    const int b = (slot / G) * 8 + xcd, g = slot - (slot / G) * G;
    if (b >= B) return;
    if (a.done && a.done[b]) return;
    const int npairs = P * (P + 1) / 2;
    const int pi0 = g * PPB;
    if (pi0 >= npairs) return;
    const int pi1 = min(pi0 + PPB, npairs) - 1;
    int pa, qa, pb, qb;
    pair_of(pi0, pa, qa);
    pair_of(pi1, pb, qb);
    // staged index segments: [lo1, hi1] then [lo2, hi2] (possibly empty)
    //   one row:   q in [qa, qb], p = pb                      -> [qa, qb] + [pb, pb]
    //   two rows, disjoint q ranges [qa, pa] and [0, qb]      -> [0, qb] + [qa, pb]
    //   otherwise (rows in between are shorter than a block)  -> [0, pb]
    // so at most (pairs of the block) + 1 <= smax values
    int lo1 = 0, hi1 = pb, lo2 = pb + 1, hi2 = pb;
    if (pa == pb) {
        lo1 = qa; hi1 = qb;
        if (pb > qb) lo2 = pb;
    } else if (pb == pa + 1 && qa > qb + 1) {
        hi1 = qb; lo2 = qa;
    }
    const int n1 = hi1 - lo1 + 1;
    const int cnt = n1 + (hi2 - lo2 + 1);

    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int li = lane & 15, lk = lane >> 4;
    // A-operand rows of pairs past the block's last pair are computed from a valid pair and
    // never stored (rows of the product are independent)
    int sp[TPW], sq[TPW];
#pragma unroll
    for (int u = 0; u < TPW; ++u) {
        const int pi = min(pi0 + (wave * TPW + u) * 16 + li, pi1);
        int p, q;
        pair_of(pi, p, q);
        sp[u] = (p <= hi1 ? p - lo1 : n1 + p - lo2) * (int)sizeof(cd);
        sq[u] = (q <= hi1 ? q - lo1 : n1 + q - lo2) * (int)sizeof(cd);
        if (STR > 0) {                            // + this lane's symbol row lk
            sp[u] += lk * STR * (int)sizeof(cd);
            sq[u] += lk * STR * (int)sizeof(cd);
        }
    }
    // S staging: thread -> fixed (symbol-in-chunk, column) slots; its source offset in S_t
    constexpr int SR = (TC * NC + 255) / 256;
    int soff[SR];
    bool sdiagim[SR];
#pragma unroll
    for (int r = 0; r < SR; ++r) {
        const int c = (tid + 256 * r) % NC;
        const int cc = c & 15, item = (c >> 4) * 8 + (cc & 7), comp = cc >> 3;
        int i, j;
        bool dg;
        herm_item<NT>(item, i, j, dg);
        soff[r] = dg ? (comp ? j : i) * (NT + 1) : i * NT + j;
        sdiagim[r] = !dg && comp;                 // imaginary part of an off-diagonal
    }
    d4v cr[TPW][NCT], ci[TPW][NCT];
#pragma unroll
    for (int u = 0; u < TPW; ++u)
#pragma unroll
        for (int v = 0; v < NCT; ++v) {
            cr[u][v] = d4v{0.0, 0.0, 0.0, 0.0};
            ci[u][v] = d4v{0.0, 0.0, 0.0, 0.0};
        }
    const cd* psd = a.psid + (size_t)b * Td * P;
    const cd* mom = a.mom + (size_t)b * Td * MS;
    const cd* psp = a.ppsi + (size_t)b * Tp * P;
    const cd* pS = a.pS + (size_t)b * Tp * NT * NT;
    const int T = Td + Tp;
    const char* s_psib = reinterpret_cast<const char*>(s_psi);
    const float rcnt = 1.0f / (float)cnt;
    const int ne = TC * cnt;
    for (int t0 = 0; t0 < T; t0 += TC) {
        __syncthreads();
        if constexpr (STR > 0) {
            // phases: row tt of the LDS image holds the block's cnt (<= STR) phases of symbol
            // t0 + tt; one LDS-DMA wave-instruction per (row, 64-slot segment), the second
            // segment ending at cnt (overlapping the first: identical values)
            for (int sg = 0; sg < (cnt > 64 ? 2 : 1); ++sg) {
                const int kb = sg ? cnt - 64 : 0;
                const int kk = min(kb + lane, cnt - 1);
                const int x = kk < n1 ? lo1 + kk : lo2 + (kk - n1);
                for (int tt = wave; tt < TC; tt += 4) {
                    const int t = t0 + tt;
                    const cd* rowp = t < Td ? psd + (size_t)t * P
                                            : (t < T ? psp + (size_t)(t - Td) * P : psd);
                    __builtin_amdgcn_global_load_lds(
                        (const __attribute__((address_space(1))) void*)(rowp + x),
                        (__attribute__((address_space(3))) void*)(s_psi + tt * STR + kb), 16, 0, 0);
                }
            }
        } else {
            // phases: LDS image linear in e = tt cnt + k, filled by LDS-DMA (global_load_lds,
            // lane-linear destination, per-lane source): every load of the chunk in flight at
            // once instead of a chain of L2 round trips; lanes past the image end land in the
            // 64-entry pad, symbols past T read a valid dummy (their S columns are 0)
            for (int e0 = wave * 64; e0 < ne; e0 += 256) {
                const int e = e0 + lane;
                int tt = (int)((float)e * rcnt);
                int k = e - tt * cnt;
                if (k < 0) { --tt; k += cnt; }
                if (k >= cnt) { ++tt; k -= cnt; }
                const int x = k < n1 ? lo1 + k : lo2 + (k - n1);
                const int t = t0 + tt;
                const cd* src = psd;
                if (e < ne && t < Td) src = psd + (size_t)t * P + x;
                else if (e < ne && t < T) src = psp + (size_t)(t - Td) * P + x;
                __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)src,
                                                 (__attribute__((address_space(3))) void*)(s_psi + e0),
                                                 16, 0, 0);
            }
        }
#pragma unroll
        for (int r = 0; r < SR; ++r) {
            const int e = tid + 256 * r;
            if (SR * 256 == TC * NC || e < TC * NC) {
                const int tt = e / NC, t = t0 + tt;
                double v = 0.0;
                if (t < Td) {
                    const cd z = mom[(size_t)t * MS + NT + soff[r]];
                    v = sdiagim[r] ? z.y : z.x;
                } else if (t < T) {
                    const cd z = pS[(size_t)(t - Td) * NT * NT + soff[r]];
                    v = sdiagim[r] ? z.y : z.x;
                }
                s_S[e] = v;
            }
        }
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
#pragma unroll
        for (int s4 = 0; s4 < TC / 4; ++s4) {
            const int tt = 4 * s4 + lk;
            // STR > 0: lane base + a compile-time offset per s4
            const char* row = STR > 0 ? s_psib + 4 * s4 * STR * (int)sizeof(cd)
                                      : s_psib + tt * cnt * (int)sizeof(cd);
            double bv[NCT];
#pragma unroll
            for (int v = 0; v < NCT; ++v) bv[v] = s_S[tt * NC + 16 * v + li];
#pragma unroll
            for (int u = 0; u < TPW; ++u) {
                const cd w = cmulc(*reinterpret_cast<const cd*>(row + sp[u]),
                                   *reinterpret_cast<const cd*>(row + sq[u]));
#pragma unroll
                for (int v = 0; v < NCT; ++v) {
                    cr[u][v] = mfma4(w.x, bv[v], cr[u][v]);
                    ci[u][v] = mfma4(w.y, bv[v], ci[u][v]);
                }
            }
        }
    }
    // epilogue: lane holds pairs lk + 4 q4 of each tile, column li (p, q stepped from one
    // pair_of: consecutive rows of the p-major pair order)
    int ep[TPW][4], eq[TPW][4];
    {
        int p, q;
        pair_of(min(pi0 + wave * TPW * 16 + lk, pi1), p, q);
#pragma unroll
        for (int u = 0; u < TPW; ++u)
#pragma unroll
            for (int q4 = 0; q4 < 4; ++q4) {
                ep[u][q4] = p;
                eq[u][q4] = q;
                q += 4;
                while (q > p) { q -= p + 1; ++p; }
            }
    }
    cd* R = a.R + (size_t)b * L * L;
    const int comp = li >> 3;
#pragma unroll
    for (int v = 0; v < NCT; ++v) {
        int i, j;
        bool dg;
        herm_item<NT>(v * 8 + (li & 7), i, j, dg);
        const int ri = dg ? (comp ? j : i) : (comp ? j : i);
        const int cj = dg ? (comp ? j : i) : (comp ? i : j);
#pragma unroll
        for (int u = 0; u < TPW; ++u)
#pragma unroll
            for (int q4 = 0; q4 < 4; ++q4) {
                const double orr = cr[u][v][q4], oi = ci[u][v][q4];
                const double pr = __shfl_xor(orr, 8), pim = __shfl_xor(oi, 8);
                double re = orr, im = oi;
                if (!dg) {
                    re = comp ? pr + oi : orr - pim;
                    im = comp ? pim - orr : oi + pr;
                }
                const int pi = pi0 + (wave * TPW + u) * 16 + lk + 4 * q4;
                if (pi <= pi1)
                    R[(size_t)(ep[u][q4] * NT + ri) * L + eq[u][q4] * NT + cj] = cmk(re, im);
            }
    }
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
__global__ __launch_bounds__(64) void tile_inverse_kernel(MstepArgs a, int L, int k0, int w, int NR,
                                                         TileExt ext) {
    const int b = blockIdx.x;
    if (a.done && a.done[b]) return;
    if (ext.col && k0 >= ext.col[b]) return;
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
    if (!ext.fwd) return;
    // fused forward substitution: y_k <- W y_k (every earlier block's L_ik y_i has been
    // subtracted by that block's TRSM launch); lane j owns row j
    cd* yk = a.rhs + ((size_t)b * L + k0) * NR;
    cd* ys = reinterpret_cast<cd*>(col + TB);                // [TB][8]
    for (int e = j; e < w * NR; e += 64) ys[e] = yk[e];
    __syncthreads();
    if (j < w) {
        for (int c = 0; c < NR; ++c) {
            cd acc = czero();
            for (int m = 0; m <= j; ++m) acc = cfma(acc, col[j][m], ys[m * NR + c]);
            yk[j * NR + c] = acc;
        }
    }
}

// ---------------------------------------------------------------- tile GEMM
// C[r][c] = init + sgn sum_k A[r][k] conj(B[c][k]) on a 64 x 64 tile, K = 64.
//   TRSM (HERK = false): tile (i, k), C = A_ik W^H written in place (init 0);
//   HERK (HERK = true):  tile (i, j), C = A_ij - L_ik L_jk^H.
// 4 waves, wave w owns the 32 x 32 quadrant (w >> 1, w & 1) = 2 x 2 MFMA tiles.
template <bool HERK, bool G3 = false>
__global__ __launch_bounds__(256) void tile_gemm_kernel(MstepArgs a, int L, int kb, int NR, TileExt ext) {
    __shared__ cd As[TB][KS + 1], Bs[TB][KS + 1];
    const int b = blockIdx.y;
    if (a.done && a.done[b]) return;
    if (ext.col && kb * TB >= ext.col[b]) return;
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
    if (ext.row && ti * TB >= ext.row[b]) return;
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

    d4v cre[2][2], cim[2][2], c2[2][2];
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
            csub_init<G3>(cre[u][v], cim[u][v], c2[u][v]);
        }
    const double sg = HERK ? 1.0 : -1.0;         // C -= (sg A) conj(B)^T
    // operand chunks (TB x KS of A and B) are loaded into registers one chunk ahead: the
    // global latency of chunk kc + KS overlaps the MFMAs of chunk kc
    constexpr int PF = TB * KS / 256;               // entries per thread and operand
    cd pa[PF], pbv[PF];
    auto fetch = [&](int kc) {
#pragma unroll
        for (int h = 0; h < PF; ++h) {
            const int e = tid + 256 * h, r = e / KS, k = e - r * KS;
            const bool kin = kc + k < kmax;
            pa[h] = (kin && r0 + r < L) ? Arow[(size_t)r * L + kc + k] : czero();
            pbv[h] = (kin && (HERK ? c0 + r < L : true)) ? Brow[(size_t)r * ldb + kc + k] : czero();
        }
    };
    fetch(0);
    for (int kc = 0; kc < TB; kc += KS) {
        __syncthreads();
#pragma unroll
        for (int h = 0; h < PF; ++h) {
            const int e = tid + 256 * h, r = e / KS, k = e - r * KS;
            As[r][k] = pa[h];
            Bs[r][k] = pbv[h];
        }
        __syncthreads();
        if (kc + KS < TB) fetch(kc + KS);
#pragma unroll
        for (int s = 0; s < KS / 4; ++s) {
            cd av[2], bv[2];
#pragma unroll
            for (int u = 0; u < 2; ++u) av[u] = As[wr + 16 * u + li][4 * s + lk];
#pragma unroll
            for (int v = 0; v < 2; ++v) bv[v] = Bs[wc + 16 * v + li][4 * s + lk];
#pragma unroll
            for (int u = 0; u < 2; ++u) {
                const cd va = cmk(sg * av[u].x, sg * av[u].y);
#pragma unroll
                for (int v = 0; v < 2; ++v) csub_step<G3>(cre[u][v], cim[u][v], c2[u][v], va, bv[v]);
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
                    R[(size_t)r * L + c] = csub_out<G3>(cre[u][v], cim[u][v], c2[u][v], q);
            }
    if (!HERK && ext.fwd) {
        // fused forward substitution: rows r0.. of y -= L_ik y_k (the tile just written)
        __syncthreads();
        cd* y = a.rhs + (size_t)b * L * NR;
        for (int e = tid; e < TB * NR; e += 256) {
            const int rr = e / NR, c = e - rr * NR;
            if (r0 + rr >= L) continue;
            const cd* lrow = R + (size_t)(r0 + rr) * L + k0;
            cd acc = czero();
            for (int m = 0; m < kmax; ++m) acc = cfma(acc, lrow[m], y[(size_t)(k0 + m) * NR + c]);
            y[(size_t)(r0 + rr) * NR + c] = csub(y[(size_t)(r0 + rr) * NR + c], acc);
        }
    }
}

// ---------------------------------------------------------------- grouped trailing update
// A_ij -= sum_{k in [kb_lo, kb_lo + nkb)} L_ik L_jk^H on the 64 x 64 tiles (i, j) with
// j in [tj_lo, tj_hi), i >= j: the K loop runs over up to nkb column blocks inside the kernel,
// so a tile's accumulator makes ONE trip through HBM per group of column blocks instead of
// one per block (tile_gemm_kernel<HERK> with K = 64 moved 18x the algorithmic bytes at cfg 2).
// Blocks of one trial sit on one XCD (block id % 8) so the panel rows the trial's tiles share
// are L2 hits.  ext.col: K and the tiles are clipped to the trial's active extent (min-norm
// early exit: columns past it are dropped and never read again).
template <bool G3 = false>
__global__ __launch_bounds__(256) void tile_herk_kernel(MstepArgs a, int L, int kb_lo, int nkb,
                                                        int tj_lo, int tj_hi, int ntiles,
                                                        TileExt ext) {
    __shared__ cd As[TB][KS + 1], Bs[TB][KS + 1];
    const int id = blockIdx.x, xcd = id & 7, slot = id >> 3;
    const int b = (slot / ntiles) * 8 + xcd, tix = slot - (slot / ntiles) * ntiles;
    if (b >= a.nbatch) return;
    if (a.done && a.done[b]) return;
    const int nb = (L + TB - 1) / TB;
    int ti, tj;
    if (tj_hi >= nb) {                      // the whole trailing triangle from tj_lo
        int x = (int)((sqrt(8.0 * tix + 1.0) - 1.0) * 0.5);
        while ((x + 1) * (x + 2) / 2 <= tix) ++x;
        while (x * (x + 1) / 2 > tix) --x;
        ti = tj_lo + x;
        tj = tj_lo + (tix - x * (x + 1) / 2);
    } else {                                // a few columns: tiles column by column
        int t = tix;
        tj = tj_lo;
        while (t >= nb - tj) { t -= nb - tj; ++tj; }
        ti = tj + t;
    }
    const int k0 = kb_lo * TB;
    int kend = (kb_lo + nkb) * TB < L ? (kb_lo + nkb) * TB : L;
    if (ext.col) {
        const int act = ext.col[b];
        if (tj * TB >= act) return;         // dropped columns: never read again
        kend = kend < act ? kend : act;
    }
    if (k0 >= kend) return;
    if (ext.row && ti * TB >= ext.row[b]) return;
    cd* R = a.R + (size_t)b * L * L;
    const int r0 = ti * TB, c0 = tj * TB;
    const cd* Arow = R + (size_t)r0 * L;
    const cd* Brow = R + (size_t)c0 * L;
    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int li = lane & 15, lk = lane >> 4;
    const int wr = (wave >> 1) * 32, wc = (wave & 1) * 32;

    d4v cre[2][2], cim[2][2], c2[2][2];
#pragma unroll
    for (int u = 0; u < 2; ++u)
#pragma unroll
        for (int v = 0; v < 2; ++v) {
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                const int r = r0 + wr + 16 * u + lk + 4 * q, c = c0 + wc + 16 * v + li;
                const cd x = (r < L && c < L) ? R[(size_t)r * L + c] : czero();
                cre[u][v][q] = x.x;
                cim[u][v][q] = x.y;
            }
            csub_init<G3>(cre[u][v], cim[u][v], c2[u][v]);
        }
    constexpr int PF = TB * KS / 256;               // entries per thread and operand
    cd pa[PF], pbv[PF];
    auto fetch = [&](int kc) {
#pragma unroll
        for (int h = 0; h < PF; ++h) {
            const int e = tid + 256 * h, r = e / KS, k = e - r * KS;
            const bool kin = kc + k < kend;
            pa[h] = (kin && r0 + r < L) ? Arow[(size_t)r * L + kc + k] : czero();
            pbv[h] = (kin && c0 + r < L) ? Brow[(size_t)r * L + kc + k] : czero();
        }
    };
    fetch(k0);
    for (int kc = k0; kc < kend; kc += KS) {
        __syncthreads();
#pragma unroll
        for (int h = 0; h < PF; ++h) {
            const int e = tid + 256 * h, r = e / KS, k = e - r * KS;
            As[r][k] = pa[h];
            Bs[r][k] = pbv[h];
        }
        __syncthreads();
        if (kc + KS < kend) fetch(kc + KS);
#pragma unroll
        for (int s4 = 0; s4 < KS / 4; ++s4) {
            cd av[2], bv[2];
#pragma unroll
            for (int u = 0; u < 2; ++u) av[u] = As[wr + 16 * u + li][4 * s4 + lk];
#pragma unroll
            for (int v = 0; v < 2; ++v) bv[v] = Bs[wc + 16 * v + li][4 * s4 + lk];
#pragma unroll
            for (int u = 0; u < 2; ++u)
#pragma unroll
                for (int v = 0; v < 2; ++v)      // C -= A conj(B)^T
                    csub_step<G3>(cre[u][v], cim[u][v], c2[u][v], av[u], bv[v]);
        }
    }
#pragma unroll
    for (int u = 0; u < 2; ++u)
#pragma unroll
        for (int v = 0; v < 2; ++v)
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                const int r = r0 + wr + 16 * u + lk + 4 * q, c = c0 + wc + 16 * v + li;
                if (r < L && c < L) R[(size_t)r * L + c] = csub_out<G3>(cre[u][v], cim[u][v], c2[u][v], q);
            }
}

// dvec[b][j] -= sum_{m in [c0, c1)} |L[j][m]|^2 for rows j >= r0 = c1 (c1 clipped to the active
// extent): the diagonal of the Schur complement after a group, for the min-norm early exit.
// One wave per row (coalesced row segments), lanes reduced in a fixed order.
__global__ __launch_bounds__(256) void dvec_kernel(MstepArgs a, int L, int c0, int r0, TileExt ext) {
    const int b = blockIdx.y;
    if (a.done && a.done[b]) return;
    int c1 = r0;
    if (ext.col) c1 = c1 < ext.col[b] ? c1 : ext.col[b];
    if (c0 >= c1) return;
    const int j = r0 + blockIdx.x * 4 + (threadIdx.x >> 6), lane = threadIdx.x & 63;
    if (j >= L) return;
    const cd* row = a.R + (size_t)b * L * L + (size_t)j * L;
    double sq = 0.0;
    for (int m = c0 + lane; m < c1; m += 64) sq += cabs2(row[m]);
    for (int off = 32; off >= 1; off >>= 1) sq += __shfl_xor(sq, off);
    if (lane == 0) a.dvec[(size_t)b * L + j] -= sq;
}

// ---------------------------------------------------------------- back substitution
// L^H x = y by 64-column blocks from the last: backdiag_kernel (one workgroup per trial)
// solves the diagonal tile, x_k = L_kk^{-H} y_k, in 16-row blocks through the inverses kept
// in R's strict upper 16 x 16 blocks (Di[c][c] = 1 / L[c][c], Di[c2][c] = conj(R[c][c2])),
// y_k already holding y_k - sum_{i > k} L_ik^H x_i; backupd_kernel then subtracts
// L_kj^H x_k from every earlier block j in parallel.  theta = conj(x) after the first block.
__global__ __launch_bounds__(256) void backdiag_kernel(MstepArgs a, int L, int NR, int k0, int w,
                                                       const int32_t* ext) {
    const int b = blockIdx.x;
    if (a.done && a.done[b]) return;
    if (ext && k0 >= ext[b]) return;
    __shared__ cd z[16][8];
    __shared__ cd Dl[16][17];
    const cd* R = a.R + (size_t)b * L * L;
    cd* y = a.rhs + (size_t)b * L * NR;
    const int tid = threadIdx.x, rr = tid >> 4, kl = tid & 15;
    const int kend = k0 + w;
    for (int c0 = k0 + (w - 1) / 16 * 16; c0 >= k0; c0 -= 16) {
        const int wb = (kend - c0) < 16 ? (kend - c0) : 16;
        const int c = rr;                                   // column of this 16-block
        cd acc[8];
#pragma unroll
        for (int r = 0; r < 8; ++r) acc[r] = czero();
        if (c < wb) {
            for (int m = c0 + 16 + kl; m < kend; m += 16) {
                const cd l = R[(size_t)m * L + c0 + c];
#pragma unroll
                for (int r = 0; r < 8; ++r)
                    if (r < NR) acc[r] = cfmac(acc[r], y[(size_t)m * NR + r], l);
            }
        }
#pragma unroll
        for (int r = 0; r < 8; ++r)
            for (int off = 8; off >= 1; off >>= 1) {
                acc[r].x += __shfl_xor(acc[r].x, off);
                acc[r].y += __shfl_xor(acc[r].y, off);
            }
        {
            const int cc = tid >> 4, c2 = tid & 15;
            cd v = czero();
            if (cc < wb && c2 < wb) {
                if (c2 == cc) {
                    const double d = R[(size_t)(c0 + cc) * L + c0 + cc].x;
                    v = cmk(d > 0.0 ? 1.0 / d : 0.0, 0.0);
                } else if (c2 < cc) {
                    v = cconj(R[(size_t)(c0 + c2) * L + c0 + cc]);
                }
            }
            Dl[cc][c2] = v;                                 // Di[cc][c2]
        }
        if (kl == 0 && c < wb) {
#pragma unroll
            for (int r = 0; r < 8; ++r)
                if (r < NR) z[c][r] = csub(y[(size_t)(c0 + c) * NR + r], acc[r]);
        }
        __syncthreads();
        if (tid < wb * NR) {
            const int c1 = tid / NR, r = tid - c1 * NR;
            cd s = czero();                                 // x[c1] = sum_{c2 >= c1} conj(Di[c2][c1]) z[c2]
            for (int c2 = c1; c2 < wb; ++c2) s = cfmac(s, z[c2][r], Dl[c2][c1]);
            y[(size_t)(c0 + c1) * NR + r] = s;
        }
        __syncthreads();
    }
    if (k0 == 0 && a.theta) {
        cd* th = a.theta + (size_t)b * L * NR;
        for (int e = tid; e < L * NR; e += 256) th[e] = cconj(y[e]);
    }
}

// Block (j, trial): y_j -= L_kj^H x_k for row block j < k: the tile (k, j) and x_k staged in
// LDS (coalesced rows), thread per (row r of y_j, right-hand side).
__global__ __launch_bounds__(256) void backupd_kernel(MstepArgs a, int L, int NR, int k0, int w,
                                                      const int32_t* ext) {
    const int j = blockIdx.x, b = blockIdx.y;
    if (a.done && a.done[b]) return;
    if (ext && k0 >= ext[b]) return;
    extern __shared__ __attribute__((aligned(16))) char smem[];
    cd(*T)[TB + 1] = reinterpret_cast<cd(*)[TB + 1]>(smem);  // [TB][TB + 1]: T[m][r] = L[k0+m][j0+r]
    cd* xs = reinterpret_cast<cd*>(smem + (size_t)TB * (TB + 1) * sizeof(cd));   // [TB][NR]
    const cd* R = a.R + (size_t)b * L * L;
    cd* y = a.rhs + (size_t)b * L * NR;
    const int j0 = j * TB, tid = threadIdx.x;
    for (int e = tid; e < w * TB; e += 256) {
        const int m = e / TB, r = e - m * TB;
        T[m][r] = R[(size_t)(k0 + m) * L + j0 + r];
    }
    for (int e = tid; e < w * NR; e += 256) xs[e] = y[(size_t)k0 * NR + e];
    __syncthreads();
    for (int e = tid; e < TB * NR; e += 256) {
        const int r = e / NR, c = e - r * NR;
        cd acc = czero();
        for (int m = 0; m < w; ++m) acc = cfmac(acc, xs[m * NR + c], T[m][r]);
        y[(size_t)(j0 + r) * NR + c] = csub(y[(size_t)(j0 + r) * NR + c], acc);
    }
}

}  // namespace

bool rbuild_herm_supported(const Problem& pb) { return pb.NT == 4 || pb.NT == 8; }

hipError_t launch_pilot_factor(const Problem& pb, const MstepArgs& a, hipStream_t s) {
    if (hipMemsetAsync(a.pflag, 0, (size_t)pb.B * sizeof(int32_t), s) != hipSuccess)
        return hipErrorInvalidValue;
    if (pb.Tp == 0 || pb.B == 0) return hipSuccess;
    hipLaunchKernelGGL(pilot_factor_kernel, dim3(pb.Tp, pb.B), dim3(64), 0, s, a, pb.P, pb.NT,
                       pb.Tp, pb.L);
    if (a.prhs)
        hipLaunchKernelGGL(pilot_rhs_kernel, dim3((pb.L * pb.NR + 255) / 256, pb.B), dim3(256), 0,
                           s, a, pb.Tp, pb.L, pb.NR);
    return hipGetLastError();
}

template <int NT, int TPW, int TC, int STR>
static hipError_t launch_herm(const Problem& pb, const MstepArgs& a, int smax, hipStream_t s) {
    constexpr int PPB = 4 * TPW * 16;
    const int npairs = pb.P * (pb.P + 1) / 2;
    const int G = (npairs + PPB - 1) / PPB;
    const long nblk = 8L * ((pb.B + 7) / 8) * G;
    const size_t lds = (size_t)(STR > 0 ? TC * STR : TC * smax + 64) * sizeof(cd) +
                       (size_t)TC * NT * NT * sizeof(double);
    if (STR > 0 && smax > STR) return hipErrorInvalidValue;
    if (nblk > 0x7fffffffL || lds > 160 * 1024) return hipErrorInvalidValue;
    hipLaunchKernelGGL((rbuild_herm_kernel<NT, TPW, TC, STR>), dim3((unsigned)nblk), dim3(256), lds, s, a,
                       pb.B, pb.P, pb.Tp, pb.Td, pb.L, G, smax);
    return hipGetLastError();
}

hipError_t launch_rbuild_herm(const Problem& pb, const MstepArgs& a, hipStream_t s) {
    // staged phases per block <= min(P, pairs per block + 1) (two p-major index segments)
    if (pb.NT == 4) {
        const int smax = pb.P < 257 ? pb.P : 257;
        // 16-symbol chunks (19 KB of LDS per block: more resident blocks per CU); measured
        // at cfg1 against 8 / 32 / 64 and 2 / 6 / 8 tiles per wave: 16 x 4 and 16 x 6 lead by
        // ~2 % of the M-step
        if (smax <= 68) return launch_herm<4, 4, 16, 68>(pb, a, smax, s);
        return smax <= 130 ? launch_herm<4, 4, 32, 0>(pb, a, smax, s)
                           : launch_herm<4, 4, 8, 0>(pb, a, smax, s);
    }
    if (pb.NT == 8) {
        const int smax = pb.P < 65 ? pb.P : 65;
        return launch_herm<8, 1, 16, 68>(pb, a, smax, s);
    }
    return hipErrorInvalidValue;
}

hipError_t launch_diag_tol(const Problem& pb, const MstepArgs& a, hipStream_t s) {
    hipLaunchKernelGGL(diag_tol_kernel, dim3(pb.B), dim3(256), 0, s, a, pb.L);
    return hipGetLastError();
}

static hipError_t launch_herk(const Problem& pb, const MstepArgs& a, int kb_lo, int nkb, int tj_lo,
                              int tj_hi, const TileExt& ex, hipStream_t s) {
    const int nb = (pb.L + TB - 1) / TB;
    long ntiles = 0;
    for (int tj = tj_lo; tj < tj_hi; ++tj) ntiles += nb - tj;
    if (ntiles <= 0) return hipSuccess;
    const long nblk = 8L * ((pb.B + 7) / 8) * ntiles;
    if (nblk > 0x7fffffffL) return hipErrorInvalidValue;
    if (g_debug.cplx3 && (a.solve_mode == SBCE_SOLVE_CHOL || a.solve_mode == kSolveClampHpd))
        hipLaunchKernelGGL(tile_herk_kernel<true>, dim3((unsigned)nblk), dim3(256), 0, s, a, pb.L, kb_lo,
                           nkb, tj_lo, tj_hi, (int)ntiles, ex);
    else
        hipLaunchKernelGGL(tile_herk_kernel<false>, dim3((unsigned)nblk), dim3(256), 0, s, a, pb.L, kb_lo,
                           nkb, tj_lo, tj_hi, (int)ntiles, ex);
    return hipGetLastError();
}

hipError_t launch_tile_factor_step(const Problem& pb, const MstepArgs& a, int k, const TileExt& ex,
                                   hipStream_t s) {
    const int nb = (pb.L + TB - 1) / TB;
    const int k0 = k * TB, w = (pb.L - k0) < TB ? (pb.L - k0) : TB;
    hipError_t e = launch_chol_tile(pb, a, k0, w, ex.col, s);
    if (e != hipSuccess) return e;
    // W = L_kk^-1 (and the fused forward substitution y_k <- W y_k when ex.fwd)
    const size_t inv_lds = (size_t)TB * TB * sizeof(cd) + (size_t)TB * 8 * sizeof(cd);
    hipLaunchKernelGGL(tile_inverse_kernel, dim3(pb.B), dim3(64), inv_lds, s, a, pb.L, k0, w, pb.NR, ex);
    const int below = nb - k - 1;
    if (below > 0 && g_debug.cplx3 && (a.solve_mode == SBCE_SOLVE_CHOL || a.solve_mode == kSolveClampHpd))
        hipLaunchKernelGGL((tile_gemm_kernel<false, true>), dim3(below, pb.B), dim3(256), 0, s, a, pb.L, k,
                           pb.NR, ex);
    else if (below > 0)
        hipLaunchKernelGGL((tile_gemm_kernel<false, false>), dim3(below, pb.B), dim3(256), 0, s, a, pb.L, k,
                           pb.NR, ex);
    return hipGetLastError();
}

// Blocked LEFT-looking factorisation by groups of kTileGroup column blocks (256 columns): per
// group, ONE update of the group's columns (rows below them too) by every earlier column
// (tile_herk_kernel, the K loop in the kernel), then per block k of the group the diagonal
// tile, its inverse, the TRSM tiles below it and the narrow update of the group's remaining
// columns by block k.  No trailing update is ever made: on a rank-deficient R (the min-norm
// solve) the columns past the numerical rank are never touched, so the work stops at the
// rank (cfg 4: ~530 of 4100 columns) instead of sweeping the whole trailing matrix.
// act_check (min-norm): before each group, act_kernel ends a trial's factorisation when the
// Schur complement's diagonal (a.dvec, kept current by dvec_kernel) is below the cut.
hipError_t launch_tile_factor(const Problem& pb, const MstepArgs& a, const TileExt& ex,
                              hipError_t (*act_check)(const Problem&, const MstepArgs&, int, hipStream_t),
                              hipStream_t s) {
    const int nb = (pb.L + TB - 1) / TB;
    hipError_t e;
    for (int g0 = 0; g0 < nb; g0 += kTileGroup) {
        const int g1 = (g0 + kTileGroup) < nb ? (g0 + kTileGroup) : nb;
        if (act_check && (e = act_check(pb, a, g0 * TB, s)) != hipSuccess) return e;
        if (g0 > 0 && (e = launch_herk(pb, a, 0, g0, g0, g1, ex, s)) != hipSuccess) return e;
        for (int k = g0; k < g1; ++k) {
            if ((e = launch_tile_factor_step(pb, a, k, ex, s)) != hipSuccess) return e;
            if (k + 1 < g1 && (e = launch_herk(pb, a, k, 1, k + 1, g1, ex, s)) != hipSuccess)
                return e;
        }
        if (act_check && g1 < nb) {
            // the Schur complement's diagonal past the group: dvec[j] -= sum_{m in group} |L_jm|^2
            const int r0 = g1 * TB;
            hipLaunchKernelGGL(dvec_kernel, dim3((pb.L - r0 + 3) / 4, pb.B), dim3(256), 0, s, a,
                               pb.L, g0 * TB, r0, ex);
            if ((e = hipGetLastError()) != hipSuccess) return e;
        }
    }
    return hipSuccess;
}

hipError_t launch_tile_back(const Problem& pb, const MstepArgs& a, const int32_t* ext, hipStream_t s) {
    const int nb = (pb.L + TB - 1) / TB;
    const size_t upd_lds = (size_t)TB * (TB + 1) * sizeof(cd) + (size_t)TB * 8 * sizeof(cd);
    hipError_t e;
    for (int k = nb - 1; k >= 0; --k) {
        const int k0 = k * TB, w = (pb.L - k0) < TB ? (pb.L - k0) : TB;
        hipLaunchKernelGGL(backdiag_kernel, dim3(pb.B), dim3(256), 0, s, a, pb.L, pb.NR, k0, w, ext);
        if (k > 0)
            hipLaunchKernelGGL(backupd_kernel, dim3(k, pb.B), dim3(256), upd_lds, s, a, pb.L, pb.NR,
                               k0, w, ext);
        if ((e = hipGetLastError()) != hipSuccess) return e;
    }
    return hipSuccess;
}

hipError_t launch_chol_large(const Problem& pb, const MstepArgs& a, hipStream_t s) {
    if (pb.NR > 8) return hipErrorInvalidValue;
    hipError_t e = launch_diag_tol(pb, a, s);
    if (e != hipSuccess) return e;
    const TileExt full{nullptr, nullptr, 1};
    if ((e = launch_tile_factor(pb, a, full, nullptr, s)) != hipSuccess) return e;
    return launch_tile_back(pb, a, nullptr, s);
}

}  // namespace sbce
