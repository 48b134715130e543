// Minimum-norm M-step solve (SBCE_SOLVE_MINNORM): np.linalg.lstsq of
// "Proposed method/PM.py":108 on the reduced normal equations R X = B^H.
//
// The reference hands the K x K system A = sum Z^H Z (K = L n_rx) to lstsq (PM.py:108; it is
// also the intended fallback of all_detectorsvsTd.py:238-241 / IRS_elements.py:247-249).
// With Z^H Z = conj(u u^H) (x) I (commutation_matrix.py:3-8) A's singular values are R's
// eigenvalues, each n_rx times, so lstsq's default cut rcond = eps * max(K, K) keeps the
// directions of R with eigenvalue > eps K lambda_max(R) and returns the minimum-norm solution
// on them.  On the GPU, per trial:
//
//   lanczos_tol_kernel  lambda_max(R) by 4 Lanczos steps (one workgroup per trial streaming
//                       R's lower triangle once per step); cut = eps K max(lambda, max diag R);
//   tiled Cholesky of R (mstep_large.hip) whose pivots at or below tau = 32 cut are dropped
//                       (their columns zeroed), R = G G^H with G lower triangular; act_kernel
//                       ends a trial's factorisation once every remaining diagonal entry of the
//                       Schur complement is below tau (all later pivots would be dropped).
//                       The factor 32: an unpivoted Cholesky's pivots past the numerical rank
//                       are rounding noise of up to ~j eps max(diag R) -- measured up to 15 cut
//                       at n_rx = 1, 0.7 cut at n_rx = 2..4 -- and a kept noise pivot would be
//                       amplified by the later eliminations, while genuine pivots of exactly
//                       rank-deficient systems sit >= 1e8 cut above it;
//   gram_kernel         C = G^H G on the active extent (64 x 64 MFMA tiles; a dropped column
//                       gives C_jj = 1, an uncoupled identity direction);
//   ghb_kernel          c = G^H B^H;
//   tiled Cholesky of C = F F^H with the fused forward substitution, then F^-H, F^-1, F^-H
//                       (fwddiag / fwdupd kernels + mstep_large.hip's back substitution);
//   gz_kernel           x = G z, theta = conj(x):  x = G (G^H G)^-2 G^H b = R^+ b.
//
// A pivot inside [4 cut, 64 tau] (or an early exit with a trailing diagonal above 4 cut) flags
// SBCE_STATUS_RANK: there the pivot-based rank may differ from lstsq's singular values.  A
// genuine direction of R BELOW the cut is removed along its Cholesky pivot rather than its
// eigenvector: theta then differs from lstsq by ~ lambda_dropped / lambda_kept_min (measured
// 1e-5 at BASELINE cfg 4, iteration 0: one eigenvalue at 0.13 cut; NMSE unchanged at 1e-3).
#include "sbce_internal.h"

namespace sbce {

namespace {

typedef double d4v __attribute__((ext_vector_type(4)));
constexpr int TB = 64;            // tile of the blocked factorisation (mstep_large.hip)
constexpr int KS = 16;            // k-chunk of the Gram tiles
constexpr int kLanczosSteps = 4;   // lambda_max to ~10 % (the cut carries a 32x margin)
constexpr double kCutSafety = 32.0;   // tau = kCutSafety * cut (see the header comment)
constexpr double kEps = 2.220446049250313e-16;   // numpy.finfo(float).eps

__device__ __forceinline__ d4v mfma4(double a, double b, d4v c) {
    return __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c, 0, 0, 0);
}

// deterministic block reductions (256 threads, fixed tree order)
__device__ __forceinline__ double block_sum(double v, double* red) {
    for (int off = 32; off >= 1; off >>= 1) v += __shfl_xor(v, off);
    __syncthreads();
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = v;
    __syncthreads();
    return (red[0] + red[1]) + (red[2] + red[3]);
}
__device__ __forceinline__ double block_max(double v, double* red) {
    for (int off = 32; off >= 1; off >>= 1) v = fmax(v, __shfl_xor(v, off));
    __syncthreads();
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = v;
    __syncthreads();
    return fmax(fmax(red[0], red[1]), fmax(red[2], red[3]));
}

// Largest eigenvalue of the k x k symmetric tridiagonal (al, be) by Sturm-count bisection.
__device__ double tridiag_max_eig(const double* al, const double* be, int k) {
    double lo = al[0], hi = al[0];
    for (int i = 0; i < k; ++i) {
        const double r = (i > 0 ? fabs(be[i - 1]) : 0.0) + (i + 1 < k ? fabs(be[i]) : 0.0);
        lo = fmin(lo, al[i] - r);
        hi = fmax(hi, al[i] + r);
    }
    for (int it = 0; it < 200 && hi - lo > 1e-15 * fmax(fabs(hi), fabs(lo)); ++it) {
        const double x = 0.5 * (lo + hi);
        int below = 0;                             // eigenvalues < x
        double q = 1.0;
        for (int i = 0; i < k; ++i) {
            const double b2 = i > 0 ? be[i - 1] * be[i - 1] : 0.0;
            q = al[i] - x - (i > 0 ? b2 / q : 0.0);
            if (q == 0.0) q = -1e-300;
            below += q < 0.0;
        }
        if (below == k) hi = x; else lo = x;
    }
    return hi;
}

// ---------------------------------------------------------------- lambda_max -> cut
// One workgroup of kLzWaves waves per trial.  Matvec y = R v from the lower triangle, each
// 64 x 64 tile read once by one wave (tile J of row block I -> wave J % kLzWaves), row by row:
// lane = column, so every load is one coalesced 1 KB row segment.  The column products
// conj(R[r][c]) v[r] (strict lower part) accumulate in the lane and go to y[c] after the tile
// (one writer per y entry per row block); the row products R[r][c] v[c] are reduce-scattered
// over the lanes 16 rows at a time, kept per lane across the wave's tiles of the row block and
// summed over the waves in a fixed order -- deterministic.  v (and y when it fits) in LDS.
constexpr int kLzWaves = 8;
template <bool YLDS>
__global__ __launch_bounds__(64 * kLzWaves) void lanczos_tol_kernel(MstepArgs a, int L, int K) {
    const int b = blockIdx.x;
    if (a.done && a.done[b]) return;
    extern __shared__ __attribute__((aligned(16))) char smem[];
    __shared__ double part[kLzWaves][TB][2];
    __shared__ double red[kLzWaves];
    __shared__ double al[kLanczosSteps], be[kLanczosSteps];
    cd* v = reinterpret_cast<cd*>(smem);
    cd* scr = a.gram + (size_t)b * L * L;          // free until the Gram build
    cd* y = YLDS ? v + L : scr;
    cd* vp = scr + L;
    const cd* R = a.R + (size_t)b * L * L;
    constexpr int NTH = 64 * kLzWaves;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int nb = (L + TB - 1) / TB;
    auto bsum = [&](double x) {
        for (int off = 32; off >= 1; off >>= 1) x += __shfl_xor(x, off);
        __syncthreads();
        if (lane == 0) red[wave] = x;
        __syncthreads();
        double t = 0.0;
        for (int w = 0; w < kLzWaves; ++w) t += red[w];
        return t;
    };
    double md = 0.0;
    const double v0 = 1.0 / sqrt((double)L);
    for (int i = tid; i < L; i += NTH) {
        const double di = R[(size_t)i * L + i].x;
        md = fmax(md, di);
        a.dvec[(size_t)b * L + i] = di;     // the Schur complement's diagonal before any column
        v[i] = cmk(v0, 0.0);
        vp[i] = czero();
    }
    for (int off = 32; off >= 1; off >>= 1) md = fmax(md, __shfl_xor(md, off));
    __syncthreads();
    if (lane == 0) red[wave] = md;
    __syncthreads();
    for (int w = 0; w < kLzWaves; ++w) md = fmax(md, red[w]);
    int ks = 0;
    double bprev = 0.0;
    for (int st = 0; st < kLanczosSteps; ++st) {
        for (int i = tid; i < L; i += NTH) y[i] = czero();
        __syncthreads();
        for (int I = 0; I < nb; ++I) {
            const int r0 = I * TB;
            const int nr = (L - r0) < TB ? (L - r0) : TB;
            // after the reduce-scatter lane l holds value l >> 1 of the 16-row chunk: row l >> 2,
            // component (l >> 1) & 1 (lanes l and l ^ 1 hold the same sum)
            double rowacc[4] = {0.0, 0.0, 0.0, 0.0};
            for (int J = wave; J <= I; J += kLzWaves) {
                const int c = J * TB + lane;
                const bool cv = c < L;
                const cd vc = cv ? v[c] : czero();
                cd cacc = czero();
#pragma unroll
                for (int q = 0; q < 4; ++q) {
                    double d[32];
                    cd g[16];
#pragma unroll
                    for (int i = 0; i < 16; ++i) {
                        const int r = r0 + 16 * q + i;
                        g[i] = (cv && 16 * q + i < nr && (J < I || c <= r)) ? R[(size_t)r * L + c]
                                                                           : czero();
                    }
#pragma unroll
                    for (int i = 0; i < 16; ++i) {
                        const int r = r0 + 16 * q + i;
                        const cd p = cmul(g[i], vc);                      // row product
                        d[2 * i] = p.x;
                        d[2 * i + 1] = p.y;
                        if (J < I || c < r) cacc = cfmac(cacc, (16 * q + i < nr) ? v[r] : czero(), g[i]);
                    }
                    // reduce-scatter of the 16 rows' products: lane ends with value lane >> 1
#pragma unroll
                    for (int m = 32, n = 32; m >= 2; m >>= 1, n >>= 1) {
                        const bool hi = (lane & m) != 0;
#pragma unroll
                        for (int i = 0; i < n / 2; ++i) {
                            const double keep = hi ? d[n / 2 + i] : d[i];
                            const double send = hi ? d[i] : d[n / 2 + i];
                            d[i] = keep + __shfl_xor(send, m);
                        }
                    }
                    rowacc[q] += d[0] + __shfl_xor(d[0], 1);
                }
                if (cv) y[c] = cadd(y[c], cacc);
            }
#pragma unroll
            for (int q = 0; q < 4; ++q)
                if ((lane & 1) == 0) part[wave][16 * q + (lane >> 2)][(lane >> 1) & 1] = rowacc[q];
            __syncthreads();
            if (tid < 2 * nr) {
                const int rr = tid >> 1, comp = tid & 1;
                double t = 0.0;
                for (int w = 0; w < kLzWaves; ++w) t += part[w][rr][comp];
                reinterpret_cast<double*>(y + r0 + rr)[comp] += t;
            }
            __syncthreads();
        }
        // three-term recurrence: alpha = v^H y, w = y - alpha v - beta vp
        double pa = 0.0;
        for (int i = tid; i < L; i += NTH) pa = fma(v[i].x, y[i].x, fma(v[i].y, y[i].y, pa));
        const double alpha = bsum(pa);
        double pw = 0.0;
        for (int i = tid; i < L; i += NTH) {
            const cd w = csub(csub(y[i], cscale(v[i], alpha)), cscale(vp[i], bprev));
            y[i] = w;
            pw += cabs2(w);
        }
        const double beta = sqrt(bsum(pw));
        if (tid == 0) {
            al[st] = alpha;
            be[st] = beta;
        }
        ks = st + 1;
        if (!(beta > 1e-13 * fabs(alpha)) || st + 1 == kLanczosSteps) break;
        const double ib = 1.0 / beta;
        for (int i = tid; i < L; i += NTH) {
            vp[i] = v[i];
            v[i] = cscale(y[i], ib);
        }
        bprev = beta;
        __syncthreads();
    }
    if (tid == 0) {
        const double lam = tridiag_max_eig(al, be, ks);
        a.tol[b] = kCutSafety * kEps * (double)K * fmax(lam, md);
    }
}

// ---------------------------------------------------------------- early exit
// Before column group k0: if every remaining diagonal entry of the Schur complement (dvec, kept
// by mstep_large.hip's dvec_kernel) is at or below the cut, all later pivots would be dropped:
// act[b] = k0 ends the trial's factorisation.
__global__ __launch_bounds__(256) void act_kernel(MstepArgs a, int L, int k0) {
    const int b = blockIdx.x;
    if (a.done && a.done[b]) return;
    if (a.act[b] <= k0) return;
    __shared__ double red[4];
    const double* dv = a.dvec + (size_t)b * L;
    double m = 0.0;
    for (int i = k0 + threadIdx.x; i < L; i += 256) m = fmax(m, dv[i]);
    m = block_max(m, red);
    if (threadIdx.x == 0) {
        const double tol = a.tol[b];
        if (!(m > tol)) {
            a.act[b] = k0;
            if (a.status)
                a.status[b] |= SBCE_STATUS_NONHPD | (m > tol * (1.0 / 8) ? SBCE_STATUS_RANK : 0);
        }
    }
}

// ---------------------------------------------------------------- C = G^H G
// Tile (ti, tj), ti >= tj, of the active extent: C_IJ = sum_{K >= ti} G_KI^H G_KJ over G's row
// tiles; the diagonal tile of a column block (K == I) is masked to its lower triangle (its strict
// upper part holds the factor's 16 x 16 inverse blocks).  4 waves, each a 32 x 32 quadrant of
// 2 x 2 MFMA tiles; 16-row chunks of both column strips staged in LDS.  The tiles of a trial run
// back to back on one XCD (blocks are dealt round-robin over the 8 XCDs), so the strips shared
// by the concurrently running tiles of a row or column are re-read from that XCD's L2.
template <bool G3 = false>
__global__ __launch_bounds__(256) void gram_kernel(MstepArgs a, int L, int ntiles) {
    __shared__ cd As[KS][TB + 1], Bs[KS][TB + 1];
    const int id = blockIdx.x, xcd = id & 7, slot = id >> 3;
    const int b = (slot / ntiles) * 8 + xcd;
    if (b >= a.nbatch) return;
    if (a.done && a.done[b]) return;
    const int tix = slot - (slot / ntiles) * ntiles;
    int x = (int)((sqrt(8.0 * tix + 1.0) - 1.0) * 0.5);
    while ((x + 1) * (x + 2) / 2 <= tix) ++x;
    while (x * (x + 1) / 2 > tix) --x;
    const int ti = x, tj = tix - x * (x + 1) / 2;
    const int act = a.act[b];
    if (ti * TB >= act) return;
    const cd* G = a.R + (size_t)b * L * L;
    cd* C = a.gram + (size_t)b * L * L;
    const int i0 = ti * TB, j0 = tj * TB;
    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int li = lane & 15, lk = lane >> 4;
    const int wr = (wave >> 1) * 32, wc = (wave & 1) * 32;
    const int nb = (L + TB - 1) / TB;
    d4v cre[2][2], cim[2][2], c2[2][2];
#pragma unroll
    for (int u = 0; u < 2; ++u)
#pragma unroll
        for (int v = 0; v < 2; ++v) {
            cre[u][v] = d4v{0.0, 0.0, 0.0, 0.0};
            cim[u][v] = d4v{0.0, 0.0, 0.0, 0.0};
            csub_init<G3>(cre[u][v], cim[u][v], c2[u][v]);
        }
    for (int K = ti; K < nb; ++K) {
        const int k0 = K * TB;
        for (int kc = 0; kc < TB && k0 + kc < L; kc += KS) {
            __syncthreads();
#pragma unroll
            for (int h = 0; h < KS * TB / 256; ++h) {
                const int e = tid + 256 * h, k = e / TB, c = e - k * TB;
                const int row = k0 + kc + k;
                const int ci = i0 + c, cj = j0 + c;
                As[k][c] = (row < L && ci < act && row >= ci) ? G[(size_t)row * L + ci] : czero();
                Bs[k][c] = (row < L && cj < act && row >= cj) ? G[(size_t)row * L + cj] : czero();
            }
            __syncthreads();
#pragma unroll
            for (int s = 0; s < KS / 4; ++s) {
                cd av[2], bv[2];
#pragma unroll
                for (int u = 0; u < 2; ++u) av[u] = As[4 * s + lk][wr + 16 * u + li];
#pragma unroll
                for (int v = 0; v < 2; ++v) bv[v] = Bs[4 * s + lk][wc + 16 * v + li];
                // C += conj(A) B  =  C - v conj(t)  with v = -conj(A), t = conj(B)
#pragma unroll
                for (int u = 0; u < 2; ++u) {
                    const cd va = cmk(-av[u].x, av[u].y);
#pragma unroll
                    for (int v = 0; v < 2; ++v)
                        csub_step<G3>(cre[u][v], cim[u][v], c2[u][v], va, cmk(bv[v].x, -bv[v].y));
                }
            }
        }
    }
#pragma unroll
    for (int u = 0; u < 2; ++u)
#pragma unroll
        for (int v = 0; v < 2; ++v)
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                const int r = i0 + wr + 16 * u + lk + 4 * q, c = j0 + wc + 16 * v + li;
                if (r < act && c < act) {
                    cd val = csub_out<G3>(cre[u][v], cim[u][v], c2[u][v], q);
                    // a dropped column of G is exactly zero: an uncoupled unit direction of C
                    if (r == c && val.x == 0.0) val = cmk(1.0, 0.0);
                    C[(size_t)r * L + c] = val;
                }
            }
}

// tol2[b] = 1e-14 max diag(C) over the active extent (C's own clamp threshold: C is HPD)
__global__ __launch_bounds__(256) void gram_tol_kernel(MstepArgs a, int L) {
    const int b = blockIdx.x;
    if (a.done && a.done[b]) return;
    __shared__ double red[4];
    const cd* C = a.gram + (size_t)b * L * L;
    const int act = a.act[b];
    double m = 0.0;
    for (int i = threadIdx.x; i < act; i += 256) m = fmax(m, C[(size_t)i * L + i].x);
    m = block_max(m, red);
    if (threadIdx.x == 0) a.tol2[b] = 1e-14 * m;
}

// ---------------------------------------------------------------- c = G^H b
// Block (column block J, trial): thread (column c, row phase q) sums conj(G[i][c]) b[i] over
// rows i = J*64 + q (mod 4) (each row read by 64 lanes: one coalesced 1 KB segment); the four
// phases are combined in a fixed order.  Rows past the active extent are written as 0.
// b = bin ([B][L][NR]), or conj(bin) with cin (the refinement's G^H x0, x0 = conj(theta)).
__global__ __launch_bounds__(256) void ghb_kernel(MstepArgs a, int L, int NR, const cd* bin, int cin) {
    const int J = blockIdx.x, b = blockIdx.y;
    if (a.done && a.done[b]) return;
    __shared__ cd part[4][TB][8];
    const cd* G = a.R + (size_t)b * L * L;
    const cd* bv = bin + (size_t)b * L * NR;
    cd* out = a.grhs + (size_t)b * L * NR;
    const int tid = threadIdx.x, c = tid & 63, q = tid >> 6;
    const int col = J * TB + c;
    const int act = a.act[b];
    cd acc[8];
#pragma unroll
    for (int r = 0; r < 8; ++r) acc[r] = czero();
    if (J * TB < act) {
        for (int i = J * TB + q; i < L; i += 4) {
            const cd g = (col < act && i >= col) ? G[(size_t)i * L + col] : czero();
#pragma unroll
            for (int r = 0; r < 8; ++r)
                if (r < NR) {
                    const cd v = bv[(size_t)i * NR + r];
                    acc[r] = cfmac(acc[r], cin ? cconj(v) : v, g);
                }
        }
    }
#pragma unroll
    for (int r = 0; r < 8; ++r) part[q][c][r] = acc[r];
    __syncthreads();
    if (q == 0 && col < L) {
        for (int r = 0; r < NR; ++r)
            out[(size_t)col * NR + r] = cadd(cadd(part[0][c][r], part[1][c][r]),
                                             cadd(part[2][c][r], part[3][c][r]));
    }
}

// ---------------------------------------------------------------- forward solve F y = c
// (the second application of F^-1; the first is fused into C's factorisation)
// fwddiag_kernel: y_k <- F_kk^-1 y_k by 16-row blocks through the inverses kept in the
// factor's strict upper 16 x 16 blocks (Di[c][c] = 1 / F[c][c], Di[c1][c2] = conj(F[c2][c1])),
// y_k already holding y_k - sum_{j < k} F_kj y_j.
__global__ __launch_bounds__(256) void fwddiag_kernel(MstepArgs a, int L, int NR, int k0, int w,
                                                      const int32_t* ext) {
    const int b = blockIdx.x;
    if (a.done && a.done[b]) return;
    if (ext && k0 >= ext[b]) return;
    __shared__ cd z[16][8];
    __shared__ cd Dl[16][17];
    const cd* F = a.R + (size_t)b * L * L;
    cd* y = a.rhs + (size_t)b * L * NR;
    const int tid = threadIdx.x, rr = tid >> 4, kl = tid & 15;
    for (int c0 = k0; c0 < k0 + w; c0 += 16) {
        const int wb = (k0 + w - c0) < 16 ? (k0 + w - c0) : 16;
        const int c = rr;                                   // row of this 16-block
        cd acc[8];
#pragma unroll
        for (int r = 0; r < 8; ++r) acc[r] = czero();
        if (c < wb) {
            for (int m = k0 + kl; m < c0; m += 16) {
                const cd l = F[(size_t)(c0 + c) * L + m];
#pragma unroll
                for (int r = 0; r < 8; ++r)
                    if (r < NR) acc[r] = cfma(acc[r], l, y[(size_t)m * NR + r]);
            }
        }
#pragma unroll
        for (int r = 0; r < 8; ++r)
            for (int off = 8; off >= 1; off >>= 1) {
                acc[r].x += __shfl_xor(acc[r].x, off);
                acc[r].y += __shfl_xor(acc[r].y, off);
            }
        {
            const int c1 = tid >> 4, c2 = tid & 15;
            cd v = czero();
            if (c1 < wb && c2 < wb) {
                if (c2 == c1) {
                    const double d = F[(size_t)(c0 + c1) * L + c0 + c1].x;
                    v = cmk(d > 0.0 ? 1.0 / d : 0.0, 0.0);
                } else if (c2 < c1) {
                    v = cconj(F[(size_t)(c0 + c2) * L + c0 + c1]);
                }
            }
            Dl[c1][c2] = v;                                 // Di[c1][c2]
        }
        if (kl == 0 && c < wb) {
#pragma unroll
            for (int r = 0; r < 8; ++r)
                if (r < NR) z[c][r] = csub(y[(size_t)(c0 + c) * NR + r], acc[r]);
        }
        __syncthreads();
        if (tid < wb * NR) {
            const int c1 = tid / NR, r = tid - c1 * NR;
            cd s = czero();                                 // y[c1] = sum_{c2 <= c1} Di[c1][c2] z[c2]
            for (int c2 = 0; c2 <= c1; ++c2) s = cfma(s, Dl[c1][c2], z[c2][r]);
            y[(size_t)(c0 + c1) * NR + r] = s;
        }
        __syncthreads();
    }
}

// Block (row block i > k, trial): y_i -= F_ik y_k, the tile and y_k staged in LDS.
__global__ __launch_bounds__(256) void fwdupd_kernel(MstepArgs a, int L, int NR, int k0, int w,
                                                     const int32_t* ext) {
    const int b = blockIdx.y;
    if (a.done && a.done[b]) return;
    const int i0 = k0 + TB * (1 + blockIdx.x);
    if (ext && (k0 >= ext[b] || i0 >= ext[b])) return;
    extern __shared__ __attribute__((aligned(16))) char smem[];
    cd(*T)[TB + 1] = reinterpret_cast<cd(*)[TB + 1]>(smem);  // T[r][m] = F[i0+r][k0+m]
    cd* xs = reinterpret_cast<cd*>(smem + (size_t)TB * (TB + 1) * sizeof(cd));
    const cd* F = a.R + (size_t)b * L * L;
    cd* y = a.rhs + (size_t)b * L * NR;
    const int tid = threadIdx.x;
    const int h = (L - i0) < TB ? (L - i0) : TB;
    for (int e = tid; e < h * TB; e += 256) {
        const int r = e / TB, m = e - r * TB;
        T[r][m] = m < w ? F[(size_t)(i0 + r) * L + k0 + m] : czero();
    }
    for (int e = tid; e < w * NR; e += 256) xs[e] = y[(size_t)k0 * NR + e];
    __syncthreads();
    for (int e = tid; e < h * NR; e += 256) {
        const int r = e / NR, c = e - r * NR;
        cd acc = czero();
        for (int m = 0; m < w; ++m) acc = cfma(acc, T[r][m], xs[m * NR + c]);
        y[(size_t)(i0 + r) * NR + c] = csub(y[(size_t)(i0 + r) * NR + c], acc);
    }
}

// ---------------------------------------------------------------- x = G z, theta = conj(x)
// Block (row block I, trial): tiles G_IJ (J <= I, columns below the active extent) staged in
// LDS by coalesced row segments, z_J beside them; thread per (row, right-hand side).
// mode 0: out = conj(G z) (theta);  1: out = bref - G z (the refinement residual);
// 2: out += conj(G z) (theta_1 = conj(x0 + dx)).
__global__ __launch_bounds__(256) void gz_kernel(MstepArgs a, int L, int NR, int mode, cd* out,
                                                 const cd* bref) {
    const int I = blockIdx.x, b = blockIdx.y;
    if (a.done && a.done[b]) return;
    extern __shared__ __attribute__((aligned(16))) char smem[];
    cd(*T)[TB + 1] = reinterpret_cast<cd(*)[TB + 1]>(smem);
    cd* zs = reinterpret_cast<cd*>(smem + (size_t)TB * (TB + 1) * sizeof(cd));
    const cd* G = a.R + (size_t)b * L * L;
    const cd* z = a.grhs + (size_t)b * L * NR;
    cd* th = out + (size_t)b * L * NR;
    const int act = a.act[b];
    const int tid = threadIdx.x, i0 = I * TB;
    const int h = (L - i0) < TB ? (L - i0) : TB;
    cd acc[2] = {czero(), czero()};                 // (row, rhs) pairs e = tid, tid + 256
    for (int J = 0; J <= I && J * TB < act; ++J) {
        const int j0 = J * TB;
        __syncthreads();
        for (int e = tid; e < h * TB; e += 256) {
            const int r = e / TB, m = e - r * TB;
            const int c = j0 + m;
            T[r][m] = (c < act && c <= i0 + r) ? G[(size_t)(i0 + r) * L + c] : czero();
        }
        for (int e = tid; e < TB * NR; e += 256) {
            const int m = e / NR;
            zs[e] = (j0 + m < act) ? z[(size_t)j0 * NR + e] : czero();
        }
        __syncthreads();
#pragma unroll
        for (int u = 0; u < 2; ++u) {
            const int e = tid + 256 * u;
            if (e < h * NR) {
                const int r = e / NR, c = e - r * NR;
                for (int m = 0; m < TB; ++m) acc[u] = cfma(acc[u], T[r][m], zs[m * NR + c]);
            }
        }
    }
#pragma unroll
    for (int u = 0; u < 2; ++u) {
        const int e = tid + 256 * u;
        if (e < h * NR) {
            const size_t o = (size_t)i0 * NR + e;
            if (mode == 0) th[o] = cconj(acc[u]);
            else if (mode == 1) th[o] = csub(bref[(size_t)b * L * NR + o], acc[u]);
            else th[o] = cadd(th[o], cconj(acc[u]));
        }
    }
}

// Refinement gate: C = F F^H's conditioning from F's diagonal over the kept columns of G.  The
// first solve's relative error grows like eps cond(C) (times a modest factor: 6e-5 measured at
// cond 9e8, tools/rank_study.py); trials with max/min F_kk^2 below 1e4 are already at the
// rounding level and skip the refinement step (skip[b] = 1, also for trials already done).  The
// diagonal ratio only bounds cond(C) from below, so a trial flagged SBCE_STATUS_RANK (a clamped
// pivot of C, or a pivot of R near the cut, in this call) is refined whatever its ratio.
__global__ __launch_bounds__(256) void mn_gate_kernel(MstepArgs a, int L) {
    const int b = blockIdx.x;
    __shared__ double red[4];
    if (a.done && a.done[b]) {
        if (threadIdx.x == 0) a.mnskip[b] = 1;
        return;
    }
    const cd* F = a.gram + (size_t)b * L * L;
    const cd* G = a.R + (size_t)b * L * L;
    const int act = a.act[b];
    double mx = 0.0, mn = INFINITY;
    for (int i = threadIdx.x; i < act; i += 256) {
        if (G[(size_t)i * L + i].x == 0.0) continue;       // a dropped column: C's unit placeholder
        const double d = F[(size_t)i * L + i].x;
        const double p = d * d;
        mx = fmax(mx, p);
        mn = fmin(mn, p);
    }
    mx = block_max(mx, red);
    __syncthreads();
    mn = -block_max(-mn, red);
    const bool flagged = a.status && (a.status[b] & SBCE_STATUS_RANK);
    if (threadIdx.x == 0) a.mnskip[b] = (act == 0 || (!flagged && mn * 1e4 >= mx)) ? 1 : 0;
}

// DIAGNOSTIC (bench.py's executed-flop count): per trial the active extent act[b] the rank-cut
// factorisation reached, the kept pivots of G (rank) and whether the refinement step ran.
__global__ __launch_bounds__(256) void mn_rank_kernel(MstepArgs a, int L, int32_t* out) {
    const int b = blockIdx.x;
    __shared__ int cnt[4];
    const cd* G = a.R + (size_t)b * L * L;
    const int act = a.act[b];
    int n = 0;
    for (int i = threadIdx.x; i < act; i += 256) n += G[(size_t)i * L + i].x != 0.0 ? 1 : 0;
    for (int off = 32; off >= 1; off >>= 1) n += __shfl_xor(n, off);
    if ((threadIdx.x & 63) == 0) cnt[threadIdx.x >> 6] = n;
    __syncthreads();
    if (threadIdx.x == 0) {
        out[3 * b] = act;
        out[3 * b + 1] = cnt[0] + cnt[1] + cnt[2] + cnt[3];
        out[3 * b + 2] = a.mnskip[b] ? 0 : 1;
    }
}

hipError_t launch_act(const Problem& pb, const MstepArgs& a, int k0, hipStream_t s) {
    hipLaunchKernelGGL(act_kernel, dim3(pb.B), dim3(256), 0, s, a, pb.L, k0);
    return hipGetLastError();
}

}  // namespace

hipError_t launch_minnorm_rank(const Problem& pb, const MstepArgs& a, int32_t* out, hipStream_t s) {
    if (!a.act || !a.mnskip) return hipErrorInvalidValue;
    hipLaunchKernelGGL(mn_rank_kernel, dim3(pb.B), dim3(256), 0, s, a, pb.L, out);
    return hipGetLastError();
}

hipError_t launch_minnorm(const Problem& pb, const MstepArgs& a, hipStream_t s) {
    if (pb.NR > 8 || !a.gram || !a.grhs || !a.act || !a.tol2 || !a.winv || !a.tol || !a.dvec ||
        !a.mnr || !a.mnskip)
        return hipErrorInvalidValue;
    const int L = pb.L, nb = (L + TB - 1) / TB;
    hipError_t e;
    if ((e = hipMemsetD32Async((hipDeviceptr_t)a.act, L, (size_t)pb.B, s)) != hipSuccess) return e;
    // rank cut from lambda_max(R)
    const size_t vbytes = (size_t)L * sizeof(cd);
    const size_t fixed = (size_t)kLzWaves * 64 * sizeof(cd) + kLzWaves * sizeof(double);
    if (2 * vbytes + fixed <= 160 * 1024)
        hipLaunchKernelGGL(lanczos_tol_kernel<true>, dim3(pb.B), dim3(64 * kLzWaves), 2 * vbytes, s, a,
                           L, pb.K);
    else
        hipLaunchKernelGGL(lanczos_tol_kernel<false>, dim3(pb.B), dim3(64 * kLzWaves), vbytes, s, a,
                           L, pb.K);
    if ((e = hipGetLastError()) != hipSuccess) return e;
    // R = G G^H, pivots at or below the cut dropped; B^H left untouched
    const TileExt exR{a.act, nullptr, 0};
    if ((e = launch_tile_factor(pb, a, exR, launch_act, s)) != hipSuccess) return e;
    // C = G^H G, c = G^H B^H
    {
        const int ntiles = nb * (nb + 1) / 2;
        const long nblk = (long)ntiles * ((pb.B + 7) / 8 * 8);
        // three-MFMA products here too: C = G^H G is formed after the rank cut, so its rounding
        // reaches theta (within lstsq's own) but no pivot decision
        if (g_debug.cplx3)
            hipLaunchKernelGGL(gram_kernel<true>, dim3((unsigned)nblk), dim3(256), 0, s, a, L, ntiles);
        else
            hipLaunchKernelGGL(gram_kernel<false>, dim3((unsigned)nblk), dim3(256), 0, s, a, L, ntiles);
    }
    hipLaunchKernelGGL(ghb_kernel, dim3(nb, pb.B), dim3(256), 0, s, a, L, pb.NR, (const cd*)a.rhs, 0);
    hipLaunchKernelGGL(gram_tol_kernel, dim3(pb.B), dim3(256), 0, s, a, L);
    if ((e = hipGetLastError()) != hipSuccess) return e;
    // z = C^-2 c:  C = F F^H with the fused F^-1, then F^-H, F^-1, F^-H
    MstepArgs c = a;
    c.R = a.gram; c.rhs = a.grhs; c.theta = nullptr; c.tol = a.tol2;
    c.clamp_status = SBCE_STATUS_RANK;     // a clamped pivot of C: flagged, the refinement below runs
    c.solve_mode = kSolveClampHpd;        // C is HPD: its rare tiny pivot is clamped, not dropped
    const TileExt exC{a.act, a.act, 1};
    if ((e = launch_tile_factor(pb, c, exC, nullptr, s)) != hipSuccess) return e;
    if ((e = launch_tile_back(pb, c, a.act, s)) != hipSuccess) return e;
    const size_t upd_lds = (size_t)TB * (TB + 1) * sizeof(cd) + (size_t)TB * 8 * sizeof(cd);
    // forward solve F y = c on grhs (the factorisation fused the first one)
    auto forward = [&](const MstepArgs& cc) -> hipError_t {
        for (int k = 0; k < nb; ++k) {
            const int k0 = k * TB, w = (L - k0) < TB ? (L - k0) : TB;
            hipLaunchKernelGGL(fwddiag_kernel, dim3(pb.B), dim3(256), 0, s, cc, L, pb.NR, k0, w, a.act);
            if (nb - k - 1 > 0)
                hipLaunchKernelGGL(fwdupd_kernel, dim3(nb - k - 1, pb.B), dim3(256), upd_lds, s, cc, L,
                                   pb.NR, k0, w, a.act);
            hipError_t e2 = hipGetLastError();
            if (e2 != hipSuccess) return e2;
        }
        return hipSuccess;
    };
    if ((e = forward(c)) != hipSuccess) return e;
    if ((e = launch_tile_back(pb, c, a.act, s)) != hipSuccess) return e;
    // theta = conj(G z)
    hipLaunchKernelGGL(gz_kernel, dim3(nb, pb.B), dim3(256), upd_lds, s, a, L, pb.NR, 0, a.theta,
                       (const cd*)nullptr);
    if ((e = hipGetLastError()) != hipSuccess) return e;
    // One refinement step on the kept subspace, for the trials whose C is ill-conditioned:
    //   x1 = x0 + G C^-2 G^H (b - G G^H x0).
    // G G^H is R up to the dropped Schur complement (below the cut), and the residual is formed
    // from G, not from C, so it is accurate to rounding; the step removes the first solve's error
    // (which the squared conditioning of C^-2 amplifies) to second order.  Its fixed point is the
    // minimum-norm solution of G G^H x = b on range(G) -- the same system, not a new answer.
    hipLaunchKernelGGL(mn_gate_kernel, dim3(pb.B), dim3(256), 0, s, a, L);
    MstepArgs r = a;                      // the refinement's launches skip the gated trials
    r.done = a.mnskip;
    MstepArgs cr = c;
    cr.done = a.mnskip;
    hipLaunchKernelGGL(ghb_kernel, dim3(nb, pb.B), dim3(256), 0, s, r, L, pb.NR, (const cd*)a.theta, 1);
    hipLaunchKernelGGL(gz_kernel, dim3(nb, pb.B), dim3(256), upd_lds, s, r, L, pb.NR, 1, a.mnr,
                       (const cd*)a.rhs);
    hipLaunchKernelGGL(ghb_kernel, dim3(nb, pb.B), dim3(256), 0, s, r, L, pb.NR, (const cd*)a.mnr, 0);
    if ((e = hipGetLastError()) != hipSuccess) return e;
    if ((e = forward(cr)) != hipSuccess) return e;
    if ((e = launch_tile_back(pb, cr, a.act, s)) != hipSuccess) return e;
    if ((e = forward(cr)) != hipSuccess) return e;
    if ((e = launch_tile_back(pb, cr, a.act, s)) != hipSuccess) return e;
    hipLaunchKernelGGL(gz_kernel, dim3(nb, pb.B), dim3(256), upd_lds, s, r, L, pb.NR, 2, a.theta,
                       (const cd*)nullptr);
    return hipGetLastError();
}

}  // namespace sbce
