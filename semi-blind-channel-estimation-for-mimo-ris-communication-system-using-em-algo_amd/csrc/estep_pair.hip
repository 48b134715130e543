// Exact soft E-step by factorised weights, for the cfg-1 geometry (n_tx = 4, 16-QAM) symbols
// the sphere pass leaves to the tile sweep because their posterior is wide (low SNR, early EM
// iterations).  Same posterior as estep.hip:
// "Proposed method/Proposed_method_NMSEvsTp.py":61-71, beta = exp(-||y - Z theta||^2/varn^2)/sum.
//
// The log-weight of hypothesis x = (x0, x1, x2, x3) with H_eff = [h_0 .. h_3],
//   l(x) = -||y - sum_a h_a x_a||^2 / s2,   s2 = varn^2,
// is a sum of terms over at most two streams:
//   l = A(x0,x1) + B(x2,x3) + E02(x0,x2) + E03(x0,x3) + E12(x1,x2) + E13(x1,x3),
//   A = -||y - h_0 x0 - h_1 x1||^2 / s2,   B = (||y||^2 - ||y - h_2 x2 - h_3 x3||^2) / s2,
//   Eab = -2 Re(conj(x_a) (h_a^H h_b) x_b) / s2,
// so w(x) = exp(l) is a product of six 16 x 16 tables, each exponentiated after subtracting its
// maximum (every factor in (0, 1]).  For each x2 the sums over x1
//   V_phi(x0, x3) = sum_x1 [A(x0,x1) E12(x1,x2)] [E13(x1,x3) phi(x1)],  phi = 1, Re x1, Im x1, |x1|^2
// are four 16 x 16 x 16 real GEMMs (16 v_mfma_f64_16x16x4f64), and the remaining factor
// f = E02(x0,x2) E03(x0,x3) B(x2,x3) with the x0 / x2 / x3 weights is applied per lane.  Every
// moment E[x_a], E[x_a conj(x_b)] follows: 256 MFMAs and ~1.5k VALU ops per lane per symbol
// instead of 65,536 distances and exponentials (the sweep's cost where nothing can be pruned).
//
// Range: with every factor <= 1 the largest weight is >= exp(-D), D = (sum of the six table
// maxima) - l(x_c), x_c the prep pass's candidate (a real hypothesis, l(x_c) <= max l).  For
// D <= kPairDmax every weight within e^-50 of the maximum is a normal double (> e^-700) and no
// partial product overflows: the symbol is resolved here.  Otherwise (D grows like 1/varn^2:
// high SNR) the sweep weighs it.  The enumeration routes a symbol here only when the tree pass's
// upper bound of D (estep.hip pair_screen, tree record word 31) is within the limit, so the exact
// test below is a safety net (a failing symbol would join the sweep's list).
#include "sbce_internal.h"

namespace sbce {

__device__ unsigned long long g_estep_pair;

namespace {

constexpr int kPairWaves = 4;
typedef double d4v __attribute__((ext_vector_type(4)));

struct PairConst {
    int B, Td, stride;     // prep record doubles per symbol
    double inv_s2;
    double thr_d;          // NT = 2 soft2 symbols: weights below e^-50 of the best are skipped
    int count;             // SBCE_ESTEP_COUNT=1: count the resolved symbols
};

__device__ __forceinline__ double wave_max(double v) {
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1) v = fmax(v, shfl_xor_d(v, off));
    return v;
}

template <int NR>
__global__ __launch_bounds__(64 * kPairWaves) __attribute__((amdgpu_waves_per_eu(3))) void estep_pair_kernel(EstepArgs a, PairConst c) {
    constexpr int NT = 4, M = 16, NO = NT * NR;
    __shared__ cd s_cons[M];
    __shared__ double s_tab[kPairWaves][6][256];     // E12, E02, B (the sweep's), A, E13, E03
    __shared__ cd s_hy[kPairWaves][NO + NR];         // H_eff (stream-major), y
    __shared__ double s_red[kPairWaves][32];
    __shared__ int32_t s_fail[kPairWaves][64];
    if (threadIdx.x < M) s_cons[threadIdx.x] = a.cons[threadIdx.x];
    __syncthreads();
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int lane = threadIdx.x & 63;
    const long nsym = (long)c.B * c.Td;
    int32_t* cnt = a.list + nsym;                    // [0] the sweep's list, [3] this pass's
    const int32_t* plist = a.list + 2 * nsym + 2 * kEstepListCnt;
    const int nwork = __builtin_amdgcn_readfirstlane(cnt[3]);
    double* E12 = s_tab[wave][0];
    double* E02 = s_tab[wave][1];
    double* TB = s_tab[wave][2];
    double* TA = s_tab[wave][3];
    double* T13 = s_tab[wave][4];
    double* T03 = s_tab[wave][5];
    cd* hy = s_hy[wave];
    const cd* H = hy;
    const cd* y = hy + NO;
    // symbol k of the list: the wave's first by its global index (no atomic: waves past the
    // list exit at once), the rest by grabbing from a counter that starts past the first round
    const int nwaves = gridDim.x * kPairWaves;
    int gi = blockIdx.x * kPairWaves + wave;
    // listed symbols this pass leaves to the sweep, staged per wave and appended in bulk
    int32_t* s_f = s_fail[wave];
    int nf = 0;
    auto flush = [&]() {
        if (nf == 0) return;
        int base = 0;
        if (lane == 0) base = atomicAdd(cnt, nf);
        base = __shfl(base, 0);
        if (lane < nf) a.list[base + lane] = s_f[lane];
        nf = 0;
        wave_sync();
    };
    for (;; gi = nwaves + __builtin_amdgcn_readfirstlane(__shfl(lane == 0 ? atomicAdd(cnt + 4, 1) : 0, 0))) {
        if (gi >= nwork) break;
        // lane-derived values (LDS addresses, constellation points) recomputed per symbol
        // instead of being hoisted and held across the symbol loop
        int ln = lane;
        asm volatile("" : "+v"(ln));
        const int cl = ln & 15, g = ln >> 4;
        const long gsym = plist[gi];
        const int b = (int)(gsym / c.Td);
        if (a.done && a.done[b]) continue;
        const double* rec = a.prep + (size_t)gsym * c.stride;
        wave_sync();                                    // the previous symbol's LDS reads are done
        if (lane < NO) hy[lane] = cmk(rec[4 + 2 * lane], rec[5 + 2 * lane]);
        else if (lane < NO + NR) hy[lane] = a.yd[(size_t)gsym * NR + lane - NO];
        const double d0 = rec[0];
        wave_sync();

        // ---- the six log tables, one at a time through LDS (few live registers): raw log
        //      values, their maxima, then the exponentials (A, E13, E03 into the registers of
        //      the MFMA operands / accumulator rows, B, E12, E02 back into LDS) ----
        const double is2 = a.varn_t ? uniform_d(trial_noise(a.varn_t[b]).inv_s2) : c.inv_s2;
        double yy = 0.0;
        cd G02 = czero(), G03 = czero(), G12 = czero(), G13 = czero();
#pragma unroll
        for (int r = 0; r < NR; ++r) {
            yy += cabs2(y[r]);
            G02 = cfmac(G02, H[2 * NR + r], H[0 * NR + r]);     // h_0^H h_2
            G03 = cfmac(G03, H[3 * NR + r], H[0 * NR + r]);
            G12 = cfmac(G12, H[2 * NR + r], H[1 * NR + r]);
            G13 = cfmac(G13, H[3 * NR + r], H[1 * NR + r]);
        }
        // every table is indexed [row rj = g + 4j][column cl] in LDS: A[x1][x0] (transposed,
        // the MFMA A operand wants x0 along the lanes), B[x2][x3], E13[x1][x3], E03[x0][x3],
        // E12[x1][x2], E02[x0][x2]
        const cd xc = s_cons[cl];
        double D = d0 * is2;                            // -l(x_c)
        double mA, mB, m13, m03, m12, m02;
        {
            double mxa = -INFINITY, mxb = -INFINITY;
#pragma unroll 1
            for (int j = 0; j < 4; ++j) {
                const int rj = g + 4 * j;
                const cd xr = s_cons[rj];
                double na = 0.0, nb = 0.0;
#pragma unroll
                for (int r = 0; r < NR; ++r) {
                    const cd ra = csub(csub(y[r], cmul(H[0 * NR + r], xc)), cmul(H[1 * NR + r], xr));
                    na += cabs2(ra);
                    const cd rb = csub(csub(y[r], cmul(H[2 * NR + r], xr)), cmul(H[3 * NR + r], xc));
                    nb += cabs2(rb);
                }
                const double la = -na * is2, lb = (yy - nb) * is2;   // A(x0 = cl, x1 = rj), B(rj, cl)
                TA[rj * 16 + cl] = la;
                TB[rj * 16 + cl] = lb;
                mxa = fmax(mxa, la);
                mxb = fmax(mxb, lb);
            }
            mA = wave_max(mxa);
            mB = wave_max(mxb);
        }
        {
            double m1 = -INFINITY, m2 = -INFINITY, m3 = -INFINITY, m4 = -INFINITY;
            const cd t13 = cmul(G13, xc), t03 = cmul(G03, xc), t12 = cmul(G12, xc), t02 = cmul(G02, xc);
#pragma unroll 1
            for (int j = 0; j < 4; ++j) {
                const int rj = g + 4 * j;
                const cd xr = s_cons[rj];
                // E(xa = xr, xb = xc) = -2 Re(conj(xr) G xc) / s2
                const double e13 = -2.0 * is2 * fma(xr.x, t13.x, xr.y * t13.y);
                const double e03 = -2.0 * is2 * fma(xr.x, t03.x, xr.y * t03.y);
                const double e12 = -2.0 * is2 * fma(xr.x, t12.x, xr.y * t12.y);
                const double e02 = -2.0 * is2 * fma(xr.x, t02.x, xr.y * t02.y);
                T13[rj * 16 + cl] = e13;
                T03[rj * 16 + cl] = e03;
                E12[rj * 16 + cl] = e12;
                E02[rj * 16 + cl] = e02;
                m1 = fmax(m1, e13);
                m2 = fmax(m2, e03);
                m3 = fmax(m3, e12);
                m4 = fmax(m4, e02);
            }
            m13 = wave_max(m1);
            m03 = wave_max(m2);
            m12 = wave_max(m3);
            m02 = wave_max(m4);
        }
        D += mA + mB + m13 + m03 + m12 + m02;
        if (!(D <= kPairDmax)) {                        // wave-uniform: to the sweep's list
            if (lane == 0) s_f[nf] = (int32_t)gsym;
            wave_sync();
            if (++nf == 64) flush();
            continue;
        }
        // exponentials in place, one entry of each table per step (the 24 exps of a lane do
        // not run side by side: their temporaries would not fit the register budget)
#pragma unroll 1
        for (int j = 0; j < 4; ++j) {
            const int e = (g + 4 * j) * 16 + cl;
            TA[e] = fexp_neg(TA[e] - mA);
            T13[e] = fexp_neg(T13[e] - m13);
            T03[e] = fexp_neg(T03[e] - m03);
            TB[e] = fexp_neg(TB[e] - mB);
            E12[e] = fexp_neg(E12[e] - m12);
            E02[e] = fexp_neg(E02[e] - m02);
        }
        wave_sync();
        double ar[4], e03[4], rr[4][4];
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const int e = (g + 4 * j) * 16 + cl;
            const cd x1 = s_cons[g + 4 * j];
            ar[j] = TA[e];
            const double e13 = T13[e];
            rr[0][j] = e13;
            rr[1][j] = e13 * x1.x;
            rr[2][j] = e13 * x1.y;
            rr[3][j] = e13 * cabs2(x1);
            e03[j] = T03[e];
        }

        // ---- sweep over x2: lane (cl, g) holds V_phi[x0 = g + 4q][x3 = cl] ----
        cd x0r[4];
        double x0s[4];
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            x0r[q] = s_cons[g + 4 * q];
            x0s[q] = cabs2(x0r[q]);
        }
        double Z = 0.0, s00 = 0.0, s11 = 0.0, s22 = 0.0;
        cd m0 = czero(), m1 = czero(), m2 = czero(), s01 = czero(), s02 = czero(), s12 = czero();
#pragma unroll 1
        for (int x2 = 0; x2 < 16; ++x2) {
            double ap[4];
#pragma unroll
            for (int s = 0; s < 4; ++s) ap[s] = ar[s] * E12[(4 * s + g) * 16 + x2];
            d4v V[4];
#pragma unroll
            for (int w = 0; w < 4; ++w) V[w] = d4v{0.0, 0.0, 0.0, 0.0};
#pragma unroll
            for (int s = 0; s < 4; ++s)
#pragma unroll
                for (int w = 0; w < 4; ++w)
                    V[w] = __builtin_amdgcn_mfma_f64_16x16x4f64(ap[s], rr[w][s], V[w], 0, 0, 0);
            const double bx = TB[x2 * 16 + cl];
            double ws = 0.0;
            cd mx0 = czero(), u = czero();
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                const double f = E02[(g + 4 * q) * 16 + x2] * (e03[q] * bx);
                const double W = f * V[0][q];
                const cd U = cmk(f * V[1][q], f * V[2][q]);   // sum_x1 w x1
                ws += W;
                mx0 = caxpy(mx0, W, x0r[q]);
                s00 = fma(W, x0s[q], s00);
                s11 = fma(f, V[3][q], s11);
                s01 = cfmac(s01, x0r[q], U);                 // x0 conj(x1)
                u = cadd(u, U);
            }
            const cd x2v = s_cons[x2];
            Z += ws;
            m2 = caxpy(m2, ws, x2v);
            s22 = fma(ws, cabs2(x2v), s22);
            m0 = cadd(m0, mx0);
            s02 = cfmac(s02, mx0, x2v);
            m1 = cadd(m1, u);
            s12 = cfmac(s12, u, x2v);
        }
        // x3 = s_cons[cl] is the lane's own: its moments from the lane's partial sums
        const cd x3v = s_cons[cl];
        const cd m3 = cscale(x3v, Z);
        const double s33 = Z * cabs2(x3v);
        const cd s03 = cmulc(m0, x3v), s13 = cmulc(m1, x3v), s23 = cmulc(m2, x3v);

        // ---- wave reduction (recursive halving, as the sweep's) and the outputs ----
        double vv[32];
        {
            int n = 0;
            auto put = [&](double x) { vv[n++] = x; };
            put(Z);
            put(m0.x); put(m0.y); put(m1.x); put(m1.y); put(m2.x); put(m2.y); put(m3.x); put(m3.y);
            put(s00); put(s11); put(s22); put(s33);
            put(s01.x); put(s01.y); put(s02.x); put(s02.y); put(s03.x); put(s03.y);
            put(s12.x); put(s12.y); put(s13.x); put(s13.y); put(s23.x); put(s23.y);
#pragma unroll
            for (int i = 25; i < 32; ++i) vv[i] = 0.0;
        }
        int xa[6];
#pragma unroll
        for (int i = 0; i < 6; ++i) xa[i] = (ln ^ (32 >> i)) << 2;
#pragma unroll
        for (int st = 0; st < 5; ++st) {
            const int h = 16 >> st;
            const bool hi = (ln >> (5 - st)) & 1;
#pragma unroll
            for (int i = 0; i < h; ++i) {
                const double snd = hi ? vv[i] : vv[h + i];
                const double kp = hi ? vv[h + i] : vv[i];
                vv[i] = kp + bperm_d(snd, xa[st]);
            }
        }
        vv[0] += bperm_d(vv[0], xa[5]);
        double* red = s_red[wave];
        const int jv = ((lane >> 5) & 1) * 16 + ((lane >> 4) & 1) * 8 + ((lane >> 3) & 1) * 4 +
                       ((lane >> 2) & 1) * 2 + ((lane >> 1) & 1);
        if (!(lane & 1)) red[jv] = vv[0];
        wave_sync();
        if (lane < NT + NT * NT) {
            // m_a at 1 + 2a; E|x_a|^2 at 9 + a; E[x_a conj(x_b)], a < b, at 13, 15, 17 (0,1..3),
            // 19, 21 (1,2..3), 23 (2,3)
            int ire, iim = -1;
            bool cj = false;
            if (lane < NT) {
                ire = 1 + 2 * lane;
                iim = ire + 1;
            } else {
                const int i = (lane - NT) >> 2, j = (lane - NT) & 3;
                if (i == j) {
                    ire = 9 + i;
                } else {
                    const int lo = i < j ? i : j, hi2 = i < j ? j : i;
                    const int pidx = lo == 0 ? hi2 - 1 : (lo == 1 ? 1 + hi2 : 5);   // 0..5
                    ire = 13 + 2 * pidx;
                    iim = ire + 1;
                    cj = i > j;
                }
            }
            const double iz = 1.0 / red[0];
            const double re = red[ire], im = iim >= 0 ? red[iim] : 0.0;
            a.mom[(size_t)gsym * (NT + NT * NT) + lane] = cmk(re * iz, (cj ? -im : im) * iz);
        }
        if (c.count && lane == 0) atomicAdd(&g_estep_pair, 1ull);
    }
    flush();
}


// ---------------------------------------------------------------- n_tx = 2, square M-QAM
// The same idea for two streams (BASELINE cfg 5: 2 x 2, 64-QAM, J = 4096 hypotheses).  With
// x_a = a_a + i b_a on a K x K level grid, z_a = h_a^H y, g_aa = ||h_a||^2, g = h_0^H h_1,
//   l(x) s2 + ||y||^2 = [2 a0 Re z0 - g00 a0^2] + [2 b0 Im z0 - g00 b0^2] + (same for x1)
//                     - 2 [a0 a1 Re g - a0 b1 Im g + b0 a1 Im g + b0 b1 Re g],
// four 1-D tables and four K x K tables, each exponentiated after subtracting its maximum.  The
// bilinear part couples {a0, b0} only with {a1, b1}, so for fixed (a0, b0) the sum over (a1, b1)
// is a PRODUCT of a sum over a1 and a sum over b1:
//   Z = sum_{a0,b0} F(a0) G(b0) U(a0,b0) V(a0,b0),  U = sum_a1 F1(a1) T1(a0,a1) T3(b0,a1),
//   V = sum_b1 G1(b1) T2(a0,b1) T4(b0,b1),
// and every moment E[x_a], E[x_a conj(x_b)] takes a1- / b1-weighted versions of U and V.  One
// WAVE per symbol, lane = (a0, b0): 288 exponentials and ~100 VALU ops per lane plus eleven wave
// sums instead of 4096 distances and exponentials.  Range as above: the largest weight is
// >= exp(-D), D = (sum of the eight table maxima) - l(x_c); the tree pass routes a symbol here
// only when its D (estep.hip fact2_bound) is within kPairDmax, and a symbol whose sum Z still
// leaves the normal range joins the sweep's list.
constexpr int kF2Waves = 4;

template <int NR>
__global__ __launch_bounds__(64 * kF2Waves) void estep_fact2_kernel(EstepArgs a, PairConst c, int M) {
    constexpr int NT = 2, MS = NT + NT * NT;
    __shared__ cd s_cons[64];
    __shared__ GridLds s_grid;
    __shared__ double s_tab[kF2Waves][4 * 8 + 4 * 64];   // F0 G0 F1 G1 [8], T1 T2 T3 T4 [8][8]
    __shared__ int32_t s_fail[kF2Waves][64];
    if ((int)threadIdx.x < M) s_cons[threadIdx.x] = a.cons[threadIdx.x];
    __syncthreads();
    grid_build(s_cons, M, &s_grid);
    const int K = s_grid.K;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int lane = threadIdx.x & 63;
    const long nsym = (long)c.B * c.Td;
    int32_t* cnt = a.list + nsym;                    // [0] the sweep's list, [3] this pass's
    const int32_t* plist = a.list + 2 * nsym + 2 * kEstepListCnt;
    const int nwork = __builtin_amdgcn_readfirstlane(cnt[3]);
    double* tab = s_tab[wave];
    double* F0 = tab;
    double* G0 = tab + 8;
    double* F1 = tab + 16;
    double* G1 = tab + 24;
    double* T1 = tab + 32;                           // [a0][a1]
    double* T2 = T1 + 64;                            // [a0][b1]
    double* T3 = T2 + 64;                            // [b0][a1]
    double* T4 = T3 + 64;                            // [b0][b1]
    const int nwaves = gridDim.x * kF2Waves;
    int gi = blockIdx.x * kF2Waves + wave;
    int32_t* s_f = s_fail[wave];
    int nf = 0;
    auto flush = [&]() {
        if (nf == 0) return;
        int base = 0;
        if (lane == 0) base = atomicAdd(cnt, nf);
        base = __shfl(base, 0);
        if (lane < nf) a.list[base + lane] = s_f[lane];
        nf = 0;
        wave_sync();
    };
    auto wmax = [](double v) { return wave_max_dpp(v); };
    auto wsum = [](double v) { return wave_sum_dpp(v); };
    // symbols by a static stride (every symbol costs the same: no work grabbing), the next one's
    // index, channel and observation loaded while the current one is computed
    auto fetch = [&](int k, long& gs, cd (&hh)[2 * NR], cd (&yy)[NR]) {
        gs = k < nwork ? (long)plist[k] : 0;
        if (k < nwork) {
            const long g0 = gs;
            const double* rec = a.prep + (size_t)g0 * c.stride;
#pragma unroll
            for (int e = 0; e < 2 * NR; ++e) hh[e] = cmk(rec[4 + 2 * e], rec[5 + 2 * e]);
#pragma unroll
            for (int r = 0; r < NR; ++r) yy[r] = a.yd[(size_t)g0 * NR + r];
        }
    };
    long gnext;
    cd hnext[2 * NR], ynext[NR];
    fetch(gi, gnext, hnext, ynext);
    for (; gi < nwork; gi += nwaves) {
        const long gsym = gnext;
        cd hc[2 * NR], yc[NR];
#pragma unroll
        for (int e = 0; e < 2 * NR; ++e) hc[e] = hnext[e];
#pragma unroll
        for (int r = 0; r < NR; ++r) yc[r] = ynext[r];
        fetch(gi + nwaves, gnext, hnext, ynext);
        const int b = (int)(gsym / c.Td);
        if (a.done && a.done[b]) continue;
        if (K == 0) {                                // not a square grid: the sweep weighs it
            if (lane == 0) s_f[nf] = (int32_t)gsym;
            ++nf;
            if (nf == 64) flush();
            continue;
        }
        const double is2 = a.varn_t ? uniform_d(trial_noise(a.varn_t[b]).inv_s2) : c.inv_s2;
        cd z0 = czero(), z1 = czero(), g = czero();
        double g00 = 0.0, g11 = 0.0;
#pragma unroll
        for (int r = 0; r < NR; ++r) {
            const cd h0 = hc[r], h1 = hc[NR + r], yr = yc[r];
            z0 = cfmac(z0, yr, h0);                  // h_0^H y
            z1 = cfmac(z1, yr, h1);
            g = cfmac(g, h1, h0);                    // h_0^H h_1
            g00 += cabs2(h0);
            g11 += cabs2(h1);
        }
        // ---- log tables (times s2), their maxima, the exponentials into LDS ----
        const int i = lane >> 3, j = lane & 7;       // lane = (row i, column j) of a K x K table
        const bool on1 = lane < 4 * K, on2 = i < K && j < K;
        double v1 = -INFINITY;                       // 1-D table entry: table lane / K, level lane % K
        const int t1 = on1 ? lane / K : 0, k1 = on1 ? lane - t1 * K : 0;
        if (on1) {
            const double lv = (t1 & 1) ? s_grid.lim[k1] : s_grid.lre[k1];
            const double zz = t1 == 0 ? z0.x : (t1 == 1 ? z0.y : (t1 == 2 ? z1.x : z1.y));
            const double gg = t1 < 2 ? g00 : g11;
            v1 = (2.0 * lv * zz - gg * lv * lv) * is2;
        }
        double w1 = -INFINITY, w2 = -INFINITY, w3 = -INFINITY, w4 = -INFINITY;
        if (on2) {
            const double ai = s_grid.lre[i], bi = s_grid.lim[i], aj = s_grid.lre[j], bj = s_grid.lim[j];
            w1 = -2.0 * g.x * ai * aj * is2;         // T1(a0 = a_i, a1 = a_j)
            w2 = 2.0 * g.y * ai * bj * is2;          // T2(a0 = a_i, b1 = b_j)
            w3 = -2.0 * g.y * bi * aj * is2;         // T3(b0 = b_i, a1 = a_j)
            w4 = -2.0 * g.x * bi * bj * is2;         // T4(b0 = b_i, b1 = b_j)
        }
        double m1[4];
#pragma unroll
        for (int t = 0; t < 4; ++t) m1[t] = wmax((on1 && t1 == t) ? v1 : -INFINITY);
        const double mT1 = wmax(w1), mT2 = wmax(w2), mT3 = wmax(w3), mT4 = wmax(w4);
        // D = (sum of the maxima) - l(x_c) with x_c the best hypothesis on the diagonal of the
        // lanes' own (a0, b0) x (a1 = a0, b1 = b0) grid is not needed: the tree pass bounded it;
        // the sum Z below is checked for the normal range instead
        wave_sync();                                 // the previous symbol's table reads are done
        if (on1) tab[8 * t1 + k1] = exp(v1 - m1[t1]);
        if (on2) {
            T1[i * 8 + j] = exp(w1 - mT1);
            T2[i * 8 + j] = exp(w2 - mT2);
            T3[i * 8 + j] = exp(w3 - mT3);
            T4[i * 8 + j] = exp(w4 - mT4);
        }
        wave_sync();
        // ---- lane (a0 = level i, b0 = level j): the a1 and b1 sums ----
        double P = 0.0, Pa1 = 0.0, Pb1 = 0.0, P11 = 0.0;
        double a0 = 0.0, b0 = 0.0;
        if (on2) {
            a0 = s_grid.lre[i];
            b0 = s_grid.lim[j];
            double U = 0.0, U1 = 0.0, U2 = 0.0, V = 0.0, V1 = 0.0, V2 = 0.0;
            for (int k = 0; k < K; ++k) {
                const double a1 = s_grid.lre[k], b1 = s_grid.lim[k];
                const double eu = F1[k] * T1[i * 8 + k] * T3[j * 8 + k];
                U += eu;
                U1 = fma(a1, eu, U1);
                U2 = fma(a1 * a1, eu, U2);
                const double ev = G1[k] * T2[i * 8 + k] * T4[j * 8 + k];
                V += ev;
                V1 = fma(b1, ev, V1);
                V2 = fma(b1 * b1, ev, V2);
            }
            const double w = F0[i] * G0[j];
            P = w * U * V;
            Pa1 = w * U1 * V;
            Pb1 = w * U * V1;
            P11 = w * fma(U2, V, U * V2);
        }
        const double Z = wsum(P);
        const double Sa0 = wsum(a0 * P), Sb0 = wsum(b0 * P), S00 = wsum(fma(a0, a0, b0 * b0) * P);
        const double Sa1 = wsum(Pa1), Sb1 = wsum(Pb1), S11 = wsum(P11);
        const double Sa0a1 = wsum(a0 * Pa1), Sb0b1 = wsum(b0 * Pb1);
        const double Sb0a1 = wsum(b0 * Pa1), Sa0b1 = wsum(a0 * Pb1);
        if (!(Z > 1e-250) || !(Z < 1e250)) {         // outside the represented range: to the sweep
            if (lane == 0) s_f[nf] = (int32_t)gsym;
            ++nf;
            if (nf == 64) flush();
            continue;
        }
        const double iz = 1.0 / Z;
        cd* out = a.mom + (size_t)gsym * MS;
        if (lane == 0) {
            out[0] = cmk(Sa0 * iz, Sb0 * iz);
            out[1] = cmk(Sa1 * iz, Sb1 * iz);
            out[2] = cmk(S00 * iz, 0.0);
            const cd s01 = cmk((Sa0a1 + Sb0b1) * iz, (Sb0a1 - Sa0b1) * iz);   // E[x0 conj(x1)]
            out[3] = s01;
            out[4] = cconj(s01);
            out[5] = cmk(S11 * iz, 0.0);
        }
        if (c.count && lane == 0) atomicAdd(&g_estep_pair, 1ull);
    }
    flush();
}


// Narrow posteriors of n_tx = 2 (the tree pass's narrow list: range D above the factorised
// tables' limit): lane = x_0, r = y - h_0 x_0; d(x_1) = g_11 |x_1 - z|^2 + (||r||^2 -
// g_11 |z|^2), z = h_1^H r / g_11, so the lane's best x_1 is the per-axis nearest level pair (taken
// when both per-axis rivals are farther by more than the distances' rounding, else every point is
// scanned), d_min the wave minimum, and the x_1 within thr = 50 varn^2 of d_min (the sweep's e^-50
// skip) lie in a box of half-width sqrt((d_min + thr - c_0) / g_11) around z; each is checked
// directly and weighted exp(-(d - d_min) / s2).
template <int NR>
__global__ __launch_bounds__(64 * kF2Waves) void estep_soft2_kernel(EstepArgs a, PairConst c, int M) {
    constexpr int MS = 6;
    __shared__ cd s_cons[64];
    __shared__ GridLds s_grid;
    __shared__ int32_t s_fail[kF2Waves][64];
    if ((int)threadIdx.x < M) s_cons[threadIdx.x] = a.cons[threadIdx.x];
    __syncthreads();
    grid_build(s_cons, M, &s_grid);
    const int K = s_grid.K;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int lane = threadIdx.x & 63;
    const long nsym = (long)c.B * c.Td;
    int32_t* cnt = a.list + nsym;
    // the tree pass's narrow symbols: the enumeration list's slots (counter 2, estep_tree_kernel)
    const int32_t* plist = cnt + kEstepListCnt;
    const int nwork = __builtin_amdgcn_readfirstlane(cnt[2]);
    const int nwaves = gridDim.x * kF2Waves;
    int32_t* s_f = s_fail[wave];
    int nf = 0;
    auto flush = [&]() {
        if (nf == 0) return;
        int base = 0;
        if (lane == 0) base = atomicAdd(cnt, nf);
        base = __shfl(base, 0);
        if (lane < nf) a.list[base + lane] = s_f[lane];
        nf = 0;
        wave_sync();
    };
    auto wmax = [](double v) { return wave_max_dpp(v); };
    auto wsum = [](double v) { return wave_sum_dpp(v); };
    double lre[8], lim[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) {
        lre[k] = k < K ? s_grid.lre[k] : INFINITY;
        lim[k] = k < K ? s_grid.lim[k] : INFINITY;
    }
    for (int gi = blockIdx.x * kF2Waves + wave; gi < nwork; gi += nwaves) {
        const long gsym = plist[gi];
        const int b = (int)(gsym / c.Td);
        if (a.done && a.done[b]) continue;
        if (K == 0) {                                // not a square grid: the sweep weighs it
            if (lane == 0) s_f[nf] = (int32_t)gsym;
            ++nf;
            if (nf == 64) flush();
            continue;
        }
        const double is2 = a.varn_t ? uniform_d(trial_noise(a.varn_t[b]).inv_s2) : c.inv_s2;
        const double* rec = a.prep + (size_t)gsym * c.stride;
        cd hc[2 * NR], yc[NR];
#pragma unroll
        for (int e = 0; e < 2 * NR; ++e) hc[e] = cmk(rec[4 + 2 * e], rec[5 + 2 * e]);
#pragma unroll
        for (int q = 0; q < NR; ++q) yc[q] = a.yd[(size_t)gsym * NR + q];
        // ---- narrow posterior: lane = x_0, the x_1 within e^-50 of the best hypothesis ----
        const double thr = a.varn_t ? uniform_d(trial_noise(a.varn_t[b]).thr_d) : c.thr_d;
        const bool on = lane < M;
        const cd x0 = s_cons[on ? lane : 0];
        cd r[NR], h1[NR];
        double g11 = 0.0, scale = 0.0;
#pragma unroll
        for (int q = 0; q < NR; ++q) {
            h1[q] = hc[NR + q];
            r[q] = csub(yc[q], cmul(hc[q], x0));
            g11 += cabs2(h1[q]);
            scale += cabs2(r[q]);
        }
        auto dist = [&](int s1) {
            const cd x1 = s_cons[s1];
            double d = 0.0;
#pragma unroll
            for (int q = 0; q < NR; ++q) d += cabs2(csub(r[q], cmul(h1[q], x1)));
            return d;
        };
        cd z = czero();
#pragma unroll
        for (int q = 0; q < NR; ++q) z = cfmac(z, r[q], h1[q]);    // h_1^H r
        const bool deg = !(g11 > 0.0);
        z = deg ? czero() : cscale(z, 1.0 / g11);
        // the lane's best x_1 (exact: every point when the per-axis candidate is not clear)
        double dbest = INFINITY;
        {
            double bx = INFINITY, bx2 = INFINITY, by = INFINITY, by2 = INFINITY;
            int ix = 0, ix2 = 0, iy = 0, iy2 = 0;
            double cm2 = 0.0;
#pragma unroll
            for (int k = 0; k < 8; ++k) {
                const double dx = fabs(z.x - lre[k]);
                if (dx < bx) { bx2 = bx; ix2 = ix; bx = dx; ix = k; }
                else if (dx < bx2) { bx2 = dx; ix2 = k; }
                const double dy = fabs(z.y - lim[k]);
                if (dy < by) { by2 = by; iy2 = iy; by = dy; iy = k; }
                else if (dy < by2) { by2 = dy; iy2 = k; }
                if (k < K) cm2 = fmax(cm2, fma(lre[k], lre[k], lim[k] * lim[k]));
            }
            const double mg = 64.0 * 2.2e-16 * (scale + 4.0 * g11 * cm2);
            const double v1 = dist(s_grid.idx[ix * K + iy]);
            const bool clear = !deg && K >= 2 && dist(s_grid.idx[ix2 * K + iy]) > v1 + mg &&
                               dist(s_grid.idx[ix * K + iy2]) > v1 + mg;
            if (clear) {
                dbest = v1;
            } else {
                for (int s1 = 0; s1 < M; ++s1) dbest = fmin(dbest, dist(s1));
            }
        }
        const double dmin = wmax(on ? -dbest : -INFINITY) * -1.0;
        // d(x_1) = g11 |x_1 - z|^2 + (||r||^2 - g11 |z|^2): the points within thr of dmin lie in
        // a box of half-width rho around z (widened for rounding); each is checked directly
        double Zl = 0.0, Q1 = 0.0;
        cd X1 = czero();
        if (on) {
            const double c0 = scale - g11 * cabs2(z);
            const double rho2 = deg ? INFINITY : (dmin + thr - c0) / g11;
            const double rho = rho2 > 0.0 ? sqrt(rho2) * (1.0 + 1e-7) + 1e-9 * sqrt(1.0 + cabs2(z)) : -1.0;
            for (int kx = 0; kx < K; ++kx) {
                if (!(fabs(lre[kx] - z.x) <= rho)) continue;
                for (int ky = 0; ky < K; ++ky) {
                    if (!(fabs(lim[ky] - z.y) <= rho)) continue;
                    const int s1 = s_grid.idx[kx * K + ky];
                    const double d = dist(s1);
                    if (d - dmin > thr) continue;
                    const double w = exp(-(d - dmin) * is2);
                    const cd x1 = s_cons[s1];
                    Zl += w;
                    X1 = caxpy(X1, w, x1);
                    Q1 = fma(w, cabs2(x1), Q1);
                }
            }
        }
        const double Z = wsum(Zl);
        const double m0r = wsum(Zl * x0.x), m0i = wsum(Zl * x0.y), S00 = wsum(Zl * cabs2(x0));
        const double m1r = wsum(X1.x), m1i = wsum(X1.y), S11 = wsum(Q1);
        const cd s01l = cmulc(x0, X1);                                 // x_0 conj(sum w x_1)
        const double s01r = wsum(s01l.x), s01i = wsum(s01l.y);
        if (!(Z > 0.0)) {                        // (cannot happen: the best hypothesis has w = 1)
            if (lane == 0) s_f[nf] = (int32_t)gsym;
            ++nf;
            if (nf == 64) flush();
            continue;
        }
        const double iz = 1.0 / Z;
        if (lane == 0) {
            cd* out = a.mom + (size_t)gsym * MS;
            out[0] = cmk(m0r * iz, m0i * iz);
            out[1] = cmk(m1r * iz, m1i * iz);
            out[2] = cmk(S00 * iz, 0.0);
            out[3] = cmk(s01r * iz, s01i * iz);
            out[4] = cmk(s01r * iz, -s01i * iz);
            out[5] = cmk(S11 * iz, 0.0);
        }
        if (c.count && lane == 0) atomicAdd(&g_estep_pair, 1ull);
    }
    flush();
}

// ---------------------------------------------------------------- n_tx = 2, hard decision
// The log-max E-step (argmin over the M^2 hypotheses of ||y - h_0 x_0 - h_1 x_1||^2, first table
// index on ties: ML_detecctor.py:65-75) for n_tx = 2 on a square M-QAM grid: lane = x_0 (its table
// index), r = y - h_0 x_0, and the best x_1 for that x_0 minimises g_11 |x_1 - z|^2 + const,
// z = h_1^H r / g_11 -- separable per axis.  The per-axis best and second-best levels give the
// candidate and its two rivals; their distances are computed the direct way, and the candidate is
// taken when both rivals are farther by more than the distances' rounding (else the lane scans all
// M points).  Then the wave's first minimum in table order (x_0 slow, x_1 fast).  The tree pass
// routes every symbol it does not resolve alone here (no range limit: no exponentials).
template <int NR>
__global__ __launch_bounds__(64 * kF2Waves) void estep_hard2_kernel(EstepArgs a, PairConst c, int M) {
    constexpr int MS = 6;
    __shared__ cd s_cons[64];
    __shared__ GridLds s_grid;
    if ((int)threadIdx.x < M) s_cons[threadIdx.x] = a.cons[threadIdx.x];
    __syncthreads();
    grid_build(s_cons, M, &s_grid);
    const int K = s_grid.K;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int lane = threadIdx.x & 63;
    const long nsym = (long)c.B * c.Td;
    const int32_t* cnt = a.list + nsym;
    const int32_t* plist = a.list + 2 * nsym + 2 * kEstepListCnt;
    const int nwork = __builtin_amdgcn_readfirstlane(cnt[3]);
    const int nwaves = gridDim.x * kF2Waves;
    double lre[8], lim[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) {
        lre[k] = k < K ? s_grid.lre[k] : INFINITY;
        lim[k] = k < K ? s_grid.lim[k] : INFINITY;
    }
    for (int gi = blockIdx.x * kF2Waves + wave; gi < nwork; gi += nwaves) {
        const long gsym = plist[gi];
        const int b = (int)(gsym / c.Td);
        if (a.done && a.done[b]) continue;
        const double* rec = a.prep + (size_t)gsym * c.stride;
        cd h0[NR], h1[NR], r[NR];
        double g11 = 0.0, scale = 0.0;
        const bool on = lane < M;
        const cd x0 = s_cons[on ? lane : 0];
#pragma unroll
        for (int q = 0; q < NR; ++q) {
            h0[q] = cmk(rec[4 + 2 * q], rec[5 + 2 * q]);
            h1[q] = cmk(rec[4 + 2 * (NR + q)], rec[5 + 2 * (NR + q)]);
            r[q] = csub(a.yd[(size_t)gsym * NR + q], cmul(h0[q], x0));
            g11 += cabs2(h1[q]);
            scale += cabs2(r[q]);
        }
        auto dist = [&](int s1) {
            const cd x1 = s_cons[s1];
            double d = 0.0;
#pragma unroll
            for (int q = 0; q < NR; ++q) d += cabs2(csub(r[q], cmul(h1[q], x1)));
            return d;
        };
        int best = 0;
        double dbest = INFINITY;
        bool scan = K == 0 || !(g11 > 0.0);
        if (!scan) {
            cd z = czero();
#pragma unroll
            for (int q = 0; q < NR; ++q) z = cfmac(z, r[q], h1[q]);     // h_1^H r
            z = cscale(z, 1.0 / g11);
            double bx = INFINITY, bx2 = INFINITY, by = INFINITY, by2 = INFINITY;
            int ix = 0, ix2 = 0, iy = 0, iy2 = 0;
#pragma unroll
            for (int k = 0; k < 8; ++k) {
                const double dx = fabs(z.x - lre[k]);
                if (dx < bx) { bx2 = bx; ix2 = ix; bx = dx; ix = k; }
                else if (dx < bx2) { bx2 = dx; ix2 = k; }
                const double dy = fabs(z.y - lim[k]);
                if (dy < by) { by2 = by; iy2 = iy; by = dy; iy = k; }
                else if (dy < by2) { by2 = dy; iy2 = k; }
            }
            const int s1 = s_grid.idx[ix * K + iy];
            const double v1 = dist(s1);
            // rounding of a distance: a few ulps of the terms it sums
            double cm2 = 0.0;
#pragma unroll
            for (int k = 0; k < 8; ++k)
                if (k < K) cm2 = fmax(cm2, fma(lre[k], lre[k], lim[k] * lim[k]));
            const double mg = 64.0 * 2.2e-16 * (scale + 4.0 * g11 * cm2);
            const bool ra = K < 2 || dist(s_grid.idx[ix2 * K + iy]) > v1 + mg;
            const bool rb = K < 2 || dist(s_grid.idx[ix * K + iy2]) > v1 + mg;
            if (ra && rb) { best = s1; dbest = v1; }
            else scan = true;
        }
        if (scan) {                                  // every point, first minimum in table order
            dbest = dist(0);
            best = 0;
            for (int s1 = 1; s1 < M; ++s1) {
                const double d = dist(s1);
                if (d < dbest) { dbest = d; best = s1; }
            }
        }
        // first minimum over the lanes (x_0 in table order)
        double dm = on ? dbest : INFINITY;
        int li = on ? lane : 64;
        wave_argmin_dpp(dm, li);                     // wave-uniform (dm, li)
        const int i1 = __builtin_amdgcn_readlane(best, li & 63);
        if (lane == 0) {
            const cd xa = s_cons[li & 63], xb = s_cons[i1];
            cd* out = a.mom + (size_t)gsym * MS;
            out[0] = xa;
            out[1] = xb;
            out[2] = cmulc(xa, xa);
            out[3] = cmulc(xa, xb);
            out[4] = cmulc(xb, xa);
            out[5] = cmulc(xb, xb);
        }
        if (c.count && lane == 0) atomicAdd(&g_estep_pair, 1ull);
    }
}

}  // namespace

bool estep_pair_supported(const Problem& pb, int mode) {
    if (g_debug.estep_nopair) return false;
    if (pb.NT == 2)                                 // estep_fact2_kernel / estep_hard2_kernel
        return (mode == SBCE_ESTEP_SOFT || mode == SBCE_ESTEP_HARD) && pb.M >= 4 && pb.M <= 64 &&
               pb.NR >= 2 && pb.NR <= 8;
    if (mode != SBCE_ESTEP_SOFT) return false;
    return pb.NT == 4 && pb.M == 16 && pb.NR >= 4 && pb.NR <= 8;
}

// a.list: this pass's list (EstepArgs::list, counters 3 and 4, zeroed by the caller); the
// symbols it cannot represent join the sweep's list (counter 0)
hipError_t launch_estep_pair(const Problem& pb, const EstepArgs& a, int stride, int count, int mode,
                             hipStream_t s) {
    PairConst c;
    c.B = pb.B; c.Td = pb.Td; c.stride = stride;
    c.inv_s2 = 1.0 / (pb.varn * pb.varn);
    c.thr_d = 50.0 * pb.varn * pb.varn;              // estep.hip kSkipThr varn^2 (TrialNoise::thr_d)
    c.count = count;
    // waves grab listed symbols until the list is exhausted: a grid that fills the chip
    const long nsym = (long)pb.B * pb.Td;
    long blocks = (nsym + kPairWaves - 1) / kPairWaves;
    if (blocks > 768) blocks = 768;                  // 3 blocks per CU are resident (LDS, VGPRs)
    const dim3 grid((unsigned)blocks), blk(64 * kPairWaves);
    if (pb.NT == 2) {
        long fb = (nsym + 8 * kF2Waves - 1) / (8 * kF2Waves);   // >= 8 symbols per wave
        if (fb > 2048) fb = 2048;
        if (fb < 1) fb = 1;
        const dim3 fgrid((unsigned)fb);
        if (mode == SBCE_ESTEP_HARD) {
            switch (pb.NR) {
#define SBCE_H2(n) case n: hipLaunchKernelGGL((estep_hard2_kernel<n>), fgrid, dim3(64 * kF2Waves), 0, s, a, c, pb.M); break;
                SBCE_H2(2) SBCE_H2(3) SBCE_H2(4) SBCE_H2(5) SBCE_H2(6) SBCE_H2(7) SBCE_H2(8)
#undef SBCE_H2
                default: return hipErrorInvalidValue;
            }
            return hipGetLastError();
        }
        switch (pb.NR) {
#define SBCE_F2(n) case n: hipLaunchKernelGGL((estep_fact2_kernel<n>), fgrid, dim3(64 * kF2Waves), 0, s, a, c, pb.M); \
                           hipLaunchKernelGGL((estep_soft2_kernel<n>), fgrid, dim3(64 * kF2Waves), 0, s, a, c, pb.M); break;
            SBCE_F2(2) SBCE_F2(3) SBCE_F2(4) SBCE_F2(5) SBCE_F2(6) SBCE_F2(7) SBCE_F2(8)
#undef SBCE_F2
            default: return hipErrorInvalidValue;
        }
        return hipGetLastError();
    }
    switch (pb.NR) {
        case 4: hipLaunchKernelGGL((estep_pair_kernel<4>), grid, blk, 0, s, a, c); break;
        case 5: hipLaunchKernelGGL((estep_pair_kernel<5>), grid, blk, 0, s, a, c); break;
        case 6: hipLaunchKernelGGL((estep_pair_kernel<6>), grid, blk, 0, s, a, c); break;
        case 7: hipLaunchKernelGGL((estep_pair_kernel<7>), grid, blk, 0, s, a, c); break;
        case 8: hipLaunchKernelGGL((estep_pair_kernel<8>), grid, blk, 0, s, a, c); break;
        default: return hipErrorInvalidValue;
    }
    return hipGetLastError();
}

hipError_t estep_debug_pair(unsigned long long* out, int reset) {
    if (reset) {
        const unsigned long long z = 0;
        return hipMemcpyToSymbol(HIP_SYMBOL(g_estep_pair), &z, sizeof(z), 0, hipMemcpyHostToDevice);
    }
    return hipMemcpyFromSymbol(out, HIP_SYMBOL(g_estep_pair), sizeof(*out), 0, hipMemcpyDeviceToHost);
}

}  // namespace sbce
