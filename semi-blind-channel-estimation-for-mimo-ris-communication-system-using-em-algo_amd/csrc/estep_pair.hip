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

}  // namespace

bool estep_pair_supported(const Problem& pb, int mode) {
    return mode == SBCE_ESTEP_SOFT && pb.NT == 4 && pb.M == 16 && pb.NR >= 4 && pb.NR <= 8 &&
           !g_debug.estep_nopair;
}

// a.list: this pass's list (EstepArgs::list, counters 3 and 4, zeroed by the caller); the
// symbols it cannot represent join the sweep's list (counter 0)
hipError_t launch_estep_pair(const Problem& pb, const EstepArgs& a, int stride, int count,
                             hipStream_t s) {
    PairConst c;
    c.B = pb.B; c.Td = pb.Td; c.stride = stride;
    c.inv_s2 = 1.0 / (pb.varn * pb.varn);
    c.count = count;
    // waves grab listed symbols until the list is exhausted: a grid that fills the chip
    const long nsym = (long)pb.B * pb.Td;
    long blocks = (nsym + kPairWaves - 1) / kPairWaves;
    if (blocks > 768) blocks = 768;                  // 3 blocks per CU are resident (LDS, VGPRs)
    const dim3 grid((unsigned)blocks), blk(64 * kPairWaves);
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
