// E-step kernel: per-symbol posterior moments over all J = M^n_tx hypotheses.
//
// Reference: "Proposed method/Proposed_method_NMSEvsTp.py":61-71 (exact soft
// posterior beta_{t,j} = exp(-||y_t - Z_{t,j} theta||^2/varn^2) / sum) and
// "Proposed method/ML_detecctor.py":65-77 (hard "log-max": argmax beta).
//
// Reduced form (SURVEY.md §8 preamble): Z_{t,j} theta = H_eff(t) x_j with
// H_eff(t) = sum_p psi_{p,t} H_c[:, p*n_tx:(p+1)*n_tx].  The streams are split
// into A = {0..NA-1} and B = {NA..NT-1}; hypothesis j = i*JB + k (itertools.product
// order, first stream slowest) with i indexing A and k indexing B.  Then
//   r_{ik} = (y - H_A x_A(i)) - H_B x_B(k) = p_i - q_k,
//   d_{ik} = ||p_i||^2 + ||q_k||^2 - 2 Re(p_i^H q_k)     (2*NR FMA + 1 add),
// and the moments m_t = E[x], S_t = E[x x^H] follow from per-lane sums:
//   lane k keeps  c_k = sum_i w_ik,  mu_k[a] = sum_i w_ik x_a(i)   (a in A),
//   and shared    nu[a] = sum w |x_a|^2,  kap = sum w x_0 conj(x_1)  (A pair);
//   B-side and A x B cross moments come from c_k x_b(k) and mu_k[a] conj(x_b(k)).
//
// Mapping (CDNA4, wave64): one SYMBOL lives in one segment of S lanes of ONE
// wave (S = min(JB, 64)); every reduction is intra-wave (xor shuffles), waves
// never synchronise.  Each lane holds KP values of k (q_k in registers) and
// sweeps all i; p_i (pre-scaled by -2) and ||p_i||^2 are computed by the wave
// into LDS, 64 entries at a time, and read back as broadcasts.
//
// Softmax numerics: weights are exp(-(d - m)/varn^2) with m a running,
// segment-uniform minimum distance (log-sum-exp; the reference uses an
// unbounded-exponent mpmath/gmpy2 exp instead).  A chunk of CH x KP hypotheses
// per lane is skipped when every lane's distances exceed m + 50*varn^2: each
// skipped weight is < e^-50 = 2e-22 of the segment maximum (total < 1e-17
// relative for J <= 2^24), far below float64 resolution of the sums.
#include <stdlib.h>

#include "sbce_internal.h"

namespace sbce {

namespace {

constexpr int kWave = 64;
constexpr int kWavesPerBlock = 4;
constexpr int kCH = 4;              // i-values per inner chunk
constexpr double kSkipThr = 50.0;   // skip weights below e^-50 of the running max

struct EstepConst {
    int B, Td, P, M, lm;       // lm = log2(M)
    int S, SPW;                // lanes per symbol, symbols per wave
    int JA, JB, npass, CI, CIp;
    int nparts;                // H_eff partial-sum split per output
    int heff_cd, ptab_cd;      // per-wave LDS carve (complex doubles)
    double inv_s2, thr_d;
};

__device__ __forceinline__ double seg_min(double v, int S) {
    for (int off = S >> 1; off >= 1; off >>= 1) v = fmin(v, shfl_xor_d(v, off));
    return v;
}
__device__ __forceinline__ double seg_sum(double v, int S) {
    for (int off = S >> 1; off >= 1; off >>= 1) v += shfl_xor_d(v, off);
    return v;
}
__device__ __forceinline__ cd seg_sum(cd v, int S) {
    return cmk(seg_sum(v.x, S), seg_sum(v.y, S));
}

template <int NT, int NR, int KP, int MODE>
__global__ __launch_bounds__(256) void estep_kernel(EstepArgs a, EstepConst c) {
    constexpr int NA = NT / 2;
    constexpr int NB = NT - NA;
    constexpr int NO = NT * NR;
    constexpr int NPA = NA * (NA - 1) / 2;   // pairs inside A (0 or 1)
    constexpr int NPB = NB * (NB - 1) / 2;   // pairs inside B (0 or 1)
    constexpr int PST = NR + 1;              // ptab row stride (complex doubles)
    static_assert(NA <= 2 && NB <= 2, "exact E-step supports n_tx <= 4");

    extern __shared__ __attribute__((aligned(16))) char smem[];
    cd* s_cons = reinterpret_cast<cd*>(smem);
    const int wave = threadIdx.x >> 6;
    const int lane = threadIdx.x & 63;
    cd* s_heff = s_cons + 64 + wave * (c.heff_cd + c.ptab_cd);
    cd* s_ptab = s_heff + c.heff_cd;

    for (int i = threadIdx.x; i < c.M; i += blockDim.x) s_cons[i] = a.cons[i];
    __syncthreads();

    const long nsym = (long)c.B * c.Td;
    const long wsym0 = ((long)blockIdx.x * kWavesPerBlock + wave) * c.SPW;
    if (wsym0 >= nsym) return;                       // whole wave out of range
    const int S = c.S;
    const int seg = lane / S;
    const int sl = lane & (S - 1);
    long gsym = wsym0 + seg;
    bool valid = gsym < nsym;
    if (!valid) gsym = nsym - 1;                     // compute on a real symbol, skip write
    const int b = (int)(gsym / c.Td);
    const int t = (int)(gsym - (long)b * c.Td);
    if (a.done && a.done[b]) valid = false;
    if (a.varn_t) {                                  // per-trial noise variance (ABI 6)
        const TrialNoise tn = trial_noise(a.varn_t[b]);
        c.inv_s2 = tn.inv_s2;
        c.thr_d = tn.thr_d;
    }

    // ---------------- effective channel H_eff(t): heff[a*NR + r] --------------
    {
        const cd* th = a.theta + (size_t)b * c.P * NO;      // [p][a][r]
        const cd* ps = a.psid + (size_t)gsym * c.P;
        const int ntask = NO * c.nparts;
        cd* part = s_ptab + seg * ntask;
        for (int task = sl; task < ntask; task += S) {
            const int o = task % NO, pp = task / NO;
            cd acc = czero();
            for (int p = pp; p < c.P; p += c.nparts) acc = cfma(acc, ps[p], th[p * NO + o]);
            part[task] = acc;
        }
        wave_sync();
        for (int o = sl; o < NO; o += S) {
            cd s = part[o];
            for (int pp = 1; pp < c.nparts; ++pp) s = cadd(s, part[pp * NO + o]);
            s_heff[seg * NO + o] = s;
        }
        wave_sync();
    }
    const cd* H = s_heff + seg * NO;
    cd y[NR];
#pragma unroll
    for (int r = 0; r < NR; ++r) y[r] = a.yd[(size_t)gsym * NR + r];

    const int mask = c.M - 1;
    const double inv_s2 = c.inv_s2;

    // per-lane state
    double mshift = INFINITY;
    double tot_c = 0.0;
    cd tot_muA[NA > 0 ? NA : 1];
    double nu[NA > 0 ? NA : 1];
    cd kap = czero();
    cd tot_mB[NB];
    double tot_nB[NB];
    cd tot_kB = czero();
    cd tot_X[NA > 0 ? NA : 1][NB];
#pragma unroll
    for (int q = 0; q < (NA > 0 ? NA : 1); ++q) {
        tot_muA[q] = czero(); nu[q] = 0.0;
#pragma unroll
        for (int bb = 0; bb < NB; ++bb) tot_X[q][bb] = czero();
    }
#pragma unroll
    for (int bb = 0; bb < NB; ++bb) { tot_mB[bb] = czero(); tot_nB[bb] = 0.0; }
    double best_d = INFINITY;
    int best_j = 0x7fffffff;

    for (int pass = 0; pass < c.npass; ++pass) {
        // ---- this lane's KP hypotheses of B: q_k = H_B x_B(k) ----
        cd q[KP][NR];
        double gam[KP];
        double ck[KP];
        cd mu[KP][NA > 0 ? NA : 1];
#pragma unroll
        for (int cc = 0; cc < KP; ++cc) {
            const int k = pass * S * KP + cc * S + sl;
#pragma unroll
            for (int r = 0; r < NR; ++r) q[cc][r] = czero();
#pragma unroll
            for (int bb = 0; bb < NB; ++bb) {
                const cd x = s_cons[(k >> (c.lm * (NB - 1 - bb))) & mask];
#pragma unroll
                for (int r = 0; r < NR; ++r) q[cc][r] = cfma(q[cc][r], H[(NA + bb) * NR + r], x);
            }
            double g = 0.0;
#pragma unroll
            for (int r = 0; r < NR; ++r) g += cabs2(q[cc][r]);
            gam[cc] = g;
            ck[cc] = 0.0;
#pragma unroll
            for (int q2 = 0; q2 < (NA > 0 ? NA : 1); ++q2) mu[cc][q2] = czero();
        }

        for (int i0 = 0; i0 < c.JA; i0 += c.CI) {
            // ---- p_i = y - H_A x_A(i), stored as (-2 p_i, ||p_i||^2) ----
            wave_sync();
            cd* pt = s_ptab + seg * c.CIp * PST;
            for (int e = sl; e < c.CIp; e += S) {
                cd* row = pt + e * PST;
                if (e < c.CI) {
                    const int i = i0 + e;
                    double al = 0.0;
#pragma unroll
                    for (int r = 0; r < NR; ++r) {
                        cd pr = y[r];
#pragma unroll
                        for (int q2 = 0; q2 < NA; ++q2) {
                            const cd x = s_cons[(i >> (c.lm * (NA - 1 - q2))) & mask];
                            const cd hx = cmul(H[q2 * NR + r], x);
                            pr = csub(pr, hx);
                        }
                        al += cabs2(pr);
                        row[r] = cscale(pr, -2.0);
                    }
                    row[NR] = cmk(al, 0.0);
                } else {
#pragma unroll
                    for (int r = 0; r < NR; ++r) row[r] = czero();
                    row[NR] = cmk(INFINITY, 0.0);
                }
            }
            wave_sync();

            for (int i1 = 0; i1 < c.CIp; i1 += kCH) {
                double d[kCH][KP];
#pragma unroll
                for (int ii = 0; ii < kCH; ++ii) {
                    const cd* row = pt + (i1 + ii) * PST;
                    cd pm[NR];
#pragma unroll
                    for (int r = 0; r < NR; ++r) pm[r] = row[r];
                    const double al = row[NR].x;
#pragma unroll
                    for (int cc = 0; cc < KP; ++cc) {
                        double acc = al + gam[cc];
#pragma unroll
                        for (int r = 0; r < NR; ++r) {
                            acc = fma(pm[r].x, q[cc][r].x, acc);
                            acc = fma(pm[r].y, q[cc][r].y, acc);
                        }
                        d[ii][cc] = acc;
                    }
                }
                if (MODE == SBCE_ESTEP_HARD) {
#pragma unroll
                    for (int ii = 0; ii < kCH; ++ii) {
                        const int i = i0 + i1 + ii;
#pragma unroll
                        for (int cc = 0; cc < KP; ++cc) {
                            const int j = i * c.JB + pass * S * KP + cc * S + sl;
                            const double dv = d[ii][cc];
                            if (dv < best_d || (dv == best_d && j < best_j)) { best_d = dv; best_j = j; }
                        }
                    }
                    continue;
                }
                double cm = d[0][0];
#pragma unroll
                for (int ii = 0; ii < kCH; ++ii)
#pragma unroll
                    for (int cc = 0; cc < KP; ++cc) cm = fmin(cm, d[ii][cc]);

                if (__any(cm < mshift)) {
                    const double mn = seg_min(fmin(cm, mshift), S);
                    const double f = (mshift == INFINITY) ? 0.0 : fexp_neg((mn - mshift) * inv_s2);
                    mshift = mn;
                    tot_c *= f; tot_kB = cscale(tot_kB, f); kap = cscale(kap, f);
#pragma unroll
                    for (int q2 = 0; q2 < (NA > 0 ? NA : 1); ++q2) {
                        tot_muA[q2] = cscale(tot_muA[q2], f); nu[q2] *= f;
#pragma unroll
                        for (int bb = 0; bb < NB; ++bb) tot_X[q2][bb] = cscale(tot_X[q2][bb], f);
                    }
#pragma unroll
                    for (int bb = 0; bb < NB; ++bb) { tot_mB[bb] = cscale(tot_mB[bb], f); tot_nB[bb] *= f; }
#pragma unroll
                    for (int cc = 0; cc < KP; ++cc) {
                        ck[cc] *= f;
#pragma unroll
                        for (int q2 = 0; q2 < (NA > 0 ? NA : 1); ++q2) mu[cc][q2] = cscale(mu[cc][q2], f);
                    }
                }
                if (!__any(cm <= mshift + c.thr_d)) continue;   // whole chunk negligible

#pragma unroll
                for (int ii = 0; ii < kCH; ++ii) {
                    const int i = i0 + i1 + ii;
                    cd xa[NA > 0 ? NA : 1];
                    double xa2[NA > 0 ? NA : 1];
#pragma unroll
                    for (int q2 = 0; q2 < NA; ++q2) {
                        xa[q2] = s_cons[(i >> (c.lm * (NA - 1 - q2))) & mask];
                        xa2[q2] = cabs2(xa[q2]);
                    }
                    cd x01 = czero();
                    if (NPA) x01 = cmulc(xa[0], xa[NA > 1 ? 1 : 0]);
#pragma unroll
                    for (int cc = 0; cc < KP; ++cc) {
                        const double w = fexp_neg((mshift - d[ii][cc]) * inv_s2);
                        ck[cc] += w;
#pragma unroll
                        for (int q2 = 0; q2 < NA; ++q2) {
                            mu[cc][q2] = caxpy(mu[cc][q2], w, xa[q2]);
                            nu[q2] = fma(w, xa2[q2], nu[q2]);
                        }
                        if (NPA) kap = caxpy(kap, w, x01);
                    }
                }
            }
        }
        if (MODE == SBCE_ESTEP_SOFT) {
            // ---- fold this pass's per-k sums into the lane totals ----
#pragma unroll
            for (int cc = 0; cc < KP; ++cc) {
                const int k = pass * S * KP + cc * S + sl;
                cd xb[NB];
#pragma unroll
                for (int bb = 0; bb < NB; ++bb) xb[bb] = s_cons[(k >> (c.lm * (NB - 1 - bb))) & mask];
                tot_c += ck[cc];
#pragma unroll
                for (int bb = 0; bb < NB; ++bb) {
                    tot_mB[bb] = caxpy(tot_mB[bb], ck[cc], xb[bb]);
                    tot_nB[bb] = fma(ck[cc], cabs2(xb[bb]), tot_nB[bb]);
                }
                if (NPB) tot_kB = caxpy(tot_kB, ck[cc], cmulc(xb[0], xb[NB > 1 ? 1 : 0]));
#pragma unroll
                for (int q2 = 0; q2 < NA; ++q2) {
                    tot_muA[q2] = cadd(tot_muA[q2], mu[cc][q2]);
#pragma unroll
                    for (int bb = 0; bb < NB; ++bb) tot_X[q2][bb] = cfmac(tot_X[q2][bb], mu[cc][q2], xb[bb]);
                }
            }
        }
    }

    constexpr int MS = NT + NT * NT;
    cd* out = a.mom + (size_t)gsym * MS;
    if (MODE == SBCE_ESTEP_HARD) {
        for (int off = S >> 1; off >= 1; off >>= 1) {
            const double od = shfl_xor_d(best_d, off);
            const int oj = __shfl_xor(best_j, off);
            if (od < best_d || (od == best_d && oj < best_j)) { best_d = od; best_j = oj; }
        }
        if (valid && sl == 0) {
            cd x[NT];
#pragma unroll
            for (int s2 = 0; s2 < NT; ++s2) x[s2] = s_cons[(best_j >> (c.lm * (NT - 1 - s2))) & mask];
#pragma unroll
            for (int s2 = 0; s2 < NT; ++s2) {
                out[s2] = x[s2];
#pragma unroll
                for (int s3 = 0; s3 < NT; ++s3) out[NT + s2 * NT + s3] = cmulc(x[s2], x[s3]);
            }
        }
        return;
    }

    // ---- segment reductions (all lanes of a segment share mshift) ----
    tot_c = seg_sum(tot_c, S);
    kap = seg_sum(kap, S);
    tot_kB = seg_sum(tot_kB, S);
#pragma unroll
    for (int q2 = 0; q2 < NA; ++q2) {
        tot_muA[q2] = seg_sum(tot_muA[q2], S);
        nu[q2] = seg_sum(nu[q2], S);
#pragma unroll
        for (int bb = 0; bb < NB; ++bb) tot_X[q2][bb] = seg_sum(tot_X[q2][bb], S);
    }
#pragma unroll
    for (int bb = 0; bb < NB; ++bb) { tot_mB[bb] = seg_sum(tot_mB[bb], S); tot_nB[bb] = seg_sum(tot_nB[bb], S); }

    if (valid && sl == 0) {
        const double iz = 1.0 / tot_c;
        cd m[NT];
        cd Sm[NT][NT];
#pragma unroll
        for (int q2 = 0; q2 < NA; ++q2) {
            m[q2] = cscale(tot_muA[q2], iz);
            Sm[q2][q2] = cmk(nu[q2] * iz, 0.0);
        }
#pragma unroll
        for (int bb = 0; bb < NB; ++bb) {
            m[NA + bb] = cscale(tot_mB[bb], iz);
            Sm[NA + bb][NA + bb] = cmk(tot_nB[bb] * iz, 0.0);
        }
        if (NPA) { Sm[0][NA > 1 ? 1 : 0] = cscale(kap, iz); Sm[NA > 1 ? 1 : 0][0] = cconj(cscale(kap, iz)); }
        if (NPB) {
            Sm[NA][NT - 1] = cscale(tot_kB, iz);
            Sm[NT - 1][NA] = cconj(cscale(tot_kB, iz));
        }
#pragma unroll
        for (int q2 = 0; q2 < NA; ++q2)
#pragma unroll
            for (int bb = 0; bb < NB; ++bb) {
                const cd v = cscale(tot_X[q2][bb], iz);
                Sm[q2][NA + bb] = v;
                Sm[NA + bb][q2] = cconj(v);
            }
#pragma unroll
        for (int s2 = 0; s2 < NT; ++s2) {
            out[s2] = m[s2];
#pragma unroll
            for (int s3 = 0; s3 < NT; ++s3) out[NT + s2 * NT + s3] = Sm[s2][s3];
        }
    }
}

// ============================================================================
// MFMA variant (gfx950 FP64 matrix cores) for JA >= 16 and JB >= 16.
//
// One wave per symbol.  The hypothesis grid (i over A, k over B) is tiled in
// 16 x 16 tiles; each tile's distances
//     d_ik = (alpha_i + gamma_k) + sum_kk P'[i][kk] Q[kk][k],
// with P' = (-2 Re p_i, -2 Im p_i) and Q = (Re q_k, Im q_k) (K = 2*NR padded to
// a multiple of 4), come out of KPAD/4 chained v_mfma_f64_16x16x4f64 whose
// accumulator is initialised with alpha_i + gamma_k.  Lane l owns column
// k = 16*kt + (l & 15) and rows i = 16*t + (l >> 4) + 4*j (j < 4), so the
// per-k posterior sums (c_k, mu_k) are per lane, exactly like the VALU kernel.
// The VALU only does the running minimum, the skip test and (rarely, at high
// SNR) the exp/accumulate work, in parallel with the matrix pipe.
// The A operand is assembled per tile from two small LDS tables, -2 p_i =
// U_{s0} + V_{s1} (U_s = -2(y - h_0 x_s), V_s = 2 h_1 x_s, layout [kk][s]:
// conflict-free ds_read_b64), and alpha_i = ||p_i||^2 is tabulated 256 at a time.
// ============================================================================
typedef double d4v __attribute__((ext_vector_type(4)));

// Initial bound for the hypothesis sweep: the distance ||y - H x_c||^2 of x_c = the
// per-stream nearest constellation points of the regularised LS estimate
// (H^H H + reg I)^-1 H^H y.  x_c is a real hypothesis, so its weight bounds the posterior
// maximum from below: as the initial log-sum-exp shift it loses nothing, and as the initial
// hard-decision bound (plus a rounding margin) it keeps the argmin.  At medium and high SNR
// x_c is the ML point, the running minimum never moves and nearly every tile group is
// dismissed by one comparison.  Wave-uniform (every lane computes the same value); `scale`
// bounds the magnitude of the terms a tile distance is assembled from (rounding margin).
template <int NT, int NR>
__device__ double candidate_distance(const cd* H, const cd* yg, const cd* s_cons, int M,
                                     double reg, cd* scratch, int lane, double& scale) {
    cd* sG = scratch;            // [NT][NT]
    cd* sHy = scratch + 16;      // [NT]
    if (lane < NT * NT) {
        const int u = lane / NT, v = lane - u * NT;
        cd acc = czero();
#pragma unroll
        for (int r = 0; r < NR; ++r) acc = cfmac(acc, H[v * NR + r], H[u * NR + r]);
        if (u == v) acc.x += reg;
        sG[lane] = acc;
    } else if (lane >= 32 && lane < 32 + NT) {
        const int u = lane - 32;
        cd acc = czero();
#pragma unroll
        for (int r = 0; r < NR; ++r) acc = cfmac(acc, yg[r], H[u * NR + r]);
        sHy[u] = acc;
    }
    wave_sync();
    // complex Cholesky G = L L^H and the two triangular solves, in registers
    cd Lm[NT][NT];
    double dinv[NT];
    cd z[NT];
#pragma unroll
    for (int j = 0; j < NT; ++j) {
        double d = sG[j * NT + j].x;
#pragma unroll
        for (int k = 0; k < j; ++k) d -= cabs2(Lm[j][k]);
        const double inv = fast_rsqrt(fmax(d, 1e-300));
        dinv[j] = inv;
#pragma unroll
        for (int i = j + 1; i < NT; ++i) {
            cd s = sG[i * NT + j];
#pragma unroll
            for (int k = 0; k < j; ++k) s = csub(s, cmulc(Lm[i][k], Lm[j][k]));
            Lm[i][j] = cscale(s, inv);
        }
    }
#pragma unroll
    for (int i = 0; i < NT; ++i) {
        cd s = sHy[i];
#pragma unroll
        for (int k = 0; k < i; ++k) s = csub(s, cmul(Lm[i][k], z[k]));
        z[i] = cscale(s, dinv[i]);
    }
#pragma unroll
    for (int i = NT - 1; i >= 0; --i) {
        cd s = z[i];
#pragma unroll
        for (int k = i + 1; k < NT; ++k) s = csub(s, cmul(cconj(Lm[k][i]), z[k]));
        z[i] = cscale(s, dinv[i]);
    }
    // nearest constellation point per stream: lanes 16 q .. 16 q + 15 handle stream q
    const int qa = lane >> 4;
    cd za = z[0];
#pragma unroll
    for (int q = 1; q < NT; ++q) za = csel(qa == q, z[q], za);
    double bd = INFINITY;
    int bs = 0;
    if (qa < NT)
        for (int s = lane & 15; s < M; s += 16) {
            const double dd = cabs2(csub(za, s_cons[s]));
            if (dd < bd) { bd = dd; bs = s; }
        }
    for (int off = 8; off >= 1; off >>= 1) {
        const double od = shfl_xor_d(bd, off);
        const int os = __shfl_xor(bs, off);
        if (od < bd || (od == bd && os < bs)) { bd = od; bs = os; }
    }
    cd x[NT];
#pragma unroll
    for (int q = 0; q < NT; ++q) x[q] = s_cons[__shfl(bs, 16 * q)];
    double d0 = 0.0, sc = 0.0;
#pragma unroll
    for (int r = 0; r < NR; ++r) {
        cd res = yg[r];
        sc += cabs2(res);
#pragma unroll
        for (int q = 0; q < NT; ++q) {
            const cd hx = cmul(H[q * NR + r], x[q]);
            res = csub(res, hx);
            sc += NT * cabs2(hx);
        }
        d0 += cabs2(res);
    }
    wave_sync();                 // scratch is reused by the caller
    scale = sc;
    return d0;
}


constexpr int kMfmaWaves = 2;
constexpr int kChunk = 256;
constexpr int kScreenD = 256;   // per-wave LDS doubles of the V16 FP32 screen tables

typedef float f4v __attribute__((ext_vector_type(4)));

// Per-wave LDS doubles of the MFMA sweep: heff | alpha | U | V | Q2 | lb | scratch (128) |
// 2 x staged record (DMA double buffer: 128 + 32 done words, or the record itself) |
// FP32 screen tables (V16: alpha and U as floats, kScreenD doubles)
constexpr int mfma_rec_d(int rec_words) { return 2 * (rec_words <= 128 ? 160 : (rec_words + 1) / 2 * 2 + 32); }
constexpr int mfma_tab_d(int NO, int chunk, int steps, int M, int nkt_pad, int rec_words) {
    return (2 * NO + chunk + 3 * (4 * steps) * M + nkt_pad + 128 + 1) / 2 * 2 + mfma_rec_d(rec_words) +
           kScreenD;
}

struct MfmaConst {
    int B, Td, P, M, lm;
    int JA, JB, chunk, nparts;
    int tab_d;                 // per-wave LDS doubles
    double inv_s2, thr_d;
    double reg;                // ridge of the candidate's LS estimate (0.1 varn^2)
    int nkt_pad;               // column tiles JB / 16, rounded up to even (LDS carve)
    int prune;                 // column-tile bounds on (SBCE_ESTEP_PRUNE=0 disables: A/B runs)
    int count;                 // diagnostic MFMA count (SBCE_ESTEP_COUNT=1)
    int prep_stride;           // doubles per symbol of EstepArgs::prep
    int rowb_off;              // offset of the row-tile bound vectors in a prep record
    int rowb;                  // row-tile bounds on (NT = 4 with a prep record)
    int rec_words;             // prep record + y_t, doubles (staged per symbol in LDS)
    int spw;                   // symbols per wave (consecutive; the next record prefetched)
    int screen;                // V16 FP32 screen of the tile groups (SBCE_ESTEP_F32=0 disables)
};

// V16 (M == 16, NA == 2): the A operand's V term, V[kk][i & 15] = V[kk][lane & 15], is the
// same for every tile, so it is hoisted into registers (one LDS read + add per MFMA
// instead of two reads + add).  gamma_k is not added to the 16 accumulators: the skip
// tests use min(acc) + gamma and the rare exp path adds it back.  (PMC at cfg1 showed
// the f64 VALU work between the MFMAs, which does not co-execute with them, as the
// limiter: 40 % MFMA busy.)
// Exact lower bounds per column tile (16 consecutive k): every hypothesis (i, k) has
//   d_ik = ||y - H_A x_A(i) - H_B x_B(k)||^2 >= min_x ||(y - H_B x_B(k)) - H_A x||^2
//        = ||P (y - H_B x_B(k))||^2,      P = projector onto span(H_A)^perp
// (the best continuous x_A can do no better: the partial distance of a sphere decoder).
// A tile whose bound exceeds the skip bound holds only hypotheses whose weights are below
// e^-50 of the posterior maximum (soft) or that cannot be the argmin (hard), exactly the
// hypotheses the per-group test already discards, so the sweep skips their MFMAs.  P comes
// from a twice-orthogonalised Gram-Schmidt basis of H_A, lane r of each 8-lane group owning
// component r; a near-dependent H_A (or n_rx <= |A|, where P = 0) leaves the bounds at 0.
// Returns the magnitude scale of the bound terms (rounding margin).
template <int NT, int NR>
__device__ double column_tile_bounds(const cd* H, const cd* yg, const cd* s_cons, int M, int lm,
                                     int nkt, double* s_lb, cd* scratch, int lane) {
    constexpr int NA = NT / 2, NB = NT - NA;
    const int mask = M - 1;
    const int r = lane & 7;
    const bool own = r < NR;
    int xa[6];
#pragma unroll
    for (int i = 0; i < 6; ++i) xa[i] = (lane ^ (32 >> i)) << 2;     // xor 32 .. 1
    auto rsum = [&](double v) {                                      // sum over the 8-lane group
#pragma unroll
        for (int i = 3; i < 6; ++i) v += bperm_d(v, xa[i]);
        return v;
    };
    auto rdot = [&](cd u, cd v) { return cmk(rsum(fma(v.x, u.x, v.y * u.y)),    // u^H v
                                             rsum(fma(v.y, u.x, -v.x * u.y))); };
    cd u[NA];
    bool ok = true;
#pragma unroll
    for (int q = 0; q < NA; ++q) {
        cd v = own ? H[q * NR + r] : czero();
        const double h2 = rsum(cabs2(v));
#pragma unroll
        for (int rep = 0; rep < 2; ++rep)
#pragma unroll
            for (int j = 0; j < q; ++j) v = csub(v, cmul(u[j], rdot(u[j], v)));
        const double n2 = rsum(cabs2(v));
        ok = ok && h2 > 0.0 && n2 > 1e-6 * h2;
        u[q] = cscale(v, ok ? fast_rsqrt(n2) : 0.0);
    }
    cd w = own ? yg[r] : czero();
    double sc = rsum(cabs2(w));
    cd g[NB];
    double g2 = 0.0;
#pragma unroll
    for (int b = 0; b < NB; ++b) {
        g[b] = own ? H[(NA + b) * NR + r] : czero();
        g2 += cabs2(g[b]);
    }
#pragma unroll
    for (int j = 0; j < NA; ++j) {
        w = csub(w, cmul(u[j], rdot(u[j], w)));
#pragma unroll
        for (int b = 0; b < NB; ++b) g[b] = csub(g[b], cmul(u[j], rdot(u[j], g[b])));
    }
    if (lane < NR) {
        scratch[r] = w;
#pragma unroll
        for (int b = 0; b < NB; ++b) scratch[8 * (b + 1) + r] = g[b];
    }
    // scale: ||y||^2 + NB sum_b ||h_b||^2 max|c|^2 bounds every term of a bound
    double cmax2 = lane < M ? cabs2(s_cons[lane]) : 0.0;
#pragma unroll
    for (int i = 0; i < 6; ++i) cmax2 = fmax(cmax2, bperm_d(cmax2, xa[i]));
    sc += NB * cmax2 * rsum(g2);
    wave_sync();
    for (int kt0 = 0; kt0 < nkt; kt0 += 4) {
        const int kt = kt0 + (lane >> 4);
        const int k = kt * 16 + (lane & 15);
        cd xb[NB];
#pragma unroll
        for (int b = 0; b < NB; ++b) xb[b] = s_cons[(k >> (lm * (NB - 1 - b))) & mask];
        double lb = 0.0;
#pragma unroll
        for (int rr = 0; rr < NR; ++rr) {
            cd res = scratch[rr];
#pragma unroll
            for (int b = 0; b < NB; ++b) res = csub(res, cmul(scratch[8 * (b + 1) + rr], xb[b]));
            lb += cabs2(res);
        }
        if (!ok) lb = 0.0;
#pragma unroll
        for (int i = 2; i < 6; ++i) lb = fmin(lb, bperm_d(lb, xa[i]));   // 16-lane minimum
        if ((lane & 15) == 0 && kt < nkt) s_lb[kt] = lb;
    }
    wave_sync();
    return sc;
}

// Diagnostic (MfmaConst::count, SBCE_ESTEP_COUNT=1): FP64 MFMAs the sweep issued, for the
// executed-work roofline next to the bounds' pruning.
__device__ unsigned long long g_estep_mfma;

template <int NT, int NR, int MODE, int TU, bool V16>
__device__ __forceinline__ void estep_mfma_body(const EstepArgs& a, const MfmaConst& c) {
    // V16 (n_tx = 4, M = 16): the layout constants are compile-time (LDS offsets fold into
    // immediates, one SGPR wave base); otherwise they come from MfmaConst
    const int k_M = V16 ? 16 : c.M;
    const int k_lm = V16 ? 4 : c.lm;
    const int k_JA = V16 ? 256 : c.JA;
    const int k_JB = V16 ? 256 : c.JB;
    const int k_chunk = V16 ? 256 : c.chunk;
    const int k_nkt_pad = V16 ? 16 : c.nkt_pad;
    const int k_rowb_off = V16 ? 4 + 2 * NT * NR + 16 : c.rowb_off;
    const int k_prep_stride = V16 ? k_rowb_off + 6 * NR : c.prep_stride;
    const int k_rec_words = V16 ? k_prep_stride + 2 * NR : c.rec_words;
    const int k_tab_d = V16 ? mfma_tab_d(NT * NR, 256, (2 * NR + 3) / 4, 16, 16, k_rec_words) : c.tab_d;
    constexpr int NA = NT / 2;
    constexpr int NB = NT - NA;
    constexpr int NO = NT * NR;
    constexpr int K2 = 2 * NR;
    constexpr int STEPS = (K2 + 3) / 4;
    constexpr int NPA = NA * (NA - 1) / 2;
    constexpr int NPB = NB * (NB - 1) / 2;
    static_assert(NA >= 1 && NA <= 2 && NB <= 2, "mfma E-step: 2 <= n_tx <= 4");

    // listed sweep: a block whose first wave has no list entry has no work at all (an empty
    // list is common: the launch then costs only its dispatch)
    if (a.list && (long)blockIdx.x * kMfmaWaves >= (long)a.list[(long)c.B * c.Td]) return;
    extern __shared__ __attribute__((aligned(16))) char smem[];
    cd* s_cons = reinterpret_cast<cd*>(smem);
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);   // uniform: SGPR addresses
    const int lane = threadIdx.x & 63;
    double* wbase = reinterpret_cast<double*>(s_cons + 64) + (size_t)wave * k_tab_d;
    cd* s_heff = reinterpret_cast<cd*>(wbase);                 // NO
    double* s_al = wbase + 2 * NO;                             // chunk
    double* s_U = s_al + k_chunk;                              // [KPAD][M]
    double* s_V = s_U + 4 * STEPS * k_M;                       // [KPAD][M]   (NA == 2)
    double* s_Q2 = s_V + 4 * STEPS * k_M;                      // [KPAD][M]   (V16)
    double* s_lb = s_Q2 + 4 * STEPS * k_M;                     // [nkt] column-tile bounds
    double* s_tab = s_lb + k_nkt_pad;                          // scratch: 64 cd
    double* s_recb = s_tab + 128;                  // 2 x [prep record | y_t (128) | done (32)]
    // V16 FP32 screen: alpha (row order: the f32 MFMA's C/D row of value q is 4 (lane >> 4) + q,
    // not the f64 form's (lane >> 4) + 4 q) and U (s_U's layout) as floats
    float* s_al32 = reinterpret_cast<float*>(s_recb + mfma_rec_d(k_rec_words));
    float* s_U32 = s_al32 + 256;

    for (int i = threadIdx.x; i < k_M; i += blockDim.x) s_cons[i] = a.cons[i];
    __syncthreads();

    const long nsym = (long)c.B * c.Td;
    // With a work list (the prep pass's sphere enumeration resolved the other symbols) the
    // waves grab chunks of spw list entries from a counter until the list is exhausted;
    // otherwise each wave takes chunk (block, wave) of all symbols.
    const bool listed = a.list != nullptr;
    int32_t* cnt = listed ? a.list + nsym : nullptr;
    const long nwork = listed ? (long)__builtin_amdgcn_readfirstlane(cnt[0]) : nsym;
    const bool prep = a.prep != nullptr;
    auto sym_of = [&](long gi) -> long { return listed ? (long)a.list[gi] : gi; };
    // listed: a wave's first entry is its global wave index (no atomic -- with a short or empty
    // list most waves exit at once; 4096 same-address atomics of an empty list cost ~50 us),
    // the later ones come from the counter, which starts past the first round
    bool first = true;
    for (;;) {
    long chunk_id;
    if (listed) {
        if (first) {
            chunk_id = (long)blockIdx.x * kMfmaWaves + wave;
        } else {
            int v = 0;
            if (lane == 0) v = atomicAdd(cnt + 1, 1);
            chunk_id = (long)gridDim.x * kMfmaWaves + __builtin_amdgcn_readfirstlane(__shfl(v, 0));
        }
        first = false;
    } else {
        chunk_id = (long)blockIdx.x * kMfmaWaves + wave;
    }
    // listed symbols are the expensive ones: one per grab (a chunk's symbols run in series)
    const int spw = listed ? 1 : c.spw;
    const long g0 = chunk_id * spw;
    if (g0 >= nwork) return;
    const long g1 = g0 + spw < nwork ? g0 + spw : nwork;
    // The wave's symbols g0 .. g1-1 in turn.  With a prep record, the next symbol's record,
    // y_t and done flag travel by LDS-DMA (global_load_lds: no VGPRs) into the other half of
    // a double buffer while the current symbol is swept; the sweep reads no global memory,
    // so the wait at the next symbol finds them landed.
    const bool dma = prep && k_rec_words <= 128;
    auto issue = [&](long g, double* dst) {
        int l = lane;                                           // recomputed per issue, not held
        asm volatile("" : "+v"(l));
        const int hs = k_prep_stride >> 1;                      // 16-byte words of the record
        const double* src = a.prep + (size_t)g * k_prep_stride;
        if (l < hs) src += 2 * l;
        else if (l < (k_rec_words >> 1))
            src = reinterpret_cast<const double*>(a.yd) + (size_t)g * 2 * NR + 2 * (l - hs);
        __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)src,
                                         (__attribute__((address_space(3))) void*)dst, 16, 0, 0);
        if (a.done)
            __builtin_amdgcn_global_load_lds(
                (const __attribute__((address_space(1))) void*)(a.done + g / c.Td),
                (__attribute__((address_space(3))) void*)(dst + 128), 4, 0, 0);
    };
    if (dma) issue(sym_of(g0), s_recb);
    for (long gi = g0; gi < g1; ++gi) {
    const long gsym = sym_of(gi);
    const int cur = (int)((gi - g0) & 1);
    double* s_rec = s_recb + cur * 160;
    int dn;
    if (dma) {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // this symbol's record has landed
        wave_sync();
        dn = a.done ? reinterpret_cast<const int*>(s_rec + 128)[0] : 0;
        if (gi + 1 < g1) issue(sym_of(gi + 1), s_recb + (cur ^ 1) * 160);
    } else {
        dn = a.done ? a.done[gsym / c.Td] : 0;
        if (prep && !dn) {
            wave_sync();
            for (int e = lane; e < k_rec_words; e += 64)
                s_rec[e] = e < k_prep_stride
                    ? a.prep[(size_t)gsym * k_prep_stride + e]
                    : reinterpret_cast<const double*>(a.yd)[(size_t)gsym * 2 * NR + e - k_prep_stride];
            wave_sync();
        }
    }
    if (dn) continue;
    // lane index opaque per symbol: values derived from it (constellation points, LDS
    // addresses) are recomputed per symbol instead of being hoisted and held across the loop
    int lane_s = lane;
    asm volatile("" : "+v"(lane_s));
    [&, lane = lane_s]() {
    const int b = (int)(gsym / c.Td);
    const int t = (int)(gsym - (long)b * c.Td);
    const int mask = k_M - 1;
    // the trial's noise constants (per-trial variances, ABI 6): wave-uniform, kept in SGPRs
    double thr_d = c.thr_d, inv_s2 = c.inv_s2, reg = c.reg;
    if (a.varn_t) {
        const TrialNoise tn = trial_noise(a.varn_t[b]);
        thr_d = uniform_d(tn.thr_d);
        inv_s2 = uniform_d(tn.inv_s2);
        reg = uniform_d(tn.reg);
    }

    // ---------------- H_eff(t) ----------------
    if (prep) {
        // H_eff, bounds and y_t are read from the staged record (s_rec)
    } else {
        const cd* th = a.theta + (size_t)b * c.P * NO;
        const cd* ps = a.psid + (size_t)gsym * c.P;
        const int ntask = NO * c.nparts;
        cd* part = reinterpret_cast<cd*>(s_tab);
        if (lane < ntask) {
            const int o = lane % NO, pp = lane / NO;
            cd acc = czero();
            for (int p = pp; p < c.P; p += c.nparts) acc = cfma(acc, ps[p], th[p * NO + o]);
            part[lane] = acc;
        }
        wave_sync();
        if (lane < NO) {
            cd s2 = part[lane];
            for (int pp = 1; pp < c.nparts; ++pp) s2 = cadd(s2, part[pp * NO + lane]);
            s_heff[lane] = s2;
        }
        wave_sync();
    }
    const cd* H = prep ? reinterpret_cast<const cd*>(s_rec + 4) : s_heff;
    const double* lbp = prep ? s_rec + 4 + 2 * NO : s_lb;        // column-tile bounds
    double cscale_d, d0, lb_scale;
    if (prep) {                      // estep_prep_kernel did these per symbol
        d0 = s_rec[0];
        cscale_d = s_rec[1];
        lb_scale = s_rec[2];
    } else {
        d0 = candidate_distance<NT, NR>(H, a.yd + (size_t)gsym * NR, s_cons, k_M, reg,
                                        reinterpret_cast<cd*>(s_tab), lane, cscale_d);
        lb_scale = column_tile_bounds<NT, NR>(H, a.yd + (size_t)gsym * NR, s_cons, k_M, k_lm,
                                              k_JB >> 4, s_lb, reinterpret_cast<cd*>(s_tab), lane);
    }
    const double lb_margin = c.prune ? 1e-9 * lb_scale : INFINITY;
    // row-tile bounds (NT = 4): lane s0 < 16 of a surviving column tile kt evaluates
    // ||Py - x_s0 Ph_0 - x_kt Ph_2||^2, a lower bound of every hypothesis with first streams
    // (s0, kt); tile groups whose four bounds all exceed the skip bound are not swept
    const bool rowb = NT == 4 && V16 && prep && c.rowb;
    // row-tile bound tables (scratch s_tab[63..111], free on the prep path): per column tile kt (= x_2 index)
    //   n_kt = ||v_kt||^2 and a_kt = (P h_0)^H v_kt, v_kt = P y - x_kt P h_2, and ||P h_0||^2,
    // so the bound of row tile s0 is n_kt - 2 Re(conj(x_s0) a_kt) + |x_s0|^2 ||P h_0||^2
    double* s_rk = s_tab + 64;       // [16][3]
    if (rowb) {
        const double* rbp = s_rec + k_rowb_off;     // [3][NR] complex: P y, P h_0, P h_2
        double n = 0.0, nb0 = 0.0;
        cd av = czero();
        if (lane < 16) {
            const cd x2 = s_cons[lane];
#pragma unroll
            for (int r = 0; r < NR; ++r) {
                const cd py = cmk(rbp[2 * r], rbp[2 * r + 1]);
                const cd p0 = cmk(rbp[2 * (NR + r)], rbp[2 * (NR + r) + 1]);
                const cd p2 = cmk(rbp[2 * (2 * NR + r)], rbp[2 * (2 * NR + r) + 1]);
                const cd v = csub(py, cmul(p2, x2));
                n += cabs2(v);
                nb0 += cabs2(p0);
                av = cfmac(av, v, p0);                 // p0^H v
            }
        }
        if (lane < 16) {
            s_rk[3 * lane] = n;
            s_rk[3 * lane + 1] = av.x;
            s_rk[3 * lane + 2] = av.y;
        }
        if (lane == 0) s_tab[63] = nb0;
        wave_sync();
    }

    // lane-level accumulators (see VALU kernel)
    // the running shift starts at a real hypothesis' distance (candidate_distance) plus a rounding
    // margin: the sweep's own distances (alpha + gamma - 2 Re p^H q) differ from d0 by rounding of
    // order eps * cscale_d, and a shift below every swept distance by more than 50 varn^2 would
    // skip every group and leave the posterior empty (0/0).  (A theta_0 ~1e13 from a near-singular
    // pinv puts that rounding at ~1e12 >> varn^2.)  The shift then falls to the true minimum.
    double mshift = d0 + 1e-10 * cscale_d;
    double tot_c = 0.0;
    cd tot_muA[NA];
    double nu[NA];
    cd kap = czero();
    cd tot_mB[NB];
    double tot_nB[NB];
    cd tot_kB = czero();
    cd tot_X[NA][NB];
#pragma unroll
    for (int q = 0; q < NA; ++q) {
        tot_muA[q] = czero(); nu[q] = 0.0;
#pragma unroll
        for (int bb = 0; bb < NB; ++bb) tot_X[q][bb] = czero();
    }
#pragma unroll
    for (int bb = 0; bb < NB; ++bb) { tot_mB[bb] = czero(); tot_nB[bb] = 0.0; }
    double best_d = d0 + 1e-10 * cscale_d + 1e-300;   // admits the argmin (rounding margin)
                                                       // (== hard_bound below)
    int best_j = 0x7fffffff;

    // U_s = -2 (y - h_0 x_s),  V_s = 2 h_1 x_s  so that  -2 p_i = U_{s0(i)} + V_{s1(i)}
    // (NA == 1: -2 p_i = U_{i}).  Layout [kk][s]: conflict-free per-lane reads.
    {
        wave_sync();
        for (int e = lane; e < k_M * 4 * STEPS; e += 64) {
            const int kk = e >> k_lm, sx = e & mask;
            double u = 0.0, v = 0.0, q2 = 0.0;
            if (kk < K2) {
                const int r = kk >> 1;
                const cd x = s_cons[sx];
                const cd yv = prep ? reinterpret_cast<const cd*>(s_rec + k_prep_stride)[r]
                                   : a.yd[(size_t)gsym * NR + r];
                const cd pu = csub(yv, cmul(H[0 * NR + r], x));
                u = -2.0 * ((kk & 1) ? pu.y : pu.x);
                if (NA == 2) {
                    const cd hv = cmul(H[1 * NR + r], x);
                    v = 2.0 * ((kk & 1) ? hv.y : hv.x);
                }
                if (V16) {
                    const cd hq = cmul(H[NA * NR + r], x);
                    q2 = (kk & 1) ? hq.y : hq.x;
                }
            }
            s_U[e] = u;
            if (NA == 2) s_V[e] = v;
            if (V16) {
                s_Q2[e] = q2;
                s_U32[e] = (float)u;
            }
        }
        wave_sync();
    }
    const int col = lane & 15;
    const int rq = lane >> 4;
    // V16: hoisted A-operand V term, and the B operand q_k = h_NA x_kt + h_NA+1 x_col split
    // into a per-kt LDS row (s_Q2) plus a lane constant (q3reg)
    double vreg[STEPS], q3reg[STEPS];
    float vreg32[STEPS];
#pragma unroll
    for (int s = 0; s < STEPS; ++s) {
        const int kk = 4 * s + rq;
        vreg[s] = V16 ? s_V[kk * 16 + col] : 0.0;
        vreg32[s] = (float)vreg[s];
        double q3 = 0.0;
        if (V16 && kk < K2) {
            const cd hx = cmul(H[(NA + 1) * NR + (kk >> 1)], s_cons[col]);
            q3 = (kk & 1) ? hx.y : hx.x;
        }
        q3reg[s] = q3;
    }
    const int xaddr16 = (lane ^ 16) << 2, xaddr32 = (lane ^ 32) << 2;
    const int nktile = k_JB >> 4;
    const int ntile_chunk = k_chunk >> 4;
    bool table_ready = false;
    // FP32 screen (V16): a tile group's distances first by FP32 MFMAs (v_mfma_f32_16x16x4f32,
    // a third of the FP64 instruction's cycles); the FP64 group runs only if some entry can be
    // within the skip bound.  |d32 - d| <= 2^-17 (2 max_i alpha_i + gamma_k) (rounding of the
    // operands and of K2 + 1 f32 sums, |sum_kk P' Q| <= 2 |p_i||q_k| <= alpha_i + gamma_k), so
    // a screened-out group is one the FP64 test below would discard too: results are bitwise
    // those of the unscreened sweep.  A symbol whose groups mostly pass (wide posterior) stops
    // screening after 16 groups.
    double amax = 0.0;               // max_i alpha_i (set with the alpha table)
    bool scr_on = V16 && c.screen;   // wave-uniform
    int scr_n = 0, scr_pass = 0;

    const double hard_bound = d0 + 1e-10 * cscale_d + 1e-300;
    unsigned groups = 0;             // wave-uniform count of issued tile groups
    // column tiles whose exact bound (column_tile_bounds) admits the skip bound as it stands
    // now; the bound only falls during the sweep, so each is checked again when reached
    unsigned long long ktmask = ~0ull;
    if (nktile <= 64) {
        const double lim0 = ((MODE == SBCE_ESTEP_HARD) ? hard_bound : mshift + thr_d) + lb_margin;
        ktmask = __ballot(lane < nktile && !(lbp[lane < nktile ? lane : 0] > lim0));
    }
    for (int kt = 0; kt < nktile; ++kt) {
        if (nktile <= 64) {
            const unsigned long long m = ktmask >> kt;
            if (!m) break;
            kt += __builtin_ctzll(m);
        }
        // exact column-tile bound: wave-uniform skip of the whole tile
        if (lbp[kt] > ((MODE == SBCE_ESTEP_HARD) ? hard_bound : mshift + thr_d) + lb_margin)
            continue;
        unsigned rowmask = 0xffffu;
        if (rowb) {
            double bnd = INFINITY;
            if (lane < 16) {
                const cd x0 = s_cons[lane];
                const double* rk = s_rk + 3 * kt;
                bnd = fma(cabs2(x0), s_tab[63], rk[0] - 2.0 * (x0.x * rk[1] + x0.y * rk[2]));
            }
            const double lim = ((MODE == SBCE_ESTEP_HARD) ? hard_bound : mshift + thr_d) + lb_margin;
            rowmask = (unsigned)__ballot(bnd <= lim);
            if (!rowmask) continue;                      // no row tile of this column survives
        }
        const int k = kt * 16 + col;
        cd xb[NB];
#pragma unroll
        for (int bb = 0; bb < NB; ++bb) xb[bb] = s_cons[(k >> (k_lm * (NB - 1 - bb))) & mask];
        double bop[STEPS];
        float bop32[STEPS];
        double gam = 0.0;
        if constexpr (V16) {
            // gamma_k = ||q_k||^2 = sum over the 4 lanes of column k of their bop^2
#pragma unroll
            for (int s = 0; s < STEPS; ++s) {
                bop[s] = s_Q2[(4 * s + rq) * 16 + kt] + q3reg[s];
                gam = fma(bop[s], bop[s], gam);
            }
            gam += bperm_d(gam, xaddr16);
            gam += bperm_d(gam, xaddr32);
#pragma unroll
            for (int s = 0; s < STEPS; ++s) bop32[s] = (float)bop[s];
        } else {
            cd qv[NR];
#pragma unroll
            for (int r = 0; r < NR; ++r) {
                cd acc = czero();
#pragma unroll
                for (int bb = 0; bb < NB; ++bb) acc = cfma(acc, H[(NA + bb) * NR + r], xb[bb]);
                qv[r] = acc;
                gam += cabs2(acc);
            }
#pragma unroll
            for (int s = 0; s < STEPS; ++s) {
                const int kk = 4 * s + rq;
                double v = 0.0;
#pragma unroll
                for (int r = 0; r < NR; ++r) {
                    if (kk == 2 * r) v = qv[r].x;
                    if (kk == 2 * r + 1) v = qv[r].y;
                }
                bop[s] = v;
            }
        }
        double ck = 0.0;
        cd mu[NA];
#pragma unroll
        for (int q = 0; q < NA; ++q) mu[q] = czero();
        bool touched = false;       // wave-uniform: an exp was taken in this column tile
        // V16 (NA = 2): hypothesis i = 16 s0 + s1 with s0 = the tile (wave-uniform per tile) and
        // s1 = rq + 4 j (the lane's row j), so the per-column-tile sums factor: R1[j] = sum over
        // tiles of w (-> ck, mu_1, nu_1), Q[j] = sum of w x_s0 (-> mu_0, and kappa through
        // conj(x_s1)), N0 = sum of w |x_s0|^2 (-> nu_0); 4 VALU ops per weight instead of 21,
        // the x_s1 products once per column tile
        double R1[4] = {0.0, 0.0, 0.0, 0.0}, N0 = 0.0;
        cd Q[4] = {czero(), czero(), czero(), czero()};

        for (int i0 = 0; i0 < k_JA; i0 += k_chunk) {
            if (!table_ready && V16) {
                // ---- alpha[s0*16 + s1] = 0.25 ||U_s0 + V_s1||^2
                //      = 0.25 (|U_s0|^2 + |V_s1|^2) + 0.5 U_s0 . V_s1: the cross terms are a
                //      16 x 16 x K2 real GEMM (STEPS MFMAs, B operand = vreg); stored as
                //      s_al[s0*16 + (s1 & 3)*4 + (s1 >> 2)] so that a tile's accumulator init
                //      (rows rq + 4j) is two 16-byte reads ----
                wave_sync();
                double nrm = 0.0;
                const double* T = lane < 16 ? s_U : s_V;
#pragma unroll
                for (int kk = 0; kk < K2; ++kk) {
                    const double v = T[kk * 16 + (lane & 15)];
                    nrm = fma(v, v, nrm);
                }
                if (lane < 32) s_tab[lane] = nrm;
                d4v cx = {0.0, 0.0, 0.0, 0.0};
#pragma unroll
                for (int s = 0; s < STEPS; ++s)
                    cx = __builtin_amdgcn_mfma_f64_16x16x4f64(s_U[(4 * s + rq) * 16 + col], vreg[s],
                                                              cx, 0, 0, 0);
                wave_sync();
                const double nvv = s_tab[16 + col];
                double am = 0.0;
#pragma unroll
                for (int j = 0; j < 4; ++j) {
                    const int s0 = rq + 4 * j;
                    const double al = 0.25 * (s_tab[s0] + nvv) + 0.5 * cx[j];
                    s_al[s0 * 16 + (col & 3) * 4 + (col >> 2)] = al;
                    s_al32[s0 * 16 + col] = (float)al;     // natural order: f32 C/D rows 4 rq + q
                    am = fmax(am, al);
                }
                amax = wave_max_dpp(am);
                wave_sync();
                table_ready = true;
            }
            if (!table_ready) {
                // ---- alpha_i = ||p_i||^2 for entries i0 .. i0+chunk-1 from U, V ----
                wave_sync();
                for (int e = lane; e < k_chunk; e += 64) {
                    const int i = i0 + e;
                    const int su = (NA == 2) ? (i >> k_lm) : i;
                    const int sv = i & mask;
                    double al = 0.0;
#pragma unroll
                    for (int kk = 0; kk < K2; ++kk) {
                        double v = s_U[kk * k_M + su];
                        if (NA == 2) v += s_V[kk * k_M + sv];
                        al = fma(v, v, al);
                    }
                    s_al[e] = 0.25 * al;
                }
                wave_sync();
                table_ready = (k_JA == k_chunk);
            }
            for (int tg = 0; tg < ntile_chunk; tg += TU) {
                // TU independent 16x16 tiles in flight: STEPS*TU MFMAs per group;
                // accumulators start at alpha_i, gamma_k (lane constant) stays outside
                if (V16 && !((rowmask >> tg) & ((1u << TU) - 1u))) continue;
                if (V16 && scr_on) {
                    f4v s32[TU];
#pragma unroll
                    for (int u = 0; u < TU; ++u)
                        s32[u] = *reinterpret_cast<const f4v*>(s_al32 + (tg + u) * 16 + rq * 4);
#pragma unroll
                    for (int s = 0; s < STEPS; ++s)
#pragma unroll
                        for (int u = 0; u < TU; ++u) {
                            const float av = s_U32[(4 * s + rq) * 16 + (i0 >> 4) + tg + u] + vreg32[s];
                            s32[u] = __builtin_amdgcn_mfma_f32_16x16x4f32(av, bop32[s], s32[u], 0, 0, 0);
                        }
                    float m32 = fminf(fminf(s32[0][0], s32[0][1]), fminf(s32[0][2], s32[0][3]));
#pragma unroll
                    for (int u = 1; u < TU; ++u)
                        m32 = fminf(m32, fminf(fminf(s32[u][0], s32[u][1]), fminf(s32[u][2], s32[u][3])));
                    const double lim = ((MODE == SBCE_ESTEP_HARD) ? best_d : mshift + thr_d) - gam +
                                       0x1p-17 * (2.0 * amax + gam);
                    ++scr_n;
                    const bool pass = __any((double)m32 <= lim);
                    scr_pass += pass;
                    if (scr_n >= 16 && 2 * scr_pass > scr_n) scr_on = false;
                    if (!pass) continue;
                }
                ++groups;
                d4v acc[TU];
#pragma unroll
                for (int u = 0; u < TU; ++u) {
                    if (V16) {            // rows rq + 4j of tile tg + u: 4 consecutive doubles
                        const cd lo = *reinterpret_cast<const cd*>(s_al + (tg + u) * 16 + rq * 4);
                        const cd hi = *reinterpret_cast<const cd*>(s_al + (tg + u) * 16 + rq * 4 + 2);
                        acc[u] = d4v{lo.x, lo.y, hi.x, hi.y};
                    } else {
#pragma unroll
                        for (int j = 0; j < 4; ++j) acc[u][j] = s_al[(tg + u) * 16 + rq + 4 * j];
                    }
                }
#pragma unroll
                for (int s = 0; s < STEPS; ++s)
#pragma unroll
                    for (int u = 0; u < TU; ++u) {
                        const int kk = 4 * s + rq;
                        double av;
                        if (V16) {
                            av = s_U[kk * 16 + (i0 >> 4) + tg + u] + vreg[s];
                        } else {
                            const int ia = i0 + (tg + u) * 16 + col;      // A-operand row
                            av = s_U[kk * k_M + ((NA == 2) ? (ia >> k_lm) : ia)];
                            if (NA == 2) av += s_V[kk * k_M + (ia & mask)];
                        }
                        acc[u] = __builtin_amdgcn_mfma_f64_16x16x4f64(av, bop[s], acc[u], 0, 0, 0);
                    }
                double cm = fmin(fmin(acc[0][0], acc[0][1]), fmin(acc[0][2], acc[0][3]));
#pragma unroll
                for (int u = 1; u < TU; ++u)
                    cm = fmin(cm, fmin(fmin(acc[u][0], acc[u][1]), fmin(acc[u][2], acc[u][3])));
                // one comparison per tile group (soft: within thr of the shift, hard: not
                // worse than this lane's best); the common case skips everything below
                if (MODE == SBCE_ESTEP_HARD) {
                    if (!__any(cm + gam <= best_d)) continue;
                } else if (!__any(cm + gam <= mshift + thr_d)) {
                    continue;
                }
                if (MODE == SBCE_ESTEP_HARD) {
                    const double lim = best_d - gam;
#pragma unroll
                    for (int u = 0; u < TU; ++u)
#pragma unroll
                        for (int j = 0; j < 4; ++j) {
                            const double dv = acc[u][j];
                            if (dv <= lim) {
                                const int jj = (i0 + (tg + u) * 16 + rq + 4 * j) * k_JB + k;
                                const double dd = dv + gam;
                                if (dd < best_d || (dd == best_d && jj < best_j)) { best_d = dd; best_j = jj; }
                            }
                        }
                    continue;
                }
                cm += gam;
                if (__any(cm < mshift)) {
                    double mn = fmin(cm, mshift);
                    mn = wave_min_dpp(mn);
                    const double f = fexp_neg((mn - mshift) * inv_s2);
                    mshift = mn;
                    // V16: ck, mu are formed at the column tile's end; the stream-3 totals
                    // (x_3 = cons[col], a lane constant) are formed after the sweep
                    constexpr int NBS = V16 ? 1 : NB;
                    tot_c *= f; kap = cscale(kap, f);
                    if constexpr (!V16) { ck *= f; tot_kB = cscale(tot_kB, f); }
#pragma unroll
                    for (int q = 0; q < NA; ++q) {
                        tot_muA[q] = cscale(tot_muA[q], f); nu[q] *= f;
                        if constexpr (!V16) mu[q] = cscale(mu[q], f);
#pragma unroll
                        for (int bb = 0; bb < NBS; ++bb) tot_X[q][bb] = cscale(tot_X[q][bb], f);
                    }
#pragma unroll
                    for (int bb = 0; bb < NBS; ++bb) { tot_mB[bb] = cscale(tot_mB[bb], f); tot_nB[bb] *= f; }
                    if constexpr (V16) {
                        N0 *= f;
#pragma unroll
                        for (int j = 0; j < 4; ++j) { R1[j] *= f; Q[j] = cscale(Q[j], f); }
                    }
                }
                if (!__any(cm <= mshift + thr_d)) continue;
                touched = true;
#pragma unroll
                for (int u = 0; u < TU; ++u) {
                    const double cmu =
                        fmin(fmin(acc[u][0], acc[u][1]), fmin(acc[u][2], acc[u][3])) + gam;
                    if (!__any(cmu <= mshift + thr_d)) continue;
                    if constexpr (V16) {
                        const cd x0 = s_cons[tg + u];          // stream 0 of the tile (i0 = 0)
                        const double n0 = cabs2(x0);
#pragma unroll
                        for (int j = 0; j < 4; ++j) {
                            const double dj = acc[u][j] + gam;
                            // rows with no lane inside the bound: weights < e^-50 of the maximum
                            if (!__any(dj <= mshift + thr_d)) continue;
                            const double w = fexp_neg((mshift - dj) * inv_s2);
                            R1[j] += w;
                            Q[j] = caxpy(Q[j], w, x0);
                            N0 = fma(w, n0, N0);
                        }
                        continue;
                    }
#pragma unroll
                    for (int j = 0; j < 4; ++j) {
                        const int i = i0 + (tg + u) * 16 + rq + 4 * j;
                        const double w = fexp_neg((mshift - (acc[u][j] + gam)) * inv_s2);
                        cd xa[NA];
#pragma unroll
                        for (int q = 0; q < NA; ++q) xa[q] = s_cons[(i >> (k_lm * (NA - 1 - q))) & mask];
                        ck += w;
#pragma unroll
                        for (int q = 0; q < NA; ++q) {
                            mu[q] = caxpy(mu[q], w, xa[q]);
                            nu[q] = fma(w, cabs2(xa[q]), nu[q]);
                        }
                        if (NPA) kap = caxpy(kap, w, cmulc(xa[0], xa[NA > 1 ? 1 : 0]));
                    }
                }
            }
        }
        if (MODE == SBCE_ESTEP_SOFT && touched) {
            if constexpr (V16) {
                // the lane's row streams x_s1 = cons[rq + 4 j]
                ck = (R1[0] + R1[1]) + (R1[2] + R1[3]);
                mu[0] = cadd(cadd(Q[0], Q[1]), cadd(Q[2], Q[3]));
                mu[1] = czero();
                nu[0] += N0;
#pragma unroll
                for (int j = 0; j < 4; ++j) {
                    const cd x1 = s_cons[rq + 4 * j];
                    mu[1] = caxpy(mu[1], R1[j], x1);
                    nu[1] = fma(R1[j], cabs2(x1), nu[1]);
                    kap = cadd(kap, cmulc(Q[j], x1));
                }
            }
            constexpr int NBS = V16 ? 1 : NB;
            tot_c += ck;
#pragma unroll
            for (int bb = 0; bb < NBS; ++bb) {
                tot_mB[bb] = caxpy(tot_mB[bb], ck, xb[bb]);
                tot_nB[bb] = fma(ck, cabs2(xb[bb]), tot_nB[bb]);
            }
            if (NPB && !V16) tot_kB = caxpy(tot_kB, ck, cmulc(xb[0], xb[NB > 1 ? 1 : 0]));
#pragma unroll
            for (int q = 0; q < NA; ++q) {
                tot_muA[q] = cadd(tot_muA[q], mu[q]);
#pragma unroll
                for (int bb = 0; bb < NBS; ++bb) tot_X[q][bb] = cfmac(tot_X[q][bb], mu[q], xb[bb]);
            }
        }
    }
    if constexpr (V16) {
        // stream 3 is the lane constant x_3 = cons[col] (k = 16 kt + col): its sums are the
        // lane's totals times x_3
        const cd x3 = s_cons[col];
        tot_mB[1] = cscale(x3, tot_c);
        tot_nB[1] = tot_c * cabs2(x3);
        tot_kB = cmulc(tot_mB[0], x3);
#pragma unroll
        for (int q = 0; q < NA; ++q) tot_X[q][1] = cmulc(tot_muA[q], x3);
    }

    if (c.count && lane == 0) atomicAdd(&g_estep_mfma, (unsigned long long)groups * STEPS * TU);
    constexpr int MS = NT + NT * NT;
    cd* out = a.mom + (size_t)gsym * MS;
    if (MODE == SBCE_ESTEP_HARD) {
        wave_argmin_dpp(best_d, best_j);
        if (lane == 0) {
            cd x[NT];
#pragma unroll
            for (int s2 = 0; s2 < NT; ++s2) x[s2] = s_cons[(best_j >> (k_lm * (NT - 1 - s2))) & mask];
#pragma unroll
            for (int s2 = 0; s2 < NT; ++s2) {
                out[s2] = x[s2];
#pragma unroll
                for (int s3 = 0; s3 < NT; ++s3) out[NT + s2 * NT + s3] = cmulc(x[s2], x[s3]);
            }
        }
        return;
    }
    int xa[6];
#pragma unroll
    for (int i = 0; i < 6; ++i) xa[i] = (lane ^ (32 >> i)) << 2;
    {
        // Reduce-scatter by recursive halving: at the step with lane offset o a lane keeps the
        // half of the remaining values selected by its bit o and receives the partner's copy
        // of that half (32 + 16 + ... doubles moved instead of 6 per value); value j ends in
        // the lanes whose bits 5..1 spell j, and is gathered through LDS.
        constexpr int NV = 1 + 2 * NPA + 2 * NPB + 3 * NA + 2 * NA * NB + 3 * NB;
        static_assert(NV <= 32, "reduce-scatter holds at most 32 values");
        double v[32];
        int n = 0;
        auto put = [&](double x) { v[n++] = x; };
        put(tot_c);
        if (NPA) { put(kap.x); put(kap.y); }
        if (NPB) { put(tot_kB.x); put(tot_kB.y); }
#pragma unroll
        for (int q = 0; q < NA; ++q) {
            put(tot_muA[q].x); put(tot_muA[q].y); put(nu[q]);
#pragma unroll
            for (int bb = 0; bb < NB; ++bb) { put(tot_X[q][bb].x); put(tot_X[q][bb].y); }
        }
#pragma unroll
        for (int bb = 0; bb < NB; ++bb) { put(tot_mB[bb].x); put(tot_mB[bb].y); put(tot_nB[bb]); }
#pragma unroll
        for (int i = NV; i < 32; ++i) v[i] = 0.0;
#pragma unroll
        for (int st = 0; st < 5; ++st) {
            const int h = 16 >> st;
            const bool hi = (lane >> (5 - st)) & 1;
#pragma unroll
            for (int i = 0; i < h; ++i) {
                const double snd = hi ? v[i] : v[h + i];
                const double kp = hi ? v[h + i] : v[i];
                v[i] = kp + bperm_d(snd, xa[st]);
            }
        }
        v[0] += bperm_d(v[0], xa[5]);
        double* red = s_tab;                 // wave scratch (>= 32 doubles)
        const int j = ((lane >> 5) & 1) * 16 + ((lane >> 4) & 1) * 8 + ((lane >> 3) & 1) * 4 +
                      ((lane >> 2) & 1) * 2 + ((lane >> 1) & 1);
        wave_sync();
        if (!(lane & 1)) red[j] = v[0];
        wave_sync();
        // lane o < NT + NT^2 writes output o (m_t, then S_t row-major) from the gathered
        // totals: numerator at red[ire] (+ i red[iim]), conjugated when cj, times 1/Z
        if (lane < NT + NT * NT) {
            constexpr int OFF_KA = 1, OFF_KB = 1 + 2 * NPA;
            constexpr int BQ = 1 + 2 * NPA + 2 * NPB, SQ = 3 + 2 * NB;
            constexpr int BB = BQ + NA * SQ;
            int ire, iim = -1;
            bool cj = false;
            if (lane < NT) {
                ire = lane < NA ? BQ + lane * SQ : BB + 3 * (lane - NA);
                iim = ire + 1;
            } else {
                const int i = (lane - NT) / NT, j = (lane - NT) - (lane - NT) / NT * NT;
                if (i == j) {
                    ire = i < NA ? BQ + i * SQ + 2 : BB + 3 * (i - NA) + 2;
                } else if (i < NA && j < NA) {
                    ire = OFF_KA; iim = OFF_KA + 1; cj = i > j;
                } else if (i >= NA && j >= NA) {
                    ire = OFF_KB; iim = OFF_KB + 1; cj = i > j;
                } else if (i < NA) {
                    ire = BQ + i * SQ + 3 + 2 * (j - NA); iim = ire + 1;
                } else {
                    ire = BQ + j * SQ + 3 + 2 * (i - NA); iim = ire + 1; cj = true;
                }
            }
            const double iz = 1.0 / red[0];
            const double re = red[ire], im = iim >= 0 ? red[iim] : 0.0;
            out[lane] = cmk(re * iz, (cj ? -im : im) * iz);
        }
    }
    }();
    }
    if (!listed) return;
    }
}

// ============================================================================
// Per-symbol preparation pass (one THREAD per symbol) for the MFMA sweep: H_eff(t), the
// candidate bound of candidate_distance and the column-tile bounds of column_tile_bounds,
// written to the workspace (PrepLayout).  These are short dependent chains (a 4 x 4
// Cholesky, a Gram-Schmidt, M-way minima): inside the sweep kernel one wave would run
// them serially per symbol; here 64 symbols run them side by side per wave.
// ============================================================================
struct PrepConst {
    int B, Td, P, M, lm, nkt, stride;
    int uni;           // wave-uniform theta loads (SBCE_PREP_UNI=0 disables: A/B runs)
    double reg;
    // sphere pass (estep_sphere_kernel; EstepArgs::list receives the symbols it leaves)
    int budget;        // DFS steps per symbol before the symbol is left to the sweep
    int count;         // SBCE_ESTEP_COUNT=1: tally resolved / listed symbols (g_estep_sphere)
    int hard;          // hard (argmin) E-step: sphere radius without the soft threshold
    int pair;          // route wide-tree symbols that pass the screen to the factorised pass
    double inv_s2, thr_d;
};

// Diagnostic (SBCE_ESTEP_COUNT=1): symbols the sphere pass's enumeration resolved, symbols it
// left to the MFMA sweep, and symbols the tree pass resolved alone (single surviving path).
__device__ unsigned long long g_estep_sphere[3];

// ---- H_eff(t) = sum_p psi_p H_p (theta of the symbol's trial, psi of the symbol) ----
template <int NT, int NR>
__device__ __forceinline__ void heff_load(const EstepArgs& a, const PrepConst& c, long gsym, int b,
                                          cd (&H)[NT][NR]) {
    constexpr int NO = NT * NR;
#pragma unroll
    for (int q = 0; q < NT; ++q)
#pragma unroll
        for (int r = 0; r < NR; ++r) H[q][r] = czero();
    const cd* ps = a.psid + (size_t)gsym * c.P;
    // the wave's 64 symbols normally belong to one trial: theta's address is then
    // wave-uniform and its loads go through the scalar cache (one vector load per p)
    const int b0 = __builtin_amdgcn_readfirstlane(b);
    if (c.uni && __all(b == b0)) {
        const cd* th = a.theta + (size_t)b0 * c.P * NO;
#pragma unroll 8
        for (int p = 0; p < c.P; ++p) {
            const cd psi = ps[p];
#pragma unroll
            for (int q = 0; q < NT; ++q)
#pragma unroll
                for (int r = 0; r < NR; ++r) H[q][r] = cfma(H[q][r], psi, th[p * NO + q * NR + r]);
        }
    } else {
        const cd* th = a.theta + (size_t)b * c.P * NO;
        for (int p = 0; p < c.P; ++p) {
            const cd psi = ps[p];
#pragma unroll
            for (int q = 0; q < NT; ++q)
#pragma unroll
                for (int r = 0; r < NR; ++r) H[q][r] = cfma(H[q][r], psi, th[p * NO + q * NR + r]);
        }
    }
}

// Ridge Cholesky G + reg I = L L^H of G = H^H H (L strictly lower in Lm, pivots piv,
// 1/sqrt(pivots) dinv) and zf = L^-1 H^H y.
template <int NT, int NR>
__device__ __forceinline__ void ridge_chol(const cd (&H)[NT][NR], const cd (&y)[NR], double reg,
                                           cd (&Lm)[NT][NT], double (&piv)[NT], double (&dinv)[NT],
                                           cd (&zf)[NT]) {
#pragma unroll
    for (int j = 0; j < NT; ++j) {
        cd gjj = czero();
#pragma unroll
        for (int r = 0; r < NR; ++r) gjj = cfmac(gjj, H[j][r], H[j][r]);
        double d = gjj.x + reg;
#pragma unroll
        for (int k = 0; k < j; ++k) d -= cabs2(Lm[j][k]);
        piv[j] = fmax(d, 1e-300);
        const double inv = fast_rsqrt(piv[j]);
        dinv[j] = inv;
#pragma unroll
        for (int i = j + 1; i < NT; ++i) {
            cd s = czero();
#pragma unroll
            for (int r = 0; r < NR; ++r) s = cfmac(s, H[j][r], H[i][r]);   // G[i][j]
#pragma unroll
            for (int k = 0; k < j; ++k) s = csub(s, cmulc(Lm[i][k], Lm[j][k]));
            Lm[i][j] = cscale(s, inv);
        }
    }
#pragma unroll
    for (int i = 0; i < NT; ++i) {
        cd s = czero();
#pragma unroll
        for (int r = 0; r < NR; ++r) s = cfmac(s, y[r], H[i][r]);          // (H^H y)_i
#pragma unroll
        for (int k = 0; k < i; ++k) s = csub(s, cmul(Lm[i][k], zf[k]));
        zf[i] = cscale(s, dinv[i]);
    }
}

// Candidate of candidate_distance (same arithmetic order): quantised ridge LS estimate from
// the factorisation above; returns its distance d0 and the magnitude scale sc.
template <int NT, int NR>
__device__ __forceinline__ double prep_candidate(const cd (&H)[NT][NR], const cd (&y)[NR],
                                                 const cd (&Lm)[NT][NT], const double (&dinv)[NT],
                                                 const cd (&zf)[NT], const cd* cons, int M,
                                                 double& sc, int& xidx) {
    cd x[NT];
    xidx = 0;
    cd z[NT];
#pragma unroll
    for (int i = 0; i < NT; ++i) z[i] = zf[i];
#pragma unroll
    for (int i = NT - 1; i >= 0; --i) {
        cd s = z[i];
#pragma unroll
        for (int k = i + 1; k < NT; ++k) s = csub(s, cmul(cconj(Lm[k][i]), z[k]));
        z[i] = cscale(s, dinv[i]);
    }
#pragma unroll
    for (int q = 0; q < NT; ++q) {
        double bd = INFINITY;
        int bs = 0;
        #pragma unroll 4
        for (int s = 0; s < M; ++s) {
            const double dd = cabs2(csub(z[q], cons[s]));
            if (dd < bd) { bd = dd; bs = s; }
        }
        x[q] = cons[bs];
        xidx |= bs << (8 * q);
    }
    double d0 = 0.0;
    sc = 0.0;
#pragma unroll
    for (int r = 0; r < NR; ++r) {
        cd res = y[r];
        sc += cabs2(res);
#pragma unroll
        for (int q = 0; q < NT; ++q) {
            const cd hx = cmul(H[q][r], x[q]);
            res = csub(res, hx);
            sc += NT * cabs2(hx);
        }
        d0 += cabs2(res);
    }
    return d0;
}

// Screen of the factorised-weight pass (estep_pair.hip), NT = 4: an UPPER bound of its range
// D = sum_f (max f - f(x_c)) over the six log tables, from the candidate x_c alone:
//   max A <= 0                        ->  A term <= ||y - h_0 x_c0 - h_1 x_c1||^2 / s2,
//   max B <= ||y||^2 / s2             ->  B term <= ||y - h_2 x_c2 - h_3 x_c3||^2 / s2,
//   max E_ab <= 2 |h_a^H h_b| max|c|^2 / s2.
// The enumeration routes a symbol it gives up on to the pass only when this bound is within the
// pass's limit, so the pass never has to hand a symbol back.
// Returns the x_c-dependent part (in units of 1/s2) and sets gsum >= sum_ab 2 |h_a^H h_b|, the
// coefficient of max|c|^2 (known after the Babai descent): D <= (part + gsum max|c|^2) / s2.
template <int NT, int NR>
__device__ __forceinline__ double pair_screen(const cd (&H)[NT][NR], const cd (&y)[NR], int xidx,
                                              const cd* cons, double& gsum) {
    gsum = 0.0;
    if constexpr (NT != 4) {
        return INFINITY;
    } else {
        cd x[NT];
#pragma unroll
        for (int q = 0; q < NT; ++q) x[q] = cons[(xidx >> (8 * q)) & 255];
        double na = 0.0, nb = 0.0;
#pragma unroll
        for (int r = 0; r < NR; ++r) {
            na += cabs2(csub(csub(y[r], cmul(H[0][r], x[0])), cmul(H[1][r], x[1])));
            nb += cabs2(csub(csub(y[r], cmul(H[2][r], x[2])), cmul(H[3][r], x[3])));
        }
        double up = na + nb;
#pragma unroll
        for (int a0 = 0; a0 < 2; ++a0)
#pragma unroll
            for (int b0 = 2; b0 < 4; ++b0) {
                cd G = czero();
#pragma unroll
                for (int r = 0; r < NR; ++r) G = cfmac(G, H[b0][r], H[a0][r]);    // h_a^H h_b
                const cd t = cmul(G, x[b0]);
                gsum += 2.0 * (fabs(G.x) + fabs(G.y));                      // >= 2 |G|
                up += 2.0 * fma(x[a0].x, t.x, x[a0].y * t.y);               // -E_ab(x_c) s2
            }
        return up;
    }
}

// NT = 2, square QAM (estep_pair.hip estep_fact2_kernel): D = (sum of the eight log-table maxima)
// - l(x_c), both times 1/s2, with x_c the prep candidate (a real hypothesis: l(x_c) <= max l).  The
// 1-D tables' maxima over the constellation's real / imaginary parts, the bilinear ones at the
// corners of the level box.  The factorised pass represents every weight within e^-50 of the
// largest as a normal double when D <= kPairDmax.
template <int NR>
__device__ __forceinline__ double fact2_bound(const cd (&H)[2][NR], const cd (&y)[NR], int xidx,
                                              const cd* cons, int M, double inv_s2) {
    cd z0 = czero(), z1 = czero(), g = czero();
    double g00 = 0.0, g11 = 0.0;
#pragma unroll
    for (int r = 0; r < NR; ++r) {
        z0 = cfmac(z0, y[r], H[0][r]);
        z1 = cfmac(z1, y[r], H[1][r]);
        g = cfmac(g, H[1][r], H[0][r]);
        g00 += cabs2(H[0][r]);
        g11 += cabs2(H[1][r]);
    }
    double fa0 = -INFINITY, fb0 = -INFINITY, fa1 = -INFINITY, fb1 = -INFINITY;
    double amin = INFINITY, amax = -INFINITY, bmin = INFINITY, bmax = -INFINITY;
    for (int s = 0; s < M; ++s) {
        const double av = cons[s].x, bv = cons[s].y;
        fa0 = fmax(fa0, 2.0 * av * z0.x - g00 * av * av);
        fb0 = fmax(fb0, 2.0 * bv * z0.y - g00 * bv * bv);
        fa1 = fmax(fa1, 2.0 * av * z1.x - g11 * av * av);
        fb1 = fmax(fb1, 2.0 * bv * z1.y - g11 * bv * bv);
        amin = fmin(amin, av); amax = fmax(amax, av);
        bmin = fmin(bmin, bv); bmax = fmax(bmax, bv);
    }
    auto corner = [](double k, double u0, double u1, double v0, double v1) {
        return fmax(fmax(k * u0 * v0, k * u0 * v1), fmax(k * u1 * v0, k * u1 * v1));
    };
    const double tmax = corner(-2.0 * g.x, amin, amax, amin, amax) + corner(2.0 * g.y, amin, amax, bmin, bmax) +
                        corner(-2.0 * g.y, bmin, bmax, amin, amax) + corner(-2.0 * g.x, bmin, bmax, bmin, bmax);
    const cd x0 = cons[xidx & 255], x1 = cons[(xidx >> 8) & 255];
    const double lc = 2.0 * (x0.x * z0.x + x0.y * z0.y) - g00 * cabs2(x0) + 2.0 * (x1.x * z1.x + x1.y * z1.y) -
                      g11 * cabs2(x1) -
                      2.0 * (x0.x * x1.x * g.x - x0.x * x1.y * g.y + x0.y * x1.x * g.y + x0.y * x1.y * g.x);
    return (fa0 + fb0 + fa1 + fb1 + tmax - lc) * inv_s2;
}

// Column-tile bounds (column_tile_bounds) and, for NT = 4, the row-tile bound vectors of
// one symbol into its prep record `out`.
template <int NT, int NR>
__device__ __forceinline__ void prep_bounds(const cd (&H)[NT][NR], const cd (&y)[NR], double* out,
                                            const cd* cons, const PrepConst& c) {
    constexpr int NA = NT / 2, NB = NT - NA, NO = NT * NR;
    const int mask = c.M - 1;
    // ---- column-tile bounds (column_tile_bounds) ----
    {
        cd u[NA][NR];
        bool ok = true;
#pragma unroll
        for (int q = 0; q < NA; ++q) {
            cd v[NR];
            double h2 = 0.0;
#pragma unroll
            for (int r = 0; r < NR; ++r) { v[r] = H[q][r]; h2 += cabs2(v[r]); }
#pragma unroll
            for (int rep = 0; rep < 2; ++rep)
#pragma unroll
                for (int j = 0; j < q; ++j) {
                    cd pj = czero();
#pragma unroll
                    for (int r = 0; r < NR; ++r) pj = cfmac(pj, v[r], u[j][r]);   // u_j^H v
#pragma unroll
                    for (int r = 0; r < NR; ++r) v[r] = csub(v[r], cmul(u[j][r], pj));
                }
            double n2 = 0.0;
#pragma unroll
            for (int r = 0; r < NR; ++r) n2 += cabs2(v[r]);
            ok = ok && h2 > 0.0 && n2 > 1e-6 * h2;
            const double inv = ok ? fast_rsqrt(n2) : 0.0;
#pragma unroll
            for (int r = 0; r < NR; ++r) u[q][r] = cscale(v[r], inv);
        }
        cd w[NR], g[NB][NR];
        double sc = 0.0, g2 = 0.0;
#pragma unroll
        for (int r = 0; r < NR; ++r) { w[r] = y[r]; sc += cabs2(y[r]); }
#pragma unroll
        for (int bb = 0; bb < NB; ++bb)
#pragma unroll
            for (int r = 0; r < NR; ++r) { g[bb][r] = H[NA + bb][r]; g2 += cabs2(g[bb][r]); }
#pragma unroll
        for (int j = 0; j < NA; ++j) {
            cd pw = czero(), pg[NB];
#pragma unroll
            for (int bb = 0; bb < NB; ++bb) pg[bb] = czero();
#pragma unroll
            for (int r = 0; r < NR; ++r) {
                pw = cfmac(pw, w[r], u[j][r]);
#pragma unroll
                for (int bb = 0; bb < NB; ++bb) pg[bb] = cfmac(pg[bb], g[bb][r], u[j][r]);
            }
#pragma unroll
            for (int r = 0; r < NR; ++r) {
                w[r] = csub(w[r], cmul(u[j][r], pw));
#pragma unroll
                for (int bb = 0; bb < NB; ++bb) g[bb][r] = csub(g[bb][r], cmul(u[j][r], pg[bb]));
            }
        }
        double cmax2 = 0.0;
        for (int s = 0; s < c.M; ++s) cmax2 = fmax(cmax2, cabs2(cons[s]));
        out[2] = sc + NB * cmax2 * g2;
        double* lbo = out + 4 + 2 * NO;
        if (NB == 2 && c.M == 16) {
            // tile kt = first B stream b0 fixed, b1 over all 16 symbols:
            //   ||r0 - g1 x||^2 = ||r0||^2 - 2 Re(conj(x) g1^H r0) + |x|^2 ||g1||^2,
            //   r0 = w - g0 x_b0  (4 flops per hypothesis instead of NR complex products)
            double ng = 0.0;
#pragma unroll
            for (int r = 0; r < NR; ++r) ng += cabs2(g[NB - 1][r]);
            for (int kt = 0; kt < c.nkt; ++kt) {
                const cd xb0 = cons[kt];
                double n0 = 0.0;
                cd aa = czero();
#pragma unroll
                for (int r = 0; r < NR; ++r) {
                    const cd r0 = csub(w[r], cmul(g[0][r], xb0));
                    n0 += cabs2(r0);
                    aa = cfmac(aa, r0, g[NB - 1][r]);          // g1^H r0
                }
                double lbm = INFINITY;
                for (int s1 = 0; s1 < 16; ++s1) {
                    const cd x = cons[s1];
                    const double lb = fma(cabs2(x), ng, n0 - 2.0 * (x.x * aa.x + x.y * aa.y));
                    lbm = fmin(lbm, lb);
                }
                lbo[kt] = ok ? fmax(lbm, 0.0) : 0.0;
            }
        } else
        for (int kt = 0; kt < c.nkt; ++kt) {
            double lbm = INFINITY;
            for (int s = 0; s < 16; ++s) {
                const int k = kt * 16 + s;
                double lb = 0.0;
#pragma unroll
                for (int r = 0; r < NR; ++r) {
                    cd res = w[r];
#pragma unroll
                    for (int bb = 0; bb < NB; ++bb)
                        res = csub(res, cmul(g[bb][r], cons[(k >> (c.lm * (NB - 1 - bb))) & mask]));
                    lb += cabs2(res);
                }
                lbm = fmin(lbm, lb);
            }
            lbo[kt] = ok ? lbm : 0.0;
        }
    }
    // ---- row-tile bound vectors (NT = 4): the block of hypotheses with first streams
    //      (x_0, x_2) fixed has d >= ||P (y - h_0 x_0 - h_2 x_2)||^2, P = projector onto
    //      span(h_1, h_3)^perp (x_1, x_3 continuous); a degenerate basis gives P = 0 ----
    if constexpr (NT == 4) {
        cd u[2][NR];
        bool ok = true;
#pragma unroll
        for (int q = 0; q < 2; ++q) {
            cd v[NR];
            double h2 = 0.0;
#pragma unroll
            for (int r = 0; r < NR; ++r) { v[r] = H[2 * q + 1][r]; h2 += cabs2(v[r]); }
#pragma unroll
            for (int rep = 0; rep < 2; ++rep)
#pragma unroll
                for (int j = 0; j < q; ++j) {
                    cd pj = czero();
#pragma unroll
                    for (int r = 0; r < NR; ++r) pj = cfmac(pj, v[r], u[j][r]);
#pragma unroll
                    for (int r = 0; r < NR; ++r) v[r] = csub(v[r], cmul(u[j][r], pj));
                }
            double n2 = 0.0;
#pragma unroll
            for (int r = 0; r < NR; ++r) n2 += cabs2(v[r]);
            ok = ok && h2 > 0.0 && n2 > 1e-6 * h2;
            const double inv = ok ? fast_rsqrt(n2) : 0.0;
#pragma unroll
            for (int r = 0; r < NR; ++r) u[q][r] = cscale(v[r], inv);
        }
        cd w[3][NR];
#pragma unroll
        for (int r = 0; r < NR; ++r) { w[0][r] = y[r]; w[1][r] = H[0][r]; w[2][r] = H[2][r]; }
#pragma unroll
        for (int j = 0; j < 2; ++j)
#pragma unroll
            for (int m = 0; m < 3; ++m) {
                cd pw = czero();
#pragma unroll
                for (int r = 0; r < NR; ++r) pw = cfmac(pw, w[m][r], u[j][r]);
#pragma unroll
                for (int r = 0; r < NR; ++r) w[m][r] = csub(w[m][r], cmul(u[j][r], pw));
            }
        double* rbo = out + 4 + 2 * NO + ((c.nkt + 1) / 2 * 2);
#pragma unroll
        for (int m = 0; m < 3; ++m)
#pragma unroll
            for (int r = 0; r < NR; ++r) {
                rbo[2 * (m * NR + r)] = ok ? w[m][r].x : 0.0;
                rbo[2 * (m * NR + r) + 1] = ok ? w[m][r].y : 0.0;
            }
    }
}

// The constellation in LDS (wave-uniform loops over it read broadcasts instead of issuing a
// dependent global load per point); every thread of the block must call it.
__device__ __forceinline__ const cd* stage_cons(const cd* cons, int M) {
    __shared__ cd s_cons[64];
    if ((int)threadIdx.x < M) s_cons[threadIdx.x] = cons[threadIdx.x];
    __syncthreads();
    return s_cons;
}

template <int NT, int NR>
__global__ __launch_bounds__(256) void estep_prep_kernel(EstepArgs a, PrepConst c) {
    const cd* cons = stage_cons(a.cons, c.M);
    const long nsym = (long)c.B * c.Td;
    const long gsym = (long)blockIdx.x * blockDim.x + threadIdx.x;
    if (gsym >= nsym) return;
    const int b = (int)(gsym / c.Td);
    if (a.done && a.done[b]) return;
    if (a.varn_t) {                                  // per-trial noise variance (ABI 6)
        const TrialNoise tn = trial_noise(a.varn_t[b]);
        c.reg = tn.reg; c.thr_d = tn.thr_d; c.inv_s2 = tn.inv_s2;
    }
    cd H[NT][NR];
    heff_load<NT, NR>(a, c, gsym, b, H);
    cd y[NR];
#pragma unroll
    for (int r = 0; r < NR; ++r) y[r] = a.yd[(size_t)gsym * NR + r];
    double* out = a.prep + (size_t)gsym * c.stride;
#pragma unroll
    for (int q = 0; q < NT; ++q)
#pragma unroll
        for (int r = 0; r < NR; ++r) {
            out[4 + 2 * (q * NR + r)] = H[q][r].x;
            out[5 + 2 * (q * NR + r)] = H[q][r].y;
        }
    cd Lm[NT][NT], zf[NT];
    double piv[NT], dinv[NT], sc;
    ridge_chol<NT, NR>(H, y, c.reg, Lm, piv, dinv, zf);
    int xidx;
    out[0] = prep_candidate<NT, NR>(H, y, Lm, dinv, zf, cons, c.M, sc, xidx);
    out[1] = sc;
    prep_bounds<NT, NR>(H, y, out, cons, c);
}

// The tile bounds of the symbols the sphere pass left to the sweep (H_eff, d0 and the scale
// are in their prep records already).  Grid over all symbols; threads past the list exit.
template <int NT, int NR>
__global__ __launch_bounds__(256) void estep_bounds_kernel(EstepArgs a, PrepConst c) {
    const long nsym = (long)c.B * c.Td;
    const long n = a.list[nsym];
    if ((long)blockIdx.x * blockDim.x >= n) return;  // the whole block is past the list
    const cd* cons = stage_cons(a.cons, c.M);
    const long gi = (long)blockIdx.x * blockDim.x + threadIdx.x;
    if (gi >= n) return;
    const long gsym = a.list[gi];
    double* out = a.prep + (size_t)gsym * c.stride;
    cd H[NT][NR], y[NR];
#pragma unroll
    for (int q = 0; q < NT; ++q)
#pragma unroll
        for (int r = 0; r < NR; ++r) H[q][r] = cmk(out[4 + 2 * (q * NR + r)], out[5 + 2 * (q * NR + r)]);
#pragma unroll
    for (int r = 0; r < NR; ++r) y[r] = a.yd[(size_t)gsym * NR + r];
    prep_bounds<NT, NR>(H, y, out, cons, c);
}

// ============================================================================
// Sphere pass (SPH = 1 soft, 2 hard), replacing the preparation pass when n_rx >= n_tx:
// every symbol's hypotheses inside
//   d(x) <= R,   R = R0 + 50 varn^2 (soft) / R0 (hard),   R0 = the distance of a real hypothesis,
// are enumerated exactly -- the hypotheses whose weights are not below e^-50 of the posterior
// maximum (or that can be the argmin): the set the sweep's tile bounds keep.
//   Streams are ordered by reliability (diag of (H^H H + reg I)^-1: the least reliable at
// level 0, the most reliable at the top level NT-1, as in V-BLAST).  With G' = Hp^H Hp + reg I
// = L L^H for the permuted H and zf = L^-1 Hp^H y:
//   ||y - Hp x||^2 = c0 + sum_i T_i,   c0 = ||y||^2 - ||zf||^2,
//   T_i = |L_ii x_i - e_i|^2 - reg |x_i|^2,   e_i = zf_i - sum_{j>i} conj(L_ji) x_j,
// and T_j >= -reg max|c|^2, so every hypothesis below a level-i node has
//   d - c0 >= sum_{j>=i} T_j - i reg max|c|^2.
// Distances are kept relative to c0 (common to all hypotheses of the symbol: it cancels from
// the weights and the argmin).  R0 = min(candidate, Babai point of the sorted tree).
// Part 1 (estep_tree_kernel, one THREAD per symbol): H_eff, the sweep's prep record, the
// ordering, the factorisation, the Babai point -> the symbol's tree record.
// Part 2 (estep_bfs_kernel, one WAVE per symbol): level by level, every (surviving path,
// child) pair in its own lane, survivors compacted by ballot into an LDS path list; leaves
// weighted in the lanes.  Control flow is wave-uniform: a symbol costs what its tree holds.
// A symbol whose path list outgrows `budget`, or whose G' is ill-conditioned, is listed for
// the tile bounds and the MFMA sweep.
// ============================================================================
constexpr int kTrec = kTreeRecDoubles;   // doubles per symbol of the tree record (NT <= 4)
constexpr int kBfsWaves = 4;       // waves per block of the enumeration
constexpr int kBfsSpw = 8;         // consecutive symbols per wave
constexpr int kBfsPmax = 256;      // path list capacity per level

template <int NT, int NR>
__global__ __launch_bounds__(256) void estep_tree_kernel(EstepArgs a, PrepConst c) {
    const cd* cons = stage_cons(a.cons, c.M);
    const long nsym = (long)c.B * c.Td;
    const long gsym = (long)blockIdx.x * blockDim.x + threadIdx.x;
    bool live = gsym < nsym;
    const int b = live ? (int)(gsym / c.Td) : 0;
    if (live && a.done && a.done[b]) live = false;
    if (live && a.varn_t) {                          // per-trial noise variance (ABI 6)
        const TrialNoise tn = trial_noise(a.varn_t[b]);
        c.reg = tn.reg; c.thr_d = tn.thr_d; c.inv_s2 = tn.inv_s2;
    }
    bool single = false;
    double f2d = INFINITY;            // NT = 2: the factorised pass's range bound (fact2_bound)
    if (live) {
    cd Lm[NT][NT], zf[NT];
    double piv[NT], dinv[NT], d0, sc, screen, gsum;
    int lev[NT];
    double c0 = 0.0;
    {
        cd H[NT][NR], y[NR];
        heff_load<NT, NR>(a, c, gsym, b, H);
#pragma unroll
        for (int r = 0; r < NR; ++r) y[r] = a.yd[(size_t)gsym * NR + r];
        double* out = a.prep + (size_t)gsym * c.stride;
#pragma unroll
        for (int q = 0; q < NT; ++q)
#pragma unroll
            for (int r = 0; r < NR; ++r) {
                out[4 + 2 * (q * NR + r)] = H[q][r].x;
                out[5 + 2 * (q * NR + r)] = H[q][r].y;
            }
        ridge_chol<NT, NR>(H, y, c.reg, Lm, piv, dinv, zf);
        int xidx;
        d0 = prep_candidate<NT, NR>(H, y, Lm, dinv, zf, cons, c.M, sc, xidx);
        out[0] = d0;
        out[1] = sc;
        screen = pair_screen<NT, NR>(H, y, xidx, cons, gsum);
        if constexpr (NT == 2)          // hard: every unresolved symbol (no exponentials, no range)
            f2d = c.pair ? (c.hard ? 0.0 : fact2_bound<NR>(H, y, xidx, cons, c.M, c.inv_s2)) : INFINITY;
        // computed here, while H and y are live anyway (left to the compiler, the computation
        // sinks to the record store at the end and keeps H_eff live across the whole kernel)
        asm volatile("" : "+v"(screen), "+v"(gsum), "+v"(f2d));
        // reliability of stream q: g_q = [(G + reg I)^-1]_qq = sum_k |(L^-1)_kq|^2
        cd W[NT][NT];
        double g[NT];
#pragma unroll
        for (int j = 0; j < NT; ++j) {
            W[j][j] = cmk(dinv[j], 0.0);
#pragma unroll
            for (int i = j + 1; i < NT; ++i) {
                cd s = czero();
#pragma unroll
                for (int k = j; k < i; ++k) s = cfma(s, Lm[i][k], W[k][j]);
                W[i][j] = cscale(s, -dinv[i]);
            }
        }
#pragma unroll
        for (int q = 0; q < NT; ++q) {
            double s = 0.0;
#pragma unroll
            for (int k = q; k < NT; ++k) s += cabs2(W[k][q]);
            g[q] = s;
        }
        // level of stream q = its rank in descending g (ties by index)
#pragma unroll
        for (int q = 0; q < NT; ++q) {
            int rk = 0;
#pragma unroll
            for (int p = 0; p < NT; ++p) rk += (g[p] > g[q] || (g[p] == g[q] && p < q)) ? 1 : 0;
            lev[q] = rk;
        }
        cd Hp[NT][NR];
#pragma unroll
        for (int l = 0; l < NT; ++l)
#pragma unroll
            for (int r = 0; r < NR; ++r) {
                cd v = H[0][r];
#pragma unroll
                for (int q = 1; q < NT; ++q) v = csel(lev[q] == l, H[q][r], v);
                Hp[l][r] = v;
            }
        ridge_chol<NT, NR>(Hp, y, c.reg, Lm, piv, dinv, zf);
#pragma unroll
        for (int r = 0; r < NR; ++r) c0 += cabs2(y[r]);
#pragma unroll
        for (int j = 0; j < NT; ++j) c0 -= cabs2(zf[j]);
    }
    double ui[NT];
    double pmin = piv[0], pmax = piv[0];
#pragma unroll
    for (int j = 0; j < NT; ++j) {
        ui[j] = piv[j] * dinv[j];                          // L_jj = sqrt(pivot)
        pmin = fmin(pmin, piv[j]);
        pmax = fmax(pmax, piv[j]);
    }
    // Babai point of the sorted tree: the nearest child level by level
    double db = 0.0, cmax2 = 0.0;
    cd xb[NT], eb[NT];
    int sb[NT];
#pragma unroll
    for (int l = NT - 1; l >= 0; --l) {
        cd e = zf[l];
#pragma unroll
        for (int j = l + 1; j < NT; ++j) e = csub(e, cmul(cconj(Lm[j][l]), xb[j]));
        const double aa = fma(ui[l], ui[l], -c.reg), m2u = -2.0 * ui[l];
        double tb = INFINITY;
        int si = 0;
        #pragma unroll 4
        for (int s = 0; s < c.M; ++s) {
            const cd x = cons[s];
            const double x2 = cabs2(x);
            cmax2 = fmax(cmax2, x2);
            const double t = fma(aa, x2, m2u * fma(x.x, e.x, x.y * e.y));
            if (t < tb) { tb = t; si = s; }
        }
        xb[l] = cons[si];
        sb[l] = si;
        eb[l] = e;
        db += tb + cabs2(e);
    }
    const bool ok = pmax <= 1e10 * pmin;                 // ill-conditioned G': to the sweep
    const double R0 = fmin(d0 - c0, db);
    // single-path check: if along the Babai path every level has exactly one child whose
    // subtree bound is inside R (the Babai child), the Babai point is the only hypothesis
    // inside the sphere -- the posterior is x_B (weights of all others < e^-50) / the argmin
    if (ok && db <= R0) {
        const double R = R0 + (c.hard ? 0.0 : c.thr_d) + 1e-9 * sc;
        const double slack = c.reg * cmax2;
        double base = 0.0;
        bool one = true;
#pragma unroll
        for (int l = NT - 1; l >= 0; --l) {
            const cd e = eb[l];
            const double aa = fma(ui[l], ui[l], -c.reg), m2u = -2.0 * ui[l];
            const double thr = R + l * slack - base - cabs2(e);
            int n = 0;
            #pragma unroll 4
            for (int s = 0; s < c.M; ++s) {
                const cd x = cons[s];
                n += fma(aa, cabs2(x), m2u * fma(x.x, e.x, x.y * e.y)) <= thr ? 1 : 0;
            }
            one = one && n == 1;
            const cd x = xb[l];
            base += fma(aa, cabs2(x), m2u * fma(x.x, e.x, x.y * e.y)) + cabs2(e);
        }
        if (one) {
            single = true;
            constexpr int MS = NT + NT * NT;
            cd xo[NT];                                   // stream order
#pragma unroll
            for (int q = 0; q < NT; ++q) {
                cd v = xb[0];
#pragma unroll
                for (int l = 1; l < NT; ++l) v = csel(lev[q] == l, xb[l], v);
                xo[q] = v;
            }
            cd* mo = a.mom + (size_t)gsym * MS;
#pragma unroll
            for (int p2 = 0; p2 < NT; ++p2) {
                mo[p2] = xo[p2];
#pragma unroll
                for (int q = 0; q < NT; ++q) mo[NT + p2 * NT + q] = cmulc(xo[p2], xo[q]);
            }
        }
    }
    // the tree record: only the enumeration reads it (not the single-path symbols, nor the
    // n_tx = 2 symbols of the factorised passes)
    if (!single && !(NT == 2 && c.pair)) {
    int packed = ok ? (1 << 16) : 0;
#pragma unroll
    for (int q = 0; q < NT; ++q) packed |= q << (4 * lev[q]);   // level l holds stream perm[l]
    double* rec = a.tree + (size_t)gsym * kTrec;
    rec[0] = c0;
    rec[1] = R0;
    rec[2] = sc;
    rec[3] = (double)packed;
    rec[kTrec - 1] = fma(gsum, cmax2, screen) * c.inv_s2;   // the pass's range bound
#pragma unroll
    for (int j = 0; j < NT; ++j) {
        rec[4 + j] = ui[j];
        rec[4 + NT + 2 * j] = zf[j].x;
        rec[5 + NT + 2 * j] = zf[j].y;
    }
    int k = 0;
#pragma unroll
    for (int i = 1; i < NT; ++i)
#pragma unroll
        for (int j = 0; j < i; ++j) {
            rec[4 + 3 * NT + 2 * k] = Lm[i][j].x;
            rec[5 + 3 * NT + 2 * k] = Lm[i][j].y;
            ++k;
        }
    }   // enumerated
    }   // live
    const bool f2 = NT == 2 && c.pair && live && !single;
    const bool wide = f2d <= kPairDmax;
    const bool enumer = live && !single && !f2;
    const int lane = threadIdx.x & 63;
    int32_t* cnt = a.list + nsym;
    // one atomic per BLOCK and list (4096 per-wave same-address atomics serialise at the L2):
    // the waves' counts through LDS, thread l reserves list l's block range
    __shared__ int s_n[2][4];
    __shared__ int s_b[2];
    const int wv = threadIdx.x >> 6;
    const unsigned long long bf = __ballot(f2 && wide), be = __ballot(enumer || (f2 && !wide));
    if (lane == 0) {
        s_n[0][wv] = __builtin_popcountll(bf);
        s_n[1][wv] = __builtin_popcountll(be);
    }
    __syncthreads();
    if (threadIdx.x < 2) {
        const int l = threadIdx.x;
        const int tot = s_n[l][0] + s_n[l][1] + s_n[l][2] + s_n[l][3];
        s_b[l] = tot ? atomicAdd(cnt + (l ? 2 : 3), tot) : 0;
    }
    __syncthreads();
    const unsigned long long lt = (1ull << lane) - 1ull;
    if (f2 || enumer) {
        // NT = 2 (pair mode): a symbol the factorised tables can represent (D within range; hard:
        // f2d = 0, every unresolved symbol) goes to the pair list (counter 3), a narrow one to
        // the enumeration list's slots (counter 2: no n_tx = 2 symbol is enumerated in pair mode,
        // and the enumeration is not launched) for estep_soft2_kernel; otherwise the live
        // unresolved symbols go to the enumeration list
        const bool p0 = f2 && wide;
        const int l = p0 ? 0 : 1;
        int base = s_b[l] + __builtin_popcountll((p0 ? bf : be) & lt);
        for (int w = 0; w < wv; ++w) base += s_n[l][w];
        if (p0) a.list[2 * nsym + 2 * kEstepListCnt + base] = (int32_t)gsym;
        else cnt[kEstepListCnt + base] = (int32_t)gsym;
    }
    if (c.count) {
        const unsigned long long one = __ballot(single);
        if (lane == 0) atomicAdd(&g_estep_sphere[2], (unsigned long long)__builtin_popcountll(one));
    }
}

template <int NT, int SPH>
__global__ __launch_bounds__(64 * kBfsWaves) void estep_bfs_kernel(EstepArgs a, PrepConst c) {
    typedef unsigned long long u64;
    constexpr int NP = NT * (NT - 1) / 2;
    constexpr int MS = NT + NT * NT;
    __shared__ cd s_cons[64];
    __shared__ double s_c2[64];
    __shared__ double s_pb[kBfsWaves][2][kBfsPmax];     // path bound (relative distance so far)
    __shared__ int s_pi[kBfsWaves][2][kBfsPmax];        // path symbols, level l at bits lm*l
    if ((int)threadIdx.x < c.M) {
        const cd x = a.cons[threadIdx.x];
        s_cons[threadIdx.x] = x;
        s_c2[threadIdx.x] = cabs2(x);
    }
    __syncthreads();
    double cmax2 = 0.0;
    for (int s = 0; s < c.M; ++s) cmax2 = fmax(cmax2, s_c2[s]);
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int lane = threadIdx.x & 63;
    const long nsym = (long)c.B * c.Td;
    // the tree pass's enumeration list: wave w takes entries w*spw .. (w+1)*spw - 1
    const int32_t* elist = a.list + nsym + kEstepListCnt;
    const long nwork = __builtin_amdgcn_readfirstlane(a.list[nsym + 2]);
    const long g0 = ((long)blockIdx.x * kBfsWaves + wave) * kBfsSpw;
    if (g0 >= nwork) return;
    const long g1 = g0 + kBfsSpw < nwork ? g0 + kBfsSpw : nwork;
    const int mask = c.M - 1, lm = c.lm;
    const int pmax = c.budget < kBfsPmax ? c.budget : kBfsPmax;
    const u64 lt = (1ull << lane) - 1ull;
    unsigned listed_mask = 0, pair_mask = 0, resolved_n = 0;
    // tree records by LDS-DMA, the next symbol's in flight while the current one is enumerated
    // (lanes 0-15 carry the record's 256 bytes; the others re-read its first 16 bytes)
    __shared__ __attribute__((aligned(16))) double s_rec[kBfsWaves][2][128];
    auto issue = [&](long gi, int buf) {
        const double* src = a.tree + (size_t)elist[gi] * kTrec + (lane < kTrec / 2 ? 2 * lane : 0);
        __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)src,
                                         (__attribute__((address_space(3))) void*)s_rec[wave][buf],
                                         16, 0, 0);
    };
    issue(g0, 0);
    for (long gi = g0; gi < g1; ++gi) {
        const long gsym = elist[gi];
        // the symbol's noise constants (per-trial variances, ABI 6); per level below: T_j >= -slack
        double thr_d = c.thr_d, inv_s2 = c.inv_s2, reg = c.reg;
        if (a.varn_t) {
            const TrialNoise tn = trial_noise(a.varn_t[gsym / c.Td]);
            thr_d = uniform_d(tn.thr_d);
            inv_s2 = uniform_d(tn.inv_s2);
            reg = uniform_d(tn.reg);
        }
        const double slack = reg * cmax2;
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");      // this symbol's record landed
        wave_sync();
        const double* rec = s_rec[wave][(gi - g0) & 1];
        if (gi + 1 < g1) issue(gi + 1, (gi + 1 - g0) & 1);
        const int packed = (int)rec[3];
        bool listed = !((packed >> 16) & 1);
        const double R0 = rec[1];
        const double margin = 1e-9 * rec[2];
        const double R = R0 + (SPH == 2 ? 0.0 : thr_d) + margin;
        double ui[NT];
        cd zf[NT], Lc[NP + 1];
#pragma unroll
        for (int j = 0; j < NT; ++j) {
            ui[j] = rec[4 + j];
            zf[j] = cmk(rec[4 + NT + 2 * j], rec[5 + NT + 2 * j]);
        }
#pragma unroll
        for (int k = 0; k < NP; ++k) Lc[k] = cmk(rec[4 + 3 * NT + 2 * k], -rec[5 + 3 * NT + 2 * k]);  // conj
        double bd = INFINITY;            // hard: this lane's best (distance, hypothesis index)
        int bj = 0x7fffffff;
        if (lane == 0) { s_pb[wave][0][0] = 0.0; s_pi[wave][0][0] = 0; }
        wave_sync();
        int n_in = 1;                    // paths entering the level; after level 0: leaves
#pragma unroll
        for (int l = NT - 1; l >= 0; --l) {
            if (listed) break;
            const int ib = (NT - 1 - l) & 1;
            const double* pbi = s_pb[wave][ib];
            const int* pii = s_pi[wave][ib];
            double* pbo = s_pb[wave][ib ^ 1];
            int* pio = s_pi[wave][ib ^ 1];
            const double u = ui[l];
            const double aa = fma(u, u, -reg), m2u = -2.0 * u;
            const double lim = R + l * slack;
            const int total = n_in << lm;
            int n_out = 0;
            for (int base = 0; base < total; base += 64) {
                const int i = base + lane;
                const bool valid = i < total;
                const int p = valid ? i >> lm : 0;
                const int s = i & mask;
                const double bp = pbi[p];
                const int ip = pii[p];
                cd e = zf[l];
#pragma unroll
                for (int j = l + 1; j < NT; ++j)      // L_jl at row-major strict index j(j-1)/2 + l
                    e = csub(e, cmul(Lc[j * (j - 1) / 2 + l], s_cons[(ip >> (lm * j)) & mask]));
                const cd x = s_cons[s];
                const double bb = bp + fma(aa, s_c2[s], m2u * fma(x.x, e.x, x.y * e.y)) + cabs2(e);
                const bool keep = valid && bb <= lim;
                const int idx = ip | (s << (lm * l));
                if (SPH == 2 && l == 0) {
                    if (keep) {
                        int jr = 0;                   // hypothesis index, original stream order
#pragma unroll
                        for (int q = 0; q < NT; ++q)
                            jr |= ((idx >> (lm * q)) & mask) << (lm * (NT - 1 - ((packed >> (4 * q)) & 15)));
                        if (bb < bd || (bb == bd && jr < bj)) { bd = bb; bj = jr; }
                    }
                } else {
                    // surviving paths (l > 0) / leaves inside the sphere (l == 0, soft)
                    const u64 bal = __ballot(keep);
                    const int slot = n_out + __builtin_popcountll(bal & lt);
                    if (keep && slot < pmax) { pbo[slot] = bb; pio[slot] = idx; }
                    n_out += __builtin_popcountll(bal);
                }
            }
            if (SPH == 2 && l == 0) break;
            if (n_out > pmax || n_out == 0) listed = true;    // too wide (or rounding lost all)
            n_in = n_out;
            wave_sync();
        }
        cd* mo = a.mom + (size_t)gsym * MS;
        if (!listed) {
            if constexpr (SPH == 2) {
#pragma unroll
                for (int off = 32; off >= 1; off >>= 1) {
                    const double od = shfl_xor_d(bd, off);
                    const int oj = __shfl_xor(bj, off);
                    if (od < bd || (od == bd && oj < bj)) { bd = od; bj = oj; }
                }
                if (bj == 0x7fffffff) listed = true;
                else if (lane < MS) {
                    const int p2 = lane < NT ? lane : (lane - NT) / NT;
                    const int q = lane < NT ? 0 : (lane - NT) % NT;
                    const cd xp = s_cons[(bj >> (lm * (NT - 1 - p2))) & mask];
                    const cd xq = s_cons[(bj >> (lm * (NT - 1 - q))) & mask];
                    mo[lane] = lane < NT ? xp : cmulc(xp, xq);
                }
            } else {
                // the n_in leaves inside the sphere (LDS list, level order): lane o < MS forms
                // output o (m_t, then S_t row-major, stream order) over the list, weights
                // exp(-(d - d_min)/varn^2) for the leaves within 50 varn^2 of the minimum
                const int ib = NT & 1;
                const double* lb = s_pb[wave][ib];
                const int* li = s_pi[wave][ib];
                // every leaf's weight lane-parallel (to the free half of the path-bound buffer);
                // the output lanes then only accumulate.  The minimum stays a serial LDS scan
                // (independent reads; a 6-step cross-lane reduction costs more for the few
                // leaves most symbols have)
                double dmin = INFINITY;
                for (int k = 0; k < n_in; ++k) dmin = fmin(dmin, lb[k]);
                double* lw = s_pb[wave][ib ^ 1];
                for (int k = lane; k < n_in; k += 64) {
                    const double d = lb[k];
                    lw[k] = d <= dmin + thr_d ? fexp_neg((dmin - d) * inv_s2) : 0.0;
                }
                wave_sync();
                if (lane < MS) {
                    const int sp_ = lane < NT ? lane : (lane - NT) / NT;   // output stream pair
                    const int sq_ = lane < NT ? 0 : (lane - NT) % NT;
                    int lp = 0, lq = 0;                                    // their levels
#pragma unroll
                    for (int l = 0; l < NT; ++l) {
                        const int st = (packed >> (4 * l)) & 15;
                        lp = st == sp_ ? l : lp;
                        lq = st == sq_ ? l : lq;
                    }
                    double z = 0.0;
                    cd v = czero();
                    for (int k = 0; k < n_in; ++k) {
                        const double w = lw[k];             // > 0 exactly for the leaves within
                        if (w != 0.0) {                     // 50 varn^2 of the minimum
                            const int id = li[k];
                            const cd xp = s_cons[(id >> (lm * lp)) & mask];
                            const cd xq = s_cons[(id >> (lm * lq)) & mask];
                            z += w;
                            v = caxpy(v, w, lane < NT ? xp : cmulc(xp, xq));
                        }
                    }
                    mo[lane] = cscale(v, 1.0 / z);
                }
            }
        }
        // a listed symbol whose range bound admits the factorised-weight pass goes to that pass
        const bool to_pair = listed && c.pair && rec[kTrec - 1] <= kPairDmax;
        wave_sync();
        if (to_pair) pair_mask |= 1u << (gi - g0);
        else if (listed) listed_mask |= 1u << (gi - g0);
        else ++resolved_n;
    }
    // the wave's listed symbols join the sweep's (or the factorised pass's) work list: one
    // atomic per wave and list
    auto append = [&](unsigned msk, int32_t* cntp, int32_t* lst) {
        const int n = __builtin_popcount(msk);
        if (!n) return;
        int base = 0;
        if (lane == 0) base = atomicAdd(cntp, n);
        base = __shfl(base, 0);
        if (lane < kBfsSpw && ((msk >> lane) & 1))
            lst[base + __builtin_popcount(msk & ((1u << lane) - 1u))] = elist[g0 + lane];
    };
    append(listed_mask, a.list + nsym, a.list);
    append(pair_mask, a.list + nsym + 3, a.list + 2 * nsym + 2 * kEstepListCnt);
    const int nl = __builtin_popcount(listed_mask) + __builtin_popcount(pair_mask);
    if (c.count && lane == 0) {
        atomicAdd(&g_estep_sphere[0], (unsigned long long)resolved_n);
        atomicAdd(&g_estep_sphere[1], (unsigned long long)nl);
    }
}

template <int NT, int NR, int MODE, int TU, bool V16 = false>
__global__ __launch_bounds__(128) void estep_mfma_kernel(EstepArgs a, MfmaConst c) {
    estep_mfma_body<NT, NR, MODE, TU, V16>(a, c);
}
bool make_mfma(const Problem& pb, MfmaConst& c, size_t& lds, long& blocks) {
    if (pb.NT < 2 || pb.NT > 4 || pb.NR < 1 || pb.NR > 8) return false;
    if (pb.M < 2 || pb.M > 64 || (pb.M & (pb.M - 1))) return false;
    int lm = 0;
    while ((1 << lm) < pb.M) ++lm;
    const int NA = pb.NT / 2, NB = pb.NT - NA;
    const long JA = 1L << (lm * NA), JB = 1L << (lm * NB);
    if (JA < 16 || JB < 16 || JA * JB > (1L << 24)) return false;
    c.B = pb.B; c.Td = pb.Td; c.P = pb.P; c.M = pb.M; c.lm = lm;
    c.JA = (int)JA; c.JB = (int)JB;
    c.chunk = (int)(JA < kChunk ? JA : kChunk);
    const int NO = pb.NT * pb.NR;
    c.nparts = NO <= 64 ? 64 / NO : 1;
    const int steps = (2 * pb.NR + 3) / 4;
    c.nkt_pad = (int)((JB / 16 + 1) / 2 * 2);

    c.prune = !g_debug.estep_noprune;
    c.count = g_debug.estep_count;
    c.inv_s2 = 1.0 / (pb.varn * pb.varn);
    c.thr_d = kSkipThr * pb.varn * pb.varn;
    c.reg = 0.1 * pb.varn * pb.varn;
    // NT = 4: + the row-tile bound vectors P y, P h_0, P h_2 (P = projector onto
    // span(h_1, h_3)^perp), 3 NR complex
    c.rowb_off = 4 + 2 * NO + c.nkt_pad;
    c.prep_stride = c.rowb_off + (pb.NT == 4 ? 6 * pb.NR : 0);
    c.rec_words = c.prep_stride + 2 * pb.NR;
    c.tab_d = mfma_tab_d(NO, c.chunk, steps, pb.M, c.nkt_pad, c.rec_words);
    c.spw = 4;                                           // symbols per wave
    c.screen = !g_debug.estep_nof32;                     // FP32 tile-group screen (V16)
    c.rowb = pb.NT == 4 && c.prune;
    lds = 64 * sizeof(cd) + (size_t)kMfmaWaves * c.tab_d * sizeof(double);
    const long nsym = (long)pb.B * pb.Td;
    const long per_block = (long)kMfmaWaves * c.spw;
    blocks = (nsym + per_block - 1) / per_block;
    return lds <= 160 * 1024;
}

template <int NT, int NR>
hipError_t dispatch_mfma_mode(const MfmaConst& c, size_t lds, long blocks, const EstepArgs& a,
                              int mode, hipStream_t s) {
    const bool tu4 = (c.chunk / 16) % 4 == 0;
    if (NT == 4 && c.M == 16 && tu4) {            // cfg1 geometry: hoisted V operand
        // the V16 body takes these layout constants as compile-time values
        if (c.JA != 256 || c.JB != 256 || c.chunk != 256 || c.nkt_pad != 16 ||
            c.prep_stride != 4 + 2 * NT * NR + 16 + 6 * NR)
            return hipErrorInvalidValue;
        if (mode == SBCE_ESTEP_HARD)
            hipLaunchKernelGGL((estep_mfma_kernel<NT, NR, SBCE_ESTEP_HARD, 4, true>),
                               dim3((unsigned)blocks), dim3(64 * kMfmaWaves), lds, s, a, c);
        else
            hipLaunchKernelGGL((estep_mfma_kernel<NT, NR, SBCE_ESTEP_SOFT, 4, true>),
                               dim3((unsigned)blocks), dim3(64 * kMfmaWaves), lds, s, a, c);
        return hipGetLastError();
    }
    if (mode == SBCE_ESTEP_HARD) {
        if (tu4)
            hipLaunchKernelGGL((estep_mfma_kernel<NT, NR, SBCE_ESTEP_HARD, 4>), dim3((unsigned)blocks),
                               dim3(64 * kMfmaWaves), lds, s, a, c);
        else
            hipLaunchKernelGGL((estep_mfma_kernel<NT, NR, SBCE_ESTEP_HARD, 1>), dim3((unsigned)blocks),
                               dim3(64 * kMfmaWaves), lds, s, a, c);
    } else {
        if (tu4)
            hipLaunchKernelGGL((estep_mfma_kernel<NT, NR, SBCE_ESTEP_SOFT, 4>), dim3((unsigned)blocks),
                               dim3(64 * kMfmaWaves), lds, s, a, c);
        else
            hipLaunchKernelGGL((estep_mfma_kernel<NT, NR, SBCE_ESTEP_SOFT, 1>), dim3((unsigned)blocks),
                               dim3(64 * kMfmaWaves), lds, s, a, c);
    }
    return hipGetLastError();
}

template <int NT>
hipError_t dispatch_mfma_nr(int NR, const MfmaConst& c, size_t lds, long blocks,
                            const EstepArgs& a, int mode, hipStream_t s) {
    switch (NR) {
        case 1: return dispatch_mfma_mode<NT, 1>(c, lds, blocks, a, mode, s);
        case 2: return dispatch_mfma_mode<NT, 2>(c, lds, blocks, a, mode, s);
        case 3: return dispatch_mfma_mode<NT, 3>(c, lds, blocks, a, mode, s);
        case 4: return dispatch_mfma_mode<NT, 4>(c, lds, blocks, a, mode, s);
        case 5: return dispatch_mfma_mode<NT, 5>(c, lds, blocks, a, mode, s);
        case 6: return dispatch_mfma_mode<NT, 6>(c, lds, blocks, a, mode, s);
        case 7: return dispatch_mfma_mode<NT, 7>(c, lds, blocks, a, mode, s);
        case 8: return dispatch_mfma_mode<NT, 8>(c, lds, blocks, a, mode, s);
    }
    return hipErrorInvalidValue;
}

struct Geometry {
    EstepConst c;
    int KP;
    size_t lds;
    long blocks;
};

bool make_geometry(const Problem& pb, Geometry& g) {
    if (pb.NT < 1 || pb.NT > 4 || pb.NR < 1 || pb.NR > 8) return false;
    if (pb.M < 2 || pb.M > 64 || (pb.M & (pb.M - 1))) return false;
    int lm = 0;
    while ((1 << lm) < pb.M) ++lm;
    const int NA = pb.NT / 2, NB = pb.NT - NA;
    const long JA = 1L << (lm * NA), JB = 1L << (lm * NB);
    if (JA * JB > (1L << 24)) return false;
    EstepConst& c = g.c;
    c.B = pb.B; c.Td = pb.Td; c.P = pb.P; c.M = pb.M; c.lm = lm;
    c.JA = (int)JA; c.JB = (int)JB;
    if (JB >= 256) { g.KP = 4; c.S = 64; }
    else { g.KP = 1; c.S = (int)(JB < 64 ? JB : 64); }
    c.SPW = 64 / c.S;
    c.npass = (int)(JB / ((long)c.S * g.KP));
    c.CI = (int)(JA < c.S ? JA : c.S);
    c.CIp = (c.CI + kCH - 1) / kCH * kCH;
    const int NO = pb.NT * pb.NR;
    c.nparts = c.S >= NO ? c.S / NO : 1;
    c.heff_cd = c.SPW * NO;
    const int ptab = c.SPW * c.CIp * (pb.NR + 1);
    const int part = c.SPW * NO * c.nparts;
    c.ptab_cd = ptab > part ? ptab : part;
    c.inv_s2 = 1.0 / (pb.varn * pb.varn);
    c.thr_d = kSkipThr * pb.varn * pb.varn;
    g.lds = (size_t)(64 + kWavesPerBlock * (c.heff_cd + c.ptab_cd)) * sizeof(cd);
    const long nsym = (long)pb.B * pb.Td;
    const long waves = (nsym + c.SPW - 1) / c.SPW;
    g.blocks = (waves + kWavesPerBlock - 1) / kWavesPerBlock;
    return g.lds <= 160 * 1024;
}

template <int NT, int NR, int KP>
hipError_t dispatch_mode(const Geometry& g, const EstepArgs& a, int mode, hipStream_t s) {
    if (mode == SBCE_ESTEP_HARD)
        hipLaunchKernelGGL((estep_kernel<NT, NR, KP, SBCE_ESTEP_HARD>), dim3((unsigned)g.blocks),
                           dim3(256), g.lds, s, a, g.c);
    else
        hipLaunchKernelGGL((estep_kernel<NT, NR, KP, SBCE_ESTEP_SOFT>), dim3((unsigned)g.blocks),
                           dim3(256), g.lds, s, a, g.c);
    return hipGetLastError();
}

template <int NT, int NR>
hipError_t dispatch_kp(const Geometry& g, const EstepArgs& a, int mode, hipStream_t s) {
    if constexpr (NT >= 3) {
        if (g.KP == 4) return dispatch_mode<NT, NR, 4>(g, a, mode, s);
    }
    return dispatch_mode<NT, NR, 1>(g, a, mode, s);
}

template <int NT>
hipError_t dispatch_nr(int NR, const Geometry& g, const EstepArgs& a, int mode, hipStream_t s) {
    switch (NR) {
        case 1: return dispatch_kp<NT, 1>(g, a, mode, s);
        case 2: return dispatch_kp<NT, 2>(g, a, mode, s);
        case 3: return dispatch_kp<NT, 3>(g, a, mode, s);
        case 4: return dispatch_kp<NT, 4>(g, a, mode, s);
        case 5: return dispatch_kp<NT, 5>(g, a, mode, s);
        case 6: return dispatch_kp<NT, 6>(g, a, mode, s);
        case 7: return dispatch_kp<NT, 7>(g, a, mode, s);
        case 8: return dispatch_kp<NT, 8>(g, a, mode, s);
    }
    return hipErrorInvalidValue;
}

}  // namespace

hipError_t estep_debug_sphere(unsigned long long* out3, int reset) {
    if (reset) {
        const unsigned long long z[3] = {0, 0, 0};
        return hipMemcpyToSymbol(HIP_SYMBOL(g_estep_sphere), z, sizeof(z), 0, hipMemcpyHostToDevice);
    }
    return hipMemcpyFromSymbol(out3, HIP_SYMBOL(g_estep_sphere), 3 * sizeof(*out3), 0,
                               hipMemcpyDeviceToHost);
}

hipError_t estep_debug_mfma(unsigned long long* out, int reset) {
    if (reset) {
        const unsigned long long z = 0;
        return hipMemcpyToSymbol(HIP_SYMBOL(g_estep_mfma), &z, sizeof(z), 0, hipMemcpyHostToDevice);
    }
    return hipMemcpyFromSymbol(out, HIP_SYMBOL(g_estep_mfma), sizeof(*out), 0,
                               hipMemcpyDeviceToHost);
}

int estep_prep_stride(const Problem& pb) {
    MfmaConst mc;
    size_t lds;
    long blocks;
    return make_mfma(pb, mc, lds, blocks) ? mc.prep_stride : 0;
}

bool estep_supported(const Problem& pb, int mode) {
    if (mode >= SBCE_ESTEP_PM && mode <= SBCE_ESTEP_GAUSS) return estep_pm_supported(pb, pb.pr, mode);
    Geometry g;
    return (mode == SBCE_ESTEP_SOFT || mode == SBCE_ESTEP_HARD) && make_geometry(pb, g);
}

hipError_t launch_estep(const Problem& pb, const EstepArgs& a, int mode, hipStream_t s) {
    if (mode >= SBCE_ESTEP_PM && mode <= SBCE_ESTEP_GAUSS) return launch_estep_pm(pb, a, mode, pb.pr, s);
    const bool force_valu = g_debug.estep_valu;     // VALU kernel (A/B runs)
    MfmaConst mc;
    size_t mlds;
    long mblocks;
    if (!force_valu && make_mfma(pb, mc, mlds, mblocks)) {
        if (mblocks == 0) return hipSuccess;
        EstepArgs as = a;            // the sweep's view: list only when the sphere pass ran
        if (a.prep) {
            PrepConst pc;
            pc.B = pb.B; pc.Td = pb.Td; pc.P = pb.P; pc.M = pb.M; pc.lm = mc.lm;
            pc.nkt = mc.JB >> 4; pc.stride = mc.prep_stride; pc.reg = mc.reg;
            pc.uni = 1;
            // sphere pass instead of the preparation pass (SBCE_ESTEP_SPHERE=0 disables: A/B);
            // n_rx < n_tx (singular H^H H) always leaves the symbol to the sweep: not compiled
            const bool sphere = a.list && a.tree && pb.NR >= pb.NT && !g_debug.estep_nosphere;
            pc.budget = g_debug.sphere_budget;                  // path list cap per level
            pc.count = mc.count;
            pc.inv_s2 = mc.inv_s2;
            pc.thr_d = mc.thr_d;
            pc.hard = mode == SBCE_ESTEP_HARD;
            pc.pair = estep_pair_supported(pb, mode) ? 1 : 0;
            if (!sphere) as.list = nullptr;
            const long nsym = (long)pb.B * pb.Td;
            const dim3 pg((unsigned)((nsym + 255) / 256)), pblk(256);
            hipError_t e = hipErrorInvalidValue;
            if (sphere) {
                // sphere pass (tree records, enumeration), then the tile bounds of the listed
                if (!a.lists_zeroed) {
                    const hipError_t me = hipMemsetAsync(a.list + nsym, 0, 5 * sizeof(int32_t), s);
                    if (me != hipSuccess) return me;
                }
                const long nbfs = (nsym + kBfsSpw * kBfsWaves - 1) / (kBfsSpw * kBfsWaves);
                const dim3 bg((unsigned)nbfs), bblk(64 * kBfsWaves);
                const bool hard = mode == SBCE_ESTEP_HARD;
                switch (pb.NT * 16 + pb.NR) {
#define SBCE_SPH(nt, nr) case nt * 16 + nr: \
    hipLaunchKernelGGL((estep_tree_kernel<nt, nr>), pg, pblk, 0, s, as, pc); \
    if (nt == 2 && pc.pair) {} /* no enumeration: the pair passes take every listed symbol */ \
    else if (hard) hipLaunchKernelGGL((estep_bfs_kernel<nt, 2>), bg, bblk, 0, s, as, pc); \
    else hipLaunchKernelGGL((estep_bfs_kernel<nt, 1>), bg, bblk, 0, s, as, pc); \
    e = hipGetLastError(); \
    break;
                    SBCE_SPH(2, 2) SBCE_SPH(2, 3) SBCE_SPH(2, 4) SBCE_SPH(2, 5)
                    SBCE_SPH(2, 6) SBCE_SPH(2, 7) SBCE_SPH(2, 8)
                    SBCE_SPH(3, 3) SBCE_SPH(3, 4) SBCE_SPH(3, 5) SBCE_SPH(3, 6) SBCE_SPH(3, 7)
                    SBCE_SPH(3, 8)
                    SBCE_SPH(4, 4) SBCE_SPH(4, 5) SBCE_SPH(4, 6) SBCE_SPH(4, 7) SBCE_SPH(4, 8)
#undef SBCE_SPH
                }
                // wide posteriors of the cfg-1 geometry: the factorised-weight pass resolves the
                // symbols the enumeration routed to it and lists the ones it cannot represent
                // for the tile bounds and the sweep
                if (e == hipSuccess && pc.pair) e = launch_estep_pair(pb, as, mc.prep_stride, mc.count, mode, s);
                if (e == hipSuccess) {
                    switch (pb.NT * 16 + pb.NR) {
#define SBCE_BND(nt, nr) case nt * 16 + nr: \
    hipLaunchKernelGGL((estep_bounds_kernel<nt, nr>), pg, pblk, 0, s, as, pc); e = hipGetLastError(); break;
                        SBCE_BND(2, 2) SBCE_BND(2, 3) SBCE_BND(2, 4) SBCE_BND(2, 5)
                        SBCE_BND(2, 6) SBCE_BND(2, 7) SBCE_BND(2, 8)
                        SBCE_BND(3, 3) SBCE_BND(3, 4) SBCE_BND(3, 5) SBCE_BND(3, 6) SBCE_BND(3, 7)
                        SBCE_BND(3, 8)
                        SBCE_BND(4, 4) SBCE_BND(4, 5) SBCE_BND(4, 6) SBCE_BND(4, 7) SBCE_BND(4, 8)
#undef SBCE_BND
                    }
                }
            } else {
                switch (pb.NT * 16 + pb.NR) {
#define SBCE_PREP(nt, nr) case nt * 16 + nr: hipLaunchKernelGGL((estep_prep_kernel<nt, nr>), pg, pblk, 0, s, as, pc); e = hipGetLastError(); break;
                    SBCE_PREP(2, 1) SBCE_PREP(2, 2) SBCE_PREP(2, 3) SBCE_PREP(2, 4)
                    SBCE_PREP(2, 5) SBCE_PREP(2, 6) SBCE_PREP(2, 7) SBCE_PREP(2, 8)
                    SBCE_PREP(3, 1) SBCE_PREP(3, 2) SBCE_PREP(3, 3) SBCE_PREP(3, 4)
                    SBCE_PREP(3, 5) SBCE_PREP(3, 6) SBCE_PREP(3, 7) SBCE_PREP(3, 8)
                    SBCE_PREP(4, 1) SBCE_PREP(4, 2) SBCE_PREP(4, 3) SBCE_PREP(4, 4)
                    SBCE_PREP(4, 5) SBCE_PREP(4, 6) SBCE_PREP(4, 7) SBCE_PREP(4, 8)
#undef SBCE_PREP
                }
            }
            if (e != hipSuccess) return e;
            // listed sweep: waves grab work until the list is exhausted, so a grid that
            // fills the chip (8 two-wave blocks per CU) is enough
            if (sphere && mblocks > 2048) mblocks = 2048;
        } else {
            as.list = nullptr;
        }
        switch (pb.NT) {
            case 2: return dispatch_mfma_nr<2>(pb.NR, mc, mlds, mblocks, as, mode, s);
            case 3: return dispatch_mfma_nr<3>(pb.NR, mc, mlds, mblocks, as, mode, s);
            case 4: return dispatch_mfma_nr<4>(pb.NR, mc, mlds, mblocks, as, mode, s);
        }
    }
    Geometry g;
    if (!make_geometry(pb, g)) return hipErrorInvalidValue;
    if (g.blocks == 0) return hipSuccess;
    switch (pb.NT) {
        case 1: return dispatch_nr<1>(pb.NR, g, a, mode, s);
        case 2: return dispatch_nr<2>(pb.NR, g, a, mode, s);
        case 3: return dispatch_nr<3>(pb.NR, g, a, mode, s);
        case 4: return dispatch_nr<4>(pb.NR, g, a, mode, s);
    }
    return hipErrorInvalidValue;
}

}  // namespace sbce
