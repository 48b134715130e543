// Internal device helpers and launch declarations for libsbce (gfx950 / CDNA4).
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>
#include <math.h>

#include "../../include/sbce.h"

namespace sbce {

// complex double, interleaved (numpy complex128 memory)
typedef double2 cd;

// C -= A conj(B)^T on a 16 x 16 complex MFMA tile, one k-step of 4 (lane values v = A, t = B,
// v_mfma_f64_16x16x4f64 operand layout): four real MFMAs, or three with G3 (Gauss):  with
// P1 = sum ar br, P2 = sum ai bi, P3 = sum (ar + ai)(br - bi) the update has
//   re = C_re - P1 - P2,   im = C_im - (P3 - P1 + P2);
// the accumulators X1 = C_re - P1 (cre), X2 = -P2 (c2), X3 = C_im + C_re - P3 (cim, csub_init)
// give re = X1 + X2, im = X3 - X1 + X2 (csub_out).  The rounding of the imaginary part grows
// (error ~ eps (|ar| + |ai|)(|br| + |bi|)), so G3 is used where no rank decision reads the
// result: the CHOL solve, and in the min-norm solve AFTER the rank cut (the Gram build C = G^H G,
// minnorm.hip gram_kernel, and C's own tiled factorisation).  Never for R's factorisation in the
// drop or min-norm paths: its pivots past the numerical rank ARE the rounding noise, and the
// pivot decisions must see four-MFMA rounding.
typedef double mf4 __attribute__((ext_vector_type(4)));
template <bool G3>
__device__ __forceinline__ void csub_init(mf4& cre, mf4& cim, mf4& c2) {
    c2 = mf4{0.0, 0.0, 0.0, 0.0};
    if constexpr (G3) cim += cre;
}
template <bool G3>
__device__ __forceinline__ void csub_step(mf4& cre, mf4& cim, mf4& c2, cd v, cd t) {
    if constexpr (G3) {
        cre = __builtin_amdgcn_mfma_f64_16x16x4f64(-v.x, t.x, cre, 0, 0, 0);
        c2 = __builtin_amdgcn_mfma_f64_16x16x4f64(-v.y, t.y, c2, 0, 0, 0);
        cim = __builtin_amdgcn_mfma_f64_16x16x4f64(-(v.x + v.y), t.x - t.y, cim, 0, 0, 0);
    } else {
        cre = __builtin_amdgcn_mfma_f64_16x16x4f64(-v.x, t.x, cre, 0, 0, 0);
        cre = __builtin_amdgcn_mfma_f64_16x16x4f64(-v.y, t.y, cre, 0, 0, 0);
        cim = __builtin_amdgcn_mfma_f64_16x16x4f64(-v.y, t.x, cim, 0, 0, 0);
        cim = __builtin_amdgcn_mfma_f64_16x16x4f64(v.x, t.y, cim, 0, 0, 0);
    }
}
template <bool G3>
__device__ __forceinline__ cd csub_out(const mf4& cre, const mf4& cim, const mf4& c2, int q) {
    cd z;
    z.x = G3 ? cre[q] + c2[q] : cre[q];
    z.y = G3 ? cim[q] - cre[q] + c2[q] : cim[q];
    return z;
}

__device__ __forceinline__ cd cmk(double r, double i) { cd z; z.x = r; z.y = i; return z; }
__device__ __forceinline__ cd czero() { return cmk(0.0, 0.0); }
__device__ __forceinline__ cd cadd(cd a, cd b) { return cmk(a.x + b.x, a.y + b.y); }
__device__ __forceinline__ cd csub(cd a, cd b) { return cmk(a.x - b.x, a.y - b.y); }
__device__ __forceinline__ cd cconj(cd a) { return cmk(a.x, -a.y); }
__device__ __forceinline__ cd cscale(cd a, double s) { return cmk(a.x * s, a.y * s); }
__device__ __forceinline__ cd cmul(cd a, cd b) {
    return cmk(fma(a.x, b.x, -a.y * b.y), fma(a.x, b.y, a.y * b.x));
}
// a * conj(b)
__device__ __forceinline__ cd cmulc(cd a, cd b) {
    return cmk(fma(a.x, b.x, a.y * b.y), fma(a.y, b.x, -a.x * b.y));
}
// acc + a*b
__device__ __forceinline__ cd cfma(cd acc, cd a, cd b) {
    acc.x = fma(a.x, b.x, acc.x); acc.x = fma(-a.y, b.y, acc.x);
    acc.y = fma(a.x, b.y, acc.y); acc.y = fma(a.y, b.x, acc.y);
    return acc;
}
// acc + a*conj(b)
__device__ __forceinline__ cd cfmac(cd acc, cd a, cd b) {
    acc.x = fma(a.x, b.x, acc.x); acc.x = fma(a.y, b.y, acc.x);
    acc.y = fma(a.y, b.x, acc.y); acc.y = fma(-a.x, b.y, acc.y);
    return acc;
}
// acc + s*a  (s real)
__device__ __forceinline__ cd caxpy(cd acc, double s, cd a) {
    acc.x = fma(s, a.x, acc.x); acc.y = fma(s, a.y, acc.y); return acc;
}
__device__ __forceinline__ double cabs2(cd a) { return fma(a.x, a.x, a.y * a.y); }
// c ? a : b per component (a ternary on the HIP vector struct can go through scratch)
__device__ __forceinline__ cd csel(bool c, cd a, cd b) { return cmk(c ? a.x : b.x, c ? a.y : b.y); }

// exp(z) for z <= ~0 (z may be -inf).  Cody-Waite reduction z = k ln2 + r,
// |r| <= ln2/2, degree-12 Taylor polynomial in Horner form (truncation
// r^13/13! < 1.7e-16 relative), then 2^k by v_ldexp_f64 (exact; underflows to
// 0 below 2^-1074).  18 f64 VALU ops, no special-case branches: the E-step
// only ever evaluates non-positive log-weights.
__device__ __forceinline__ double fexp_neg(double z) {
    z = fmax(z, -745.5);
    const double kd = __builtin_rint(z * 1.4426950408889634074);
    double r = fma(-kd, 6.93147180559945286227e-01, z);
    r = fma(-kd, 2.31904681384629955842e-17, r);
    double p = 2.08767569878680989792e-09;          // 1/12!
    p = fma(p, r, 2.50521083854417187751e-08);      // 1/11!
    p = fma(p, r, 2.75573192239858906526e-07);      // 1/10!
    p = fma(p, r, 2.75573192239858906526e-06);      // 1/9!
    p = fma(p, r, 2.48015873015873015873e-05);      // 1/8!
    p = fma(p, r, 1.98412698412698412698e-04);      // 1/7!
    p = fma(p, r, 1.38888888888888888889e-03);      // 1/6!
    p = fma(p, r, 8.33333333333333333333e-03);      // 1/5!
    p = fma(p, r, 4.16666666666666666667e-02);      // 1/4!
    p = fma(p, r, 1.66666666666666666667e-01);      // 1/3!
    p = fma(p, r, 0.5);
    p = fma(p, r, 1.0);
    p = fma(p, r, 1.0);
    return __builtin_amdgcn_ldexp(p, (int)kd);
}

__device__ __forceinline__ void wave_sync() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

__device__ __forceinline__ double shfl_xor_d(double v, int m) { return __shfl_xor(v, m); }
// Wave-wide sum / max of a double without LDS permutes: DPP within each 16-lane row (quad_perm
// xor 1, xor 2, row_half_mirror, row_mirror: every lane then holds its row's value), then the
// four row values by v_readlane.  The result is wave-uniform.
template <int CTRL>
__device__ __forceinline__ double dpp_d(double v) {
    const long long b = __double_as_longlong(v);
    const int lo = __builtin_amdgcn_update_dpp(0, (int)b, CTRL, 0xF, 0xF, false);
    const int hi = __builtin_amdgcn_update_dpp(0, (int)(b >> 32), CTRL, 0xF, 0xF, false);
    return __longlong_as_double(((long long)hi << 32) | (unsigned)lo);
}
__device__ __forceinline__ double lane_d(double v, int l) {
    const long long b = __double_as_longlong(v);
    const int lo = __builtin_amdgcn_readlane((int)b, l);
    const int hi = __builtin_amdgcn_readlane((int)(b >> 32), l);
    return __longlong_as_double(((long long)hi << 32) | (unsigned)lo);
}
__device__ __forceinline__ double wave_sum_dpp(double v) {
    v += dpp_d<0xB1>(v);
    v += dpp_d<0x4E>(v);
    v += dpp_d<0x141>(v);
    v += dpp_d<0x140>(v);
    return (lane_d(v, 0) + lane_d(v, 16)) + (lane_d(v, 32) + lane_d(v, 48));
}
// First minimum of (d, i) over the wave (smallest d, ties to the smallest i), by the same
// DPP / readlane steps; exact comparisons, so the result is that of any reduction order.
template <int CTRL>
__device__ __forceinline__ void argmin_step(double& d, int& i) {
    const double od = dpp_d<CTRL>(d);
    const int oi = __builtin_amdgcn_update_dpp(0, i, CTRL, 0xF, 0xF, false);
    if (od < d || (od == d && oi < i)) { d = od; i = oi; }
}
__device__ __forceinline__ void wave_argmin_dpp(double& d, int& i) {
    argmin_step<0xB1>(d, i);
    argmin_step<0x4E>(d, i);
    argmin_step<0x141>(d, i);
    argmin_step<0x140>(d, i);
    double bd = lane_d(d, 0);
    int bi = __builtin_amdgcn_readlane(i, 0);
#pragma unroll
    for (int r = 16; r < 64; r += 16) {
        const double od = lane_d(d, r);
        const int oi = __builtin_amdgcn_readlane(i, r);
        if (od < bd || (od == bd && oi < bi)) { bd = od; bi = oi; }
    }
    d = bd;
    i = bi;
}
__device__ __forceinline__ double wave_min_dpp(double v) {
    v = fmin(v, dpp_d<0xB1>(v));
    v = fmin(v, dpp_d<0x4E>(v));
    v = fmin(v, dpp_d<0x141>(v));
    v = fmin(v, dpp_d<0x140>(v));
    return fmin(fmin(lane_d(v, 0), lane_d(v, 16)), fmin(lane_d(v, 32), lane_d(v, 48)));
}
__device__ __forceinline__ double wave_max_dpp(double v) {
    v = fmax(v, dpp_d<0xB1>(v));
    v = fmax(v, dpp_d<0x4E>(v));
    v = fmax(v, dpp_d<0x141>(v));
    v = fmax(v, dpp_d<0x140>(v));
    return fmax(fmax(lane_d(v, 0), lane_d(v, 16)), fmax(lane_d(v, 32), lane_d(v, 48)));
}
// a wave-uniform double moved to SGPRs (readfirstlane of both halves)
__device__ __forceinline__ double uniform_d(double v) {
    return __hiloint2double(__builtin_amdgcn_readfirstlane(__double2hiint(v)),
                            __builtin_amdgcn_readfirstlane(__double2loint(v)));
}
// ds_bpermute of a double from the lane whose byte address (4 * lane) is `addr`; with the
// address computed once, a butterfly step costs no VALU beyond the combine
__device__ __forceinline__ double bperm_d(double v, int addr) {
    const int lo = __builtin_amdgcn_ds_bpermute(addr, __double2loint(v));
    const int hi = __builtin_amdgcn_ds_bpermute(addr, __double2hiint(v));
    return __hiloint2double(hi, lo);
}

// 1/sqrt(x) for x > 0 in ~10 dependent VALU ops instead of the ~25 of the IEEE sqrt +
// division sequences (whose latency sets the pace of the column chain): exponent split,
// v_rsq_f32 seed on the mantissa, two f64 Newton steps (2^-24 -> 2^-48 -> ~1 ulp).
__device__ __forceinline__ double fast_rsqrt(double x) {
    const int e = __builtin_amdgcn_frexp_exp(x);          // x = m 2^e, m in [0.5, 1)
    const int h = e >> 1;
    const double xs = __builtin_amdgcn_ldexp(x, -2 * h);  // in [0.5, 2)
    double y = (double)__builtin_amdgcn_rsqf((float)xs);
    double r = fma(-xs * y, y, 1.0);
    y = fma(0.5 * y, r, y);
    r = fma(-xs * y, y, 1.0);
    y = fma(0.5 * y, r, y);
    return __builtin_amdgcn_ldexp(y, -h);
}
// The same from the FP64 hardware seed (v_rsq_f64, no exponent split or f32 round trip): five
// dependent ops instead of ten on the Cholesky pivot chain; two Newton steps as above.
__device__ __forceinline__ double fast_rsqrt64(double x) {
    double y = __builtin_amdgcn_rsq(x);
    double r = fma(-x * y, y, 1.0);
    y = fma(0.5 * y, r, y);
    r = fma(-x * y, y, 1.0);
    return fma(0.5 * y, r, y);
}


// ------------------------------------------------------------------ debug configuration
// A/B switches of the development runs (SBCE_* environment variables).  They exist only in the
// A/B build, libsbce_ab.so (compiled with SBCE_AB=1, the tests' and tools' cross-check library):
// there they are read ONCE when the library is loaded (api.hip) and again only through
// sbce_debug_reload_env(), and any result-affecting non-default value makes sbce_em /
// sbce_mstep / sbce_estep mark every trial SBCE_STATUS_DEBUG.  The product library libsbce.so
// (SBCE_AB=0) has no switch: g_debug is the compile-time default below, every selection on it
// folds away, and nothing reads the environment.
// Only the independent cross-check paths the tests compare against stay selectable; the
// measured-and-rejected schedules of earlier rounds live in git history.
#ifndef SBCE_AB
#define SBCE_AB 0
#endif
struct DebugConfig {
    bool estep_valu;     // SBCE_ESTEP_IMPL=valu   VALU E-step instead of the MFMA sweep
    bool estep_noprune;  // SBCE_ESTEP_PRUNE=0     no column-tile bounds
    bool estep_count;    // SBCE_ESTEP_COUNT=1     device counters (results unchanged)
    bool estep_nof32;    // SBCE_ESTEP_F32=0       no FP32 screen of the sweep's tile groups
    bool estep_nosphere; // SBCE_ESTEP_SPHERE=0    tile sweep only
    int sphere_budget;   // SBCE_SPHERE_BUDGET     path list cap per level (default 128)
    bool backsub_general;// SBCE_BACKSUB=1         the general back substitution at every shape
    bool chol_valu;      // SBCE_CHOL_IMPL=valu    VALU blocked Cholesky (L <= 1024)
    bool estep_nopair;   // SBCE_ESTEP_PAIR=0      no factorised-weight pass (estep_pair.hip)
    bool cplx3;          // SBCE_CPLX3=0           four real MFMAs per complex product (default: three, Gauss)
    bool mstep_nosmall;  // SBCE_MSTEP_SMALL=0     L <= 64: the batched build + panel Cholesky instead of
                         //                        the one-workgroup M-step (mstep_small.hip)
    bool small_valu;     // SBCE_MSTEP_SMALL=v     the 256-thread VALU-build kernel also at P <= 16
    bool small_v1;       // SBCE_MSTEP_SMALL=1     n_tx <= 2: the round-5 MFMA-build kernel instead of
                         //                        mstep_small2_kernel (A/B; not flagged)
    int small_stop;      // SBCE_SMALL_STOP=1|2|3  DIAGNOSTIC: the one-workgroup M-step stops after its
                         //                        build (1) / factorisation (2) / symbol staging
                         //                        without the build's arithmetic (3); results invalid
    bool small_col;      // SBCE_SMALL_SOLVE=col   n_tx <= 2 small M-step: the round-6 column-by-column
                         //                        solve instead of the 4-column-panel MFMA one
    char pm_impl;        // SBCE_PM_IMPL=wave      ZF/MMSE (n_tx <= 2) and PM (n_tx = 2, |A| = 1) E-steps
                         //                        one wave per symbol too; =t / =q the PM one thread /
                         //                        one quad per symbol at any size (all bitwise the
                         //                        same results; not flagged)
};
inline constexpr DebugConfig kDebugDefault = {false, false, false, false, false, 128, false, false,
                                              false, true, false, false, false, 0, false, 0};
#if SBCE_AB
extern DebugConfig g_debug;
#else
inline constexpr DebugConfig g_debug = kDebugDefault;
#endif
bool debug_nondefault();   // a result-affecting switch differs from its default

// ------------------------------------------------------------------ launch API
struct Problem {
    int B, NT, NR, P, Tp, Td, M, L, K;
    int pr;            // partition_r (PM E-step modes)
    double varn;
    double varx;       // Gaussian-prior E-step (SBCE_ESTEP_GAUSS)
};

struct EstepArgs {
    const cd* yd;      // [B][Td][NR]
    const cd* psid;    // [B][Td][P]
    const cd* theta;   // [B][K]
    const cd* cons;    // [M]
    cd* mom;           // [B][Td][NT + NT*NT]
    const int32_t* done;  // [B] or null
    int32_t* status;   // [B] or null (detector index flag)
    double* prep;      // [B*Td][estep_prep_stride] workspace of the MFMA sweep, or null
                       // (then the sweep kernel prepares each symbol itself)
    int32_t* list;     // [B*Td] symbols the sphere pass left to the sweep, 16 counters
                       // (0 listed, 1 grabbed by the sweep, 2 listed for the enumeration,
                       // 3 listed for the factorised-weight pass, 4 grabbed by it), [B*Td]
                       // symbols the tree pass left to the enumeration, 16 spare, [B*Td]
                       // symbols the enumeration left to the factorised-weight pass;
                       // null: no sphere
    double* tree;      // [B*Td][32] the sphere pass's per-symbol search-tree records
    const double* varn_t = nullptr;   // [B] per-trial noise variances (sbce_ptrs.varn_t), or null
    bool lists_zeroed = false;        // the 5 list counters after list[B*Td] are already 0 (zeroed
                                      // by em_init_kernel / the previous M-step's solve launch)
};

// The posterior constants of one noise variance v, in the operation order of the host's scalar
// path (the launchers' 1 / (varn varn), kSkipThr varn varn, 0.1 varn varn), so that a trial with
// varn_t[b] == dims.varn gets bitwise the constants of a scalar call.  kSkipThr = 50 (estep.hip).
struct TrialNoise {
    double inv_s2, thr_d, reg, s2;
};
__device__ __forceinline__ TrialNoise trial_noise(double v) {
    TrialNoise n;
    n.inv_s2 = 1.0 / (v * v);
    n.thr_d = 50.0 * v * v;
    n.reg = 0.1 * v * v;
    n.s2 = v * v;
    return n;
}
// A square M-QAM table as a K x K grid of real / imaginary levels (any table order), built once per
// block by grid_build (estep_pm.hip's nearest-point search, estep_pair.hip's NT = 2 factorised
// pass); K = 0: the table is not such a grid.
struct GridLds {
    double lre[8], lim[8];
    int idx[64];
    int K;                                          // 0: not a square grid, exhaustive scans
};

// Every thread of the block calls it (blockDim >= M).  Thread s < M places point s: its level
// index on each axis is (#points strictly below it) / K, valid when exactly K points share its
// level and no other point equals it -- then the K x K cells are filled one-to-one.
__device__ inline void grid_build(const cd* cons, int M, GridLds* g) {
    const int tid = threadIdx.x;
    int K = 0;
    while (K * K < M) ++K;
    const bool sq = K * K == M && K <= 8;
    bool ok = true;
    if (sq && tid < M) {
        const cd v = cons[tid];
        int lt_x = 0, eq_x = 0, lt_y = 0, eq_y = 0, same = 0;
        for (int s = 0; s < M; ++s) {
            const cd u = cons[s];
            lt_x += u.x < v.x;
            eq_x += u.x == v.x;
            lt_y += u.y < v.y;
            eq_y += u.y == v.y;
            same += (u.x == v.x) && (u.y == v.y);
        }
        ok = eq_x == K && eq_y == K && same == 1 && lt_x % K == 0 && lt_y % K == 0;
        if (ok) {
            const int ir = lt_x / K, ii = lt_y / K;
            g->lre[ir] = v.x;
            g->lim[ii] = v.y;
            g->idx[ir * K + ii] = tid;
        }
    }
    const bool all = __syncthreads_and(ok ? 1 : 0) != 0;
    if (tid == 0) g->K = (sq && all) ? K : 0;
    __syncthreads();
}

constexpr int kTreeRecDoubles = 32;   // (word 31: the factorised-weight pass's screen)
constexpr int kEstepListCnt = 16;      // int32 counters after the sweep's list
// the factorised-weight pass (estep_pair.hip) takes a symbol whose range D is at most this
constexpr double kPairDmax = 640.0;

// Internal solve mode of the min-norm solve's second factorisation (C = G^H G, minnorm.hip):
// a pivot at or below its threshold is CLAMPED there (C is HPD by construction, so the clamp
// never meets a non-PSD Schur complement).  R's own factorisations never clamp: in every
// public mode a pivot at or below 1e-14 max diag R is dropped (see SBCE_SOLVE_CHOL, sbce.h).
constexpr int kSolveClampHpd = 16;

struct MstepArgs {
    const cd* yd;
    const cd* yp;      // [B][Tp][NR]
    const cd* psid;
    const cd* up;      // [B][Tp][L]
    const cd* mom;
    cd* R;             // [B][L][L]
    cd* rhs;           // [B][L][NR]
    cd* theta;         // [B][K]
    int32_t* status;   // [B] or null
    const int32_t* done;
    int solve_mode;
    int nbatch;        // B (kernels whose grid is padded past the batch)
    // MFMA R build (NT in {4, 8}) workspace
    cd* ppsi;          // [B][Tp][P]  pilot phases psi' (Kronecker factor of u_p)
    cd* pS;            // [B][Tp][NT*NT] pilot x' x'^H
    int32_t* pflag;    // [B] u_p of the trial is not a Kronecker product (set by pilot_factor)
    cd* prhs;          // [B][L][NR] pilot part of B^H, sum_p u_p y_p (set by pilot_factor; null:
                       // not kept, the B^H kernel sums the pilots itself)
    const int32_t* gate;  // VALU build: only trials with gate[b] != 0 (null: all trials)
    // tiled factorisation workspace (L > 512, and the min-norm solve at every L)
    double* tol;       // [B]     pivot threshold
    cd* winv;          // [B][64][64] inverse of the current diagonal tile
    // min-norm solve (SBCE_SOLVE_MINNORM, minnorm.hip) workspace
    cd* gram;          // [B][L][L]  C = G^H G of the rank-cut factor G (lower triangle)
    cd* grhs;          // [B][L][NR] G^H B^H, then the solves with C in place
    int32_t* act;      // [B]  active extent: columns of G past act[b] are all dropped
    double* tol2;      // [B]  pivot threshold of C's Cholesky
    double* dvec;      // [B][L] diagonal of R's Schur complement (left-looking early exit)
    cd* mnr;           // [B][L][NR] min-norm refinement: the residual b - G G^H x0
    int32_t* mnskip;   // [B] min-norm refinement: 1 = the trial needs no refinement step
    // status bit a clamped pivot sets: NONHPD for R; RANK for the min-norm solve's C = G^H G
    // (HPD by construction: a clamp there means the kept subspace is too ill-conditioned for
    // the normal equations to hold lstsq's accuracy)
    int clamp_status = SBCE_STATUS_NONHPD;
    // the oracle early stop folded into the M-step launch (mstep_small2_kernel; null: not folded)
    const cd* h_true = nullptr;   // [B][K]
    int32_t* done_w = nullptr;    // [B] set when |‖theta‖ - ‖h‖| < 1 after iteration it > 0
    int32_t* iters_done = nullptr;
    int it = 0;
    int32_t* zero_cnt = nullptr;  // the small solve launch zeroes these 5 E-step list counters
};

// Per-trial extents of one tiled-factorisation launch sequence (mstep_large.hip): column
// blocks at or past col[b] and row tiles at or past row[b] are skipped (null: L); fwd = 0
// leaves the right-hand side untouched (no fused forward substitution).
struct TileExt {
    const int32_t* col;
    const int32_t* row;
    int fwd;
};

hipError_t launch_estep(const Problem& pb, const EstepArgs& a, int mode, hipStream_t s);
hipError_t launch_estep_pm(const Problem& pb, const EstepArgs& a, int mode, int partition_r,
                           hipStream_t s);
bool estep_pm_supported(const Problem& pb, int partition_r, int mode);
bool estep_supported(const Problem& pb, int mode);
int estep_prep_stride(const Problem& pb);   // doubles per symbol, 0 if no MFMA sweep
// pilots_factored: launch_pilot_factor already ran for these u_p (ppsi, pS, pflag valid)
hipError_t launch_mstep_build(const Problem& pb, const MstepArgs& a, hipStream_t s,
                              bool pilots_factored = false);
hipError_t launch_chol_solve(const Problem& pb, const MstepArgs& a, hipStream_t s);
bool chol_supported(const Problem& pb);
// L <= 64 (n_tx not 4, 8), CHOL / CHOL_DROP: build + solve of one trial in one workgroup
// (mstep_small.hip); write_sys also stores R and B^H in a.R / a.rhs (sbce_mstep's outputs)
bool mstep_small_supported(const Problem& pb, int solve_mode);
bool mstep_small2_selected(const Problem& pb);   // the launch folds the early stop (a.h_true)
hipError_t small_debug_clock(unsigned long long* out48);   // SBCE_SMALL_STOP=4 stamps
hipError_t launch_mstep_small(const Problem& pb, const MstepArgs& a, bool write_sys, hipStream_t s);
int chol_debug_skip_mask();
constexpr int kLargeL = 512;   // L above this: tiled build + blocked right-looking Cholesky
constexpr int kMaxL = 8192;    // largest supported L (R alone is 1 GiB per trial there)
bool rbuild_herm_supported(const Problem& pb);   // MFMA build of the Hermitian R: NT in {4, 8}
// DIAGNOSTIC: HIP-event timing of the L <= 512 Cholesky's update / factor / back-substitution
// launches (mode 1 arms it; mode 0 returns {ms x 3, launches x 3} in out6)
hipError_t chol_debug_timing(int mode, double* out6);
hipError_t launch_pilot_factor(const Problem& pb, const MstepArgs& a, hipStream_t s);
hipError_t launch_rbuild_herm(const Problem& pb, const MstepArgs& a, hipStream_t s);
hipError_t launch_chol_large(const Problem& pb, const MstepArgs& a, hipStream_t s);
hipError_t launch_diag_tol(const Problem& pb, const MstepArgs& a, hipStream_t s);  // a.tol[b]
hipError_t launch_chol_tile(const Problem& pb, const MstepArgs& a, int k0, int w, const int32_t* ext,
                            hipStream_t s);
// one column block k of the tiled right-looking factorisation: diagonal tile, its inverse and
// the TRSM tiles below it (the trailing updates are launch_tile_factor's)
hipError_t launch_tile_factor_step(const Problem& pb, const MstepArgs& a, int k, const TileExt& e,
                                   hipStream_t s);
// the whole tiled factorisation, trailing updates grouped (mstep_large.hip); act_check, when
// given, runs before each column block (the min-norm early exit)
hipError_t launch_tile_factor(const Problem& pb, const MstepArgs& a, const TileExt& e,
                              hipError_t (*act_check)(const Problem&, const MstepArgs&, int, hipStream_t),
                              hipStream_t s);
// DIAGNOSTIC: out[3b..3b+2] = (active extent, rank of G, refinement ran) of the last min-norm solve
hipError_t launch_minnorm_rank(const Problem& pb, const MstepArgs& a, int32_t* out, hipStream_t s);
// L^H x = y on a.rhs by 64-column blocks (theta = conj(x) written when a.theta != null)
hipError_t launch_tile_back(const Problem& pb, const MstepArgs& a, const int32_t* ext, hipStream_t s);
// minimum-norm solve (SBCE_SOLVE_MINNORM, minnorm.hip): R, rhs built; writes theta
hipError_t launch_minnorm(const Problem& pb, const MstepArgs& a, hipStream_t s);
hipError_t chol_debug_clock(unsigned long long* out);   // diagnostic (SBCE_CHOL_SKIP & 64)
hipError_t chol_debug_clock_reset();
void chol_debug_skip(int mask);   // diagnostic phase-skip mask (results flagged SBCE_STATUS_DEBUG)
int chol_debug_skip_mask();       // the current mask (process-wide, every stream)
hipError_t launch_decisions(const Problem& pb, const cd* mom, cd* xdest, hipStream_t s);
hipError_t launch_sup_shift_y(const Problem& pb, const cd* yd, const cd* psid, const cd* theta,
                              const cd* xsup, cd* yout, const int32_t* done, hipStream_t s);
hipError_t launch_sup_shift_mom(const Problem& pb, cd* mom, const cd* xsup, const int32_t* done,
                                hipStream_t s);
hipError_t launch_ser(const Problem& pb, const cd* xdest, const cd* xtrue, double* out,
                      hipStream_t s);
hipError_t estep_debug_mfma(unsigned long long* out, int reset);   // SBCE_ESTEP_COUNT=1
hipError_t estep_debug_sphere(unsigned long long* out3, int reset);   // [enumerated, listed, single path]
// factorised-weight soft E-step (estep_pair.hip) for the sphere pass's listed symbols
bool estep_pair_supported(const Problem& pb, int mode);
hipError_t launch_estep_pair(const Problem& pb, const EstepArgs& a, int stride, int count, int mode,
                             hipStream_t s);
hipError_t estep_debug_pair(unsigned long long* out, int reset);      // SBCE_ESTEP_COUNT=1
hipError_t launch_gauss_rank1(const Problem& pb, const MstepArgs& a, hipStream_t s);
hipError_t launch_gauss_expand(const Problem& pb, const cd* theta, cd* out, hipStream_t s);
hipError_t launch_nmse(const Problem& pb, const cd* theta, const cd* h, double* out,
                       hipStream_t s);
hipError_t launch_llf(const Problem& pb, const cd* theta, const cd* yp, const cd* up,
                      const cd* yd, const cd* psid, const cd* xd, double* llf, int iters,
                      int it, const int32_t* done, const double* varn_t, hipStream_t s);
// sbce_em's start in one launch: done[b] = 0, status[b] = status_value, and (cnt) 5 counters = 0
hipError_t launch_em_init(int B, int32_t* done, int32_t* status, int status_value, int32_t* cnt,
                          hipStream_t s);
hipError_t launch_early_stop(const Problem& pb, const cd* theta, const cd* h,
                             int32_t* done, int32_t* iters_done, int it, hipStream_t s);

}  // namespace sbce
