// extern "C" entry points of libsbce.so (declared in include/sbce.h).
//
// The EM loop replaces em() of "Proposed method/Proposed_method_NMSEvsTp.py":50-83
// for a whole batch of Monte-Carlo trials: per iteration one E-step launch over
// every (trial, symbol), one normal-equation build and one batched Cholesky
// solve, all stream-ordered, with no host synchronisation and no allocation.
#include <stdlib.h>
#include <string.h>

#include "sbce_internal.h"

using namespace sbce;

namespace sbce {

#if SBCE_AB
DebugConfig g_debug;

namespace {
constexpr int kSphereBudgetMax = 256;      // estep.hip kBfsPmax

void read_debug_env(DebugConfig& c) {
    c = kDebugDefault;
    auto env = [](const char* n) { const char* v = getenv(n); return (v && v[0]) ? v : nullptr; };
    const char* v;
    if ((v = env("SBCE_ESTEP_IMPL"))) c.estep_valu = v[0] == 'v';
    if ((v = env("SBCE_ESTEP_PRUNE"))) c.estep_noprune = v[0] == '0';
    if ((v = env("SBCE_ESTEP_COUNT"))) c.estep_count = v[0] == '1';
    if ((v = env("SBCE_ESTEP_F32"))) c.estep_nof32 = v[0] == '0';
    if ((v = env("SBCE_ESTEP_SPHERE"))) c.estep_nosphere = v[0] == '0';
    if ((v = env("SBCE_SPHERE_BUDGET"))) {
        const int bu = atoi(v);
        c.sphere_budget = bu < 1 ? 1 : (bu > kSphereBudgetMax ? kSphereBudgetMax : bu);
    }
    if ((v = env("SBCE_BACKSUB"))) c.backsub_general = v[0] == '1';
    if ((v = env("SBCE_CHOL_IMPL"))) c.chol_valu = v[0] == 'v';
    if ((v = env("SBCE_ESTEP_PAIR"))) c.estep_nopair = v[0] == '0';
    if ((v = env("SBCE_CPLX3"))) c.cplx3 = v[0] != '0';
    if ((v = env("SBCE_MSTEP_SMALL"))) {
        c.mstep_nosmall = v[0] == '0';
        c.small_valu = v[0] == 'v';
        c.small_v1 = v[0] == '1';
    }
    if ((v = env("SBCE_PM_IMPL"))) c.pm_impl = (v[0] == 'w' || v[0] == 't' || v[0] == 'q') ? v[0] : 0;
    if ((v = env("SBCE_SMALL_SOLVE"))) c.small_col = v[0] == 'c';
    if ((v = env("SBCE_SMALL_STOP"))) c.small_stop = (v[0] >= '1' && v[0] <= '4') ? v[0] - '0' : 0;
}

__attribute__((constructor)) void load_debug_env() { read_debug_env(g_debug); }
}  // namespace

bool debug_nondefault() {
    const DebugConfig& c = g_debug;
    const DebugConfig& d = kDebugDefault;
    return c.estep_valu != d.estep_valu || c.estep_noprune != d.estep_noprune ||
           c.estep_nof32 != d.estep_nof32 ||
           c.estep_nosphere != d.estep_nosphere || c.sphere_budget != d.sphere_budget ||
           c.backsub_general != d.backsub_general || c.chol_valu != d.chol_valu ||
           c.estep_nopair != d.estep_nopair || c.cplx3 != d.cplx3 ||
           c.mstep_nosmall != d.mstep_nosmall || c.small_stop != d.small_stop ||
           c.small_valu != d.small_valu || c.small_v1 != d.small_v1 || c.small_col != d.small_col ||
           (chol_debug_skip_mask() & 31);
}
#else
bool debug_nondefault() { return false; }   // the product build has no switch
#endif

}  // namespace sbce

namespace {

constexpr size_t kAlign = 256;
size_t align_up(size_t v) { return (v + kAlign - 1) / kAlign * kAlign; }

struct Carve {
    size_t mom, R, rhs, done, ysh, prep, list, tree, tol, winv, ppsi, pS, pflag, prhs, gram, grhs,
        act, tol2, dvec, mnr, mnskip, total;
    bool has_prep, has_prhs, has_winv, has_mn;
};

constexpr int kAnySolve = -1;            // carve for every solve mode (sbce_workspace_bytes)

bool make_problem(const sbce_dims* d, Problem& pb) {
    if (!d) return false;
    if (d->batch < 0 || d->n_tx < 1 || d->n_rx < 1 || d->n_psi < 1 || d->t_p < 0 || d->t_d < 1 ||
        d->m < 2 || d->partition_r < 0 || !(d->varn > 0.0))
        return false;
    if (d->n_tx > 8 || d->n_rx > 8) return false;
    pb.B = d->batch; pb.NT = d->n_tx; pb.NR = d->n_rx; pb.P = d->n_psi;
    pb.Tp = d->t_p; pb.Td = d->t_d; pb.M = d->m; pb.varn = d->varn; pb.pr = d->partition_r;
    pb.varx = d->varx;
    pb.L = pb.P * pb.NT;
    pb.K = pb.L * pb.NR;
    return true;
}

// Workspace layout for `solve` (SBCE_SOLVE_*, or kAnySolve): the regions only the tiled
// factorisation (L > 512) or the min-norm solve use are appended last and carved only when that
// solve can run, so a CHOL workspace at L <= 512 holds no Gram matrix.  Offsets of every region
// that is carved do not depend on `solve`.
Carve carve(const Problem& pb, int solve = kAnySolve) {
    Carve c;
    const size_t MS = (size_t)pb.NT + (size_t)pb.NT * pb.NT;
    c.mom = 0;
    c.R = align_up(c.mom + (size_t)pb.B * pb.Td * MS * sizeof(cd));
    c.rhs = align_up(c.R + (size_t)pb.B * pb.L * pb.L * sizeof(cd));
    c.done = align_up(c.rhs + (size_t)pb.B * pb.L * pb.NR * sizeof(cd));
    c.ysh = align_up(c.done + (size_t)pb.B * sizeof(int32_t));         // superimposed pilots
    c.prep = align_up(c.ysh + (size_t)pb.B * pb.Td * pb.NR * sizeof(cd));   // MFMA sweep prep
    const int ps = estep_prep_stride(pb);
    c.has_prep = ps > 0;
    c.list = align_up(c.prep + (size_t)pb.B * pb.Td * ps * sizeof(double));
    c.tree = align_up(c.list + (3 * (size_t)pb.B * pb.Td + 2 * kEstepListCnt) * sizeof(int32_t));
    c.tol = c.has_prep ? align_up(c.tree + (size_t)pb.B * pb.Td * kTreeRecDoubles * sizeof(double))
                       : c.list;
    c.ppsi = c.pS = c.pflag = c.winv = c.tol;
    c.total = c.tol;
    if (rbuild_herm_supported(pb)) {         // MFMA R build: Kronecker-factored pilots
        c.ppsi = c.total;
        c.pS = align_up(c.ppsi + (size_t)pb.B * pb.Tp * pb.P * sizeof(cd));
        c.pflag = align_up(c.pS + (size_t)pb.B * pb.Tp * pb.NT * pb.NT * sizeof(cd));
        c.total = align_up(c.pflag + (size_t)pb.B * sizeof(int32_t));
    }
    // the pilot part of B^H is fixed across iterations: kept once per run for the L <= 512
    // B^H kernel (mstep.hip rhs_dma_kernel), which then reads L*NR values instead of u_p, y_p
    c.has_prhs = rbuild_herm_supported(pb) && pb.L <= kLargeL;
    c.prhs = c.total;
    if (c.has_prhs) c.total = align_up(c.prhs + (size_t)pb.B * pb.L * pb.NR * sizeof(cd));
    c.tol = c.total;                         // per-trial pivot threshold
    c.winv = align_up(c.tol + (size_t)pb.B * sizeof(double));
    c.total = c.winv;
    c.has_mn = solve == kAnySolve || solve == SBCE_SOLVE_MINNORM;
    // tiled factorisation (L > 512, and the min-norm solve at every L): diagonal-tile inverse
    c.has_winv = c.has_mn || pb.L > kLargeL;
    c.gram = c.winv;
    if (c.has_winv) c.total = c.gram = align_up(c.winv + (size_t)pb.B * 64 * 64 * sizeof(cd));
    c.grhs = c.act = c.tol2 = c.dvec = c.mnr = c.mnskip = c.total;
    if (c.has_mn) {
        // min-norm solve (minnorm.hip): Gram matrix C = G^H G, its right-hand sides, extents
        c.grhs = align_up(c.gram + (size_t)pb.B * pb.L * pb.L * sizeof(cd));
        c.act = align_up(c.grhs + (size_t)pb.B * pb.L * pb.NR * sizeof(cd));
        c.tol2 = align_up(c.act + (size_t)pb.B * sizeof(int32_t));
        c.dvec = align_up(c.tol2 + (size_t)pb.B * sizeof(double));
        // one refinement step on the kept subspace: residual and per-trial gate
        c.mnr = align_up(c.dvec + (size_t)pb.B * pb.L * sizeof(double));
        c.mnskip = align_up(c.mnr + (size_t)pb.B * pb.L * pb.NR * sizeof(cd));
        c.total = align_up(c.mnskip + (size_t)pb.B * sizeof(int32_t));
    }
    return c;
}

int hip_rc(hipError_t e) { return e == hipSuccess ? SBCE_OK : SBCE_EHIP; }

// The launchers check their kernels with hipGetLastError(), which reports the last error of ANY
// HIP call on this host thread until it is read.  A caller's earlier failed or "not ready" call
// (e.g. an event query by the framework that owns the buffers) must not be reported as a failure
// of this library's launches: every entry point that launches clears it first.
void clear_stale_error() { (void)hipGetLastError(); }

void set_large(MstepArgs& ma, char* ws, const Carve& c) {
    ma.tol = (double*)(ws + c.tol);
    ma.winv = c.has_winv ? (cd*)(ws + c.winv) : nullptr;
    ma.ppsi = (cd*)(ws + c.ppsi);
    ma.pS = (cd*)(ws + c.pS);
    ma.pflag = (int32_t*)(ws + c.pflag);
    ma.prhs = c.has_prhs ? (cd*)(ws + c.prhs) : nullptr;
    ma.gate = nullptr;
    ma.gram = c.has_mn ? (cd*)(ws + c.gram) : nullptr;
    ma.grhs = c.has_mn ? (cd*)(ws + c.grhs) : nullptr;
    ma.act = c.has_mn ? (int32_t*)(ws + c.act) : nullptr;
    ma.tol2 = c.has_mn ? (double*)(ws + c.tol2) : nullptr;
    ma.dvec = c.has_mn ? (double*)(ws + c.dvec) : nullptr;
    ma.mnr = c.has_mn ? (cd*)(ws + c.mnr) : nullptr;
    ma.mnskip = c.has_mn ? (int32_t*)(ws + c.mnskip) : nullptr;
}

bool aligned16(const void* p) { return ((uintptr_t)p & 15) == 0; }

// per-trial status starts at 0, or at SBCE_STATUS_DEBUG while a result-affecting debug switch
// (DebugConfig) is active
int status_init(int32_t* status, int B, hipStream_t s) {
    if (!status) return SBCE_OK;
    const unsigned v = debug_nondefault() ? SBCE_STATUS_DEBUG : 0u;
    return hipMemsetD32Async((hipDeviceptr_t)status, v, (size_t)B, s) == hipSuccess ? SBCE_OK
                                                                                    : SBCE_EHIP;
}

int check_ptrs(const sbce_ptrs* p, const Problem& pb, bool need_ws, int solve = kAnySolve) {
    if (!p) return SBCE_EINVAL;
    const void* req[] = {p->y_d, p->y_p, p->psi_d, p->u_p, p->cons, p->theta};
    for (const void* q : req)
        if (!q || !aligned16(q)) return SBCE_EINVAL;
    if (pb.Tp == 0) { /* pilots optional */ }
    if (p->varn_t && ((uintptr_t)p->varn_t & 7)) return SBCE_EINVAL;
    if (need_ws) {
        if (!p->workspace || !aligned16(p->workspace)) return SBCE_EINVAL;
        if (p->workspace_bytes < carve(pb, solve).total) return SBCE_EWORKSPACE;
    }
    return SBCE_OK;
}

}  // namespace

extern "C" {

int sbce_abi_version(void) { return SBCE_ABI_VERSION; }

const char* sbce_strerror(int code) {
    switch (code) {
        case SBCE_OK: return "ok";
        case SBCE_EINVAL: return "invalid argument (dims, null or misaligned pointer)";
        case SBCE_EUNSUPPORTED: return "shape not supported by the compiled kernel set";
        case SBCE_EHIP: return "HIP launch failed";
        case SBCE_EWORKSPACE: return "workspace too small";
    }
    return "unknown error";
}

int sbce_workspace_bytes(const sbce_dims* d, size_t* bytes) {
    Problem pb;
    if (!bytes || !make_problem(d, pb)) return SBCE_EINVAL;
    *bytes = carve(pb).total;
    return SBCE_OK;
}

int sbce_workspace_bytes_solve(const sbce_dims* d, int solve_mode, size_t* bytes) {
    Problem pb;
    if (!bytes || !make_problem(d, pb)) return SBCE_EINVAL;
    if (solve_mode != SBCE_SOLVE_CHOL && solve_mode != SBCE_SOLVE_CHOL_DROP &&
        solve_mode != SBCE_SOLVE_MINNORM)
        return SBCE_EINVAL;
    *bytes = carve(pb, solve_mode).total;
    return SBCE_OK;
}

int sbce_em(const sbce_dims* d, const sbce_ptrs* p, int iters, int estep_mode, int solve_mode,
            void* hip_stream) {
    clear_stale_error();
    Problem pb;
    if (!make_problem(d, pb) || iters < 0) return SBCE_EINVAL;
    if (!estep_supported(pb, estep_mode) || !chol_supported(pb)) return SBCE_EUNSUPPORTED;
    if (solve_mode != SBCE_SOLVE_CHOL && solve_mode != SBCE_SOLVE_CHOL_DROP &&
        solve_mode != SBCE_SOLVE_MINNORM)
        return SBCE_EINVAL;
    int rc = check_ptrs(p, pb, true, solve_mode);
    if (rc) return rc;
    if (p->llf && !p->x_d_true) return SBCE_EINVAL;
    const bool gauss = estep_mode == SBCE_ESTEP_GAUSS;
    if (gauss && !(pb.varx > 0.0)) return SBCE_EINVAL;
    const bool hard = estep_mode == SBCE_ESTEP_HARD || estep_mode == SBCE_ESTEP_ZF ||
                      estep_mode == SBCE_ESTEP_MMSE;
    if (p->x_dest && (!hard || !aligned16(p->x_dest))) return SBCE_EINVAL;
    if (p->x_sup && ((estep_mode != SBCE_ESTEP_SOFT && estep_mode != SBCE_ESTEP_HARD) ||
                     !aligned16(p->x_sup)))
        return SBCE_EINVAL;
    if (pb.B == 0 || iters == 0) return SBCE_OK;
    hipStream_t s = (hipStream_t)hip_stream;
    const Carve c = carve(pb, solve_mode);
    char* ws = (char*)p->workspace;
    int32_t* done = (int32_t*)(ws + c.done);
    const bool early = p->h_true != nullptr;
    // L <= 64: the whole M-step in one launch (BASELINE cfg 5: L = 32)
    const bool small = mstep_small_supported(pb, solve_mode) && !(gauss && pb.NR == 1);
    // n_tx <= 2 small path: its solve launch zeroes the E-step's list counters for the next
    // iteration, em_init_kernel for the first -- no counter memset per E-step
    const bool small2 = small && mstep_small2_selected(pb);
    int32_t* list_cnt = c.has_prep ? (int32_t*)(ws + c.list) + (size_t)pb.B * pb.Td : nullptr;
    if ((rc = hip_rc(launch_em_init(pb.B, done, p->status, debug_nondefault() ? SBCE_STATUS_DEBUG : 0,
                                    small2 ? list_cnt : nullptr, s))))
        return rc;

    EstepArgs ea;
    ea.yd = (const cd*)p->y_d; ea.psid = (const cd*)p->psi_d; ea.theta = (const cd*)p->theta;
    ea.cons = (const cd*)p->cons; ea.mom = (cd*)(ws + c.mom); ea.done = early ? done : nullptr;
    ea.status = p->status;
    ea.varn_t = p->varn_t;
    ea.prep = c.has_prep ? (double*)(ws + c.prep) : nullptr;
    ea.list = c.has_prep ? (int32_t*)(ws + c.list) : nullptr;
    ea.tree = c.has_prep ? (double*)(ws + c.tree) : nullptr;
    ea.lists_zeroed = small2 && list_cnt != nullptr;
    MstepArgs ma;
    ma.yd = ea.yd; ma.yp = (const cd*)p->y_p; ma.psid = ea.psid; ma.up = (const cd*)p->u_p;
    ma.mom = ea.mom; ma.R = (cd*)(ws + c.R); ma.rhs = (cd*)(ws + c.rhs); ma.theta = (cd*)p->theta;
    ma.status = p->status; ma.done = ea.done; ma.solve_mode = solve_mode; ma.nbatch = pb.B;
    set_large(ma, ws, c);

    EstepArgs eas = ea;                      // superimposed pilots: E-step on y - H x_p
    if (p->x_sup) eas.yd = (const cd*)(ws + c.ysh);
    // the Kronecker factors of the pilot regressors do not change across iterations
    const bool prefactor = rbuild_herm_supported(pb);
    if (prefactor && (rc = hip_rc(launch_pilot_factor(pb, ma, s)))) return rc;
    // the LLF kernel reads theta before the stop decision of the same iteration: no fold with it
    const bool fold_stop = small2 && early && !p->llf;
    for (int it = 0; it < iters; ++it) {
        if (p->x_sup) {
            if ((rc = hip_rc(launch_sup_shift_y(pb, ea.yd, ea.psid, ea.theta, (const cd*)p->x_sup,
                                                (cd*)(ws + c.ysh), ea.done, s))))
                return rc;
            if ((rc = hip_rc(launch_estep(pb, eas, estep_mode, s)))) return rc;
            if ((rc = hip_rc(launch_sup_shift_mom(pb, ea.mom, (const cd*)p->x_sup, ea.done, s))))
                return rc;
        } else {
            if ((rc = hip_rc(launch_estep(pb, ea, estep_mode, s)))) return rc;
        }
        if (small) {
            MstepArgs ms = ma;
            if (ea.lists_zeroed) ms.zero_cnt = list_cnt;
            if (fold_stop) {                 // the oracle early stop rides in the M-step launch
                ms.h_true = (const cd*)p->h_true;
                ms.done_w = done;
                ms.iters_done = p->iters_done;
                ms.it = it;
            }
            if ((rc = hip_rc(launch_mstep_small(pb, ms, false, s)))) return rc;
        } else {
            if ((rc = hip_rc(launch_mstep_build(pb, ma, s, prefactor)))) return rc;
            // Gaussian prior, n_rx = 1: the reference's all-ones covariance term stays in A
            // (MIMO_Gaussian_proposed.py:73-76): R += c 1 1^T
            if (gauss && pb.NR == 1 && (rc = hip_rc(launch_gauss_rank1(pb, ma, s)))) return rc;
            if ((rc = hip_rc(launch_chol_solve(pb, ma, s)))) return rc;
        }
        if (p->llf &&
            (rc = hip_rc(launch_llf(pb, ma.theta, ma.yp, ma.up, ma.yd, ma.psid,
                                    (const cd*)p->x_d_true, p->llf, iters, it, ea.done, p->varn_t,
                                    s))))
            return rc;
        if (early && !fold_stop &&
            (rc = hip_rc(launch_early_stop(pb, ma.theta, (const cd*)p->h_true, done, p->iters_done,
                                           it, s))))
            return rc;
    }
    if (p->x_dest && (rc = hip_rc(launch_decisions(pb, ea.mom, (cd*)p->x_dest, s)))) return rc;
    if (!early && p->iters_done) {
        // every trial ran all iterations: fill with `iters` via a tiny host-free memset pattern
        // (int32 fill is done on device by hipMemsetD32Async)
        if (hipMemsetD32Async((hipDeviceptr_t)p->iters_done, iters, (size_t)pb.B, s) != hipSuccess)
            return SBCE_EHIP;
    }
    return SBCE_OK;
}

int sbce_estep(const sbce_dims* d, const sbce_ptrs* p, int estep_mode, void* moments,
               void* hip_stream) {
    clear_stale_error();
    Problem pb;
    if (!make_problem(d, pb)) return SBCE_EINVAL;
    int rc = check_ptrs(p, pb, false);
    if (rc) return rc;
    if (!moments || !aligned16(moments)) return SBCE_EINVAL;
    if (estep_mode == SBCE_ESTEP_GAUSS && !(pb.varx > 0.0)) return SBCE_EINVAL;
    if (!estep_supported(pb, estep_mode)) return SBCE_EUNSUPPORTED;
    if (pb.B == 0) return SBCE_OK;
    if ((rc = status_init(p->status, pb.B, (hipStream_t)hip_stream))) return rc;
    EstepArgs ea;
    ea.yd = (const cd*)p->y_d; ea.psid = (const cd*)p->psi_d; ea.theta = (const cd*)p->theta;
    ea.cons = (const cd*)p->cons; ea.mom = (cd*)moments; ea.done = nullptr;
    ea.status = p->status;
    ea.varn_t = p->varn_t;
    ea.prep = nullptr;               // workspace optional here: use it when it is large enough
    ea.list = nullptr;
    ea.tree = nullptr;
    if (p->workspace && aligned16(p->workspace)) {
        const Carve c = carve(pb, SBCE_SOLVE_CHOL);      // the E-step regions come first
        if (c.has_prep && p->workspace_bytes >= c.total) {
            ea.prep = (double*)((char*)p->workspace + c.prep);
            ea.list = (int32_t*)((char*)p->workspace + c.list);
            ea.tree = (double*)((char*)p->workspace + c.tree);
        }
    }
    return hip_rc(launch_estep(pb, ea, estep_mode, (hipStream_t)hip_stream));
}

int sbce_mstep(const sbce_dims* d, const sbce_ptrs* p, const void* moments, int solve_mode,
               void* r_out, void* rhs_out, void* hip_stream) {
    clear_stale_error();
    Problem pb;
    if (!make_problem(d, pb)) return SBCE_EINVAL;
    if (!chol_supported(pb)) return SBCE_EUNSUPPORTED;
    if (solve_mode != SBCE_SOLVE_CHOL && solve_mode != SBCE_SOLVE_CHOL_DROP &&
        solve_mode != SBCE_SOLVE_MINNORM)
        return SBCE_EINVAL;
    int rc = check_ptrs(p, pb, true, solve_mode);
    if (rc) return rc;
    if (!moments) return SBCE_EINVAL;
    if (pb.B == 0) return SBCE_OK;
    hipStream_t s = (hipStream_t)hip_stream;
    const Carve c = carve(pb, solve_mode);
    char* ws = (char*)p->workspace;
    if ((rc = status_init(p->status, pb.B, s))) return rc;
    MstepArgs ma;
    ma.yd = (const cd*)p->y_d; ma.yp = (const cd*)p->y_p; ma.psid = (const cd*)p->psi_d;
    ma.up = (const cd*)p->u_p; ma.mom = (const cd*)moments; ma.R = (cd*)(ws + c.R);
    ma.rhs = (cd*)(ws + c.rhs); ma.theta = (cd*)p->theta; ma.status = p->status; ma.done = nullptr;
    ma.solve_mode = solve_mode; ma.nbatch = pb.B;
    set_large(ma, ws, c);
    const bool small = mstep_small_supported(pb, solve_mode);
    if (small) {
        if ((rc = hip_rc(launch_mstep_small(pb, ma, r_out || rhs_out, s)))) return rc;
    } else if ((rc = hip_rc(launch_mstep_build(pb, ma, s)))) {
        return rc;
    }
    if (r_out &&
        hipMemcpyAsync(r_out, ma.R, (size_t)pb.B * pb.L * pb.L * sizeof(cd), hipMemcpyDeviceToDevice,
                       s) != hipSuccess)
        return SBCE_EHIP;
    if (rhs_out &&
        hipMemcpyAsync(rhs_out, ma.rhs, (size_t)pb.B * pb.L * pb.NR * sizeof(cd),
                       hipMemcpyDeviceToDevice, s) != hipSuccess)
        return SBCE_EHIP;
    return small ? SBCE_OK : hip_rc(launch_chol_solve(pb, ma, s));
}

// Diagnostic, not part of include/sbce.h: HIP-event timing of the L <= 512 Cholesky's update /
// factor / back-substitution launches (bench.py's panel_factor line).  mode 1 arms it for the
// following M-steps; mode 0 (after the caller synchronised) returns {update, factor, back
// substitution} ms and launch counts in out6 and disarms it.
int sbce_debug_chol_timing(int mode, double* out6) {
    clear_stale_error();
    return hip_rc(chol_debug_timing(mode, out6));
}

// Diagnostic, not part of include/sbce.h: per-phase cycle sums (32) of the MFMA Cholesky
// (SBCE_CHOL_SKIP bit 64); reset != 0 clears them.
// Diagnostic, not part of include/sbce.h: s_memtime stamps (48) of trial 0's solve wave in the
// n_tx <= 2 small M-step (SBCE_SMALL_STOP=4).
int sbce_debug_small_clock(unsigned long long* out48) {
    return out48 ? hip_rc(small_debug_clock(out48)) : SBCE_EINVAL;
}

int sbce_debug_chol_clock(unsigned long long* out32, int reset) {
    if (reset) return hip_rc(chol_debug_clock_reset());
    return out32 ? hip_rc(chol_debug_clock(out32)) : SBCE_EINVAL;
}

// Diagnostic, not part of include/sbce.h: phase-skip mask of the L <= 512 Cholesky kernels (1
// panel update, 2 diagonal factor, 8 TRSM tiles, 16 back substitution: results INVALID; 64:
// per-phase clocks of the fused kernel, results valid).  Process-wide (every thread and
// stream); while bits 0-4 are set every trial of every path is flagged SBCE_STATUS_DEBUG.
// 0 restores normal operation.
int sbce_debug_chol_skip(int mask) {
#if SBCE_AB
    if (mask < 0) return SBCE_EINVAL;
    chol_debug_skip(mask);
    return SBCE_OK;
#else
    (void)mask;
    return SBCE_EUNSUPPORTED;                        // libsbce_ab.so only
#endif
}

// Diagnostic, not part of include/sbce.h: one piece of the M-step for kernel timing (bench.py's
// dominant-kernel roofline), from the given moments: phase 0 = the pilot factorisation (once per
// EM run), 1 = the R build alone (the MFMA Hermitian build rbuild_herm_kernel when n_tx is 4 or
// 8 -- phase 0 must have run -- else the VALU build with B^H), 2 = the whole build (R and B^H).
int sbce_debug_mstep_phase(const sbce_dims* d, const sbce_ptrs* p, const void* moments, int phase,
                           void* hip_stream) {
    clear_stale_error();
    Problem pb;
    if (!make_problem(d, pb)) return SBCE_EINVAL;
    if (!chol_supported(pb)) return SBCE_EUNSUPPORTED;
    int rc = check_ptrs(p, pb, true, SBCE_SOLVE_CHOL);
    if (rc) return rc;
    if (!moments || phase < 0 || phase > 2) return SBCE_EINVAL;
    if (pb.B == 0) return SBCE_OK;
    hipStream_t s = (hipStream_t)hip_stream;
    const Carve c = carve(pb, SBCE_SOLVE_CHOL);
    char* ws = (char*)p->workspace;
    MstepArgs ma;
    ma.yd = (const cd*)p->y_d; ma.yp = (const cd*)p->y_p; ma.psid = (const cd*)p->psi_d;
    ma.up = (const cd*)p->u_p; ma.mom = (const cd*)moments; ma.R = (cd*)(ws + c.R);
    ma.rhs = (cd*)(ws + c.rhs); ma.theta = (cd*)p->theta; ma.status = nullptr; ma.done = nullptr;
    ma.solve_mode = SBCE_SOLVE_CHOL; ma.nbatch = pb.B;
    set_large(ma, ws, c);
    if (phase == 0) return rbuild_herm_supported(pb) ? hip_rc(launch_pilot_factor(pb, ma, s)) : SBCE_OK;
    if (phase == 1 && rbuild_herm_supported(pb)) return hip_rc(launch_rbuild_herm(pb, ma, s));
    return hip_rc(launch_mstep_build(pb, ma, s, rbuild_herm_supported(pb)));
}

// Diagnostic, not part of include/sbce.h: the per-trial pivot threshold tau = 32 eps K lambda_max
// the last min-norm M-step left in the workspace (tol_out [B] doubles, host or device memory).
int sbce_debug_minnorm_tol(const sbce_dims* d, const sbce_ptrs* p, double* tol_out, void* hip_stream) {
    Problem pb;
    if (!make_problem(d, pb) || !tol_out) return SBCE_EINVAL;
    int rc = check_ptrs(p, pb, true, SBCE_SOLVE_CHOL);
    if (rc) return rc;
    const Carve c = carve(pb, SBCE_SOLVE_CHOL);           // tol precedes the solve regions
    return hip_rc(hipMemcpyAsync(tol_out, (char*)p->workspace + c.tol, (size_t)pb.B * sizeof(double),
                                 hipMemcpyDefault, (hipStream_t)hip_stream));
}

// Diagnostic, not part of include/sbce.h: per trial (active extent, rank, refinement ran) of the
// last SBCE_SOLVE_MINNORM M-step whose workspace `p` holds (out3: [B][3] int32, device memory);
// bench.py prices the min-norm solve at its executed flops from them.
int sbce_debug_minnorm_rank(const sbce_dims* d, const sbce_ptrs* p, int32_t* out3, void* hip_stream) {
    clear_stale_error();
    Problem pb;
    if (!make_problem(d, pb) || !out3) return SBCE_EINVAL;
    int rc = check_ptrs(p, pb, true, SBCE_SOLVE_MINNORM);
    if (rc) return rc;
    if (pb.B == 0) return SBCE_OK;
    const Carve c = carve(pb, SBCE_SOLVE_MINNORM);
    MstepArgs ma;
    ma.R = (cd*)((char*)p->workspace + c.R);
    ma.done = nullptr;
    ma.nbatch = pb.B;
    set_large(ma, (char*)p->workspace, c);
    return hip_rc(launch_minnorm_rank(pb, ma, out3, (hipStream_t)hip_stream));
}

// Diagnostic, not part of include/sbce.h: re-read the SBCE_* debug switches from the
// environment (they are otherwise read once, when the library is loaded).  Returns 1 when a
// result-affecting switch is now non-default (every trial is then flagged SBCE_STATUS_DEBUG).
// The product build has no switches and reads nothing: it returns -1.
int sbce_debug_reload_env(void) {
#if SBCE_AB
    read_debug_env(g_debug);
    return debug_nondefault() ? 1 : 0;
#else
    return -1;
#endif
}

// Diagnostic, not part of include/sbce.h: FP64 MFMAs issued by the exact E-step sweep since
// the last reset (counted only with SBCE_ESTEP_COUNT=1); reset != 0 clears the counter.
int sbce_debug_estep_mfma(unsigned long long* out, int reset) {
    if (!reset && !out) return SBCE_EINVAL;
    return hip_rc(estep_debug_mfma(out, reset));
}

// Diagnostic, not part of include/sbce.h: symbols the sphere pass resolved by enumeration
// (out3[0]), left to the MFMA sweep (out3[1]) and resolved by the tree pass's single-path check
// (out3[2]) since the last reset (counted only with SBCE_ESTEP_COUNT=1).
int sbce_debug_estep_sphere(unsigned long long* out3, int reset) {
    if (!reset && !out3) return SBCE_EINVAL;
    return hip_rc(estep_debug_sphere(out3, reset));
}

// Diagnostic, not part of include/sbce.h: listed symbols the factorised-weight pass resolved
// (estep_pair.hip) since the last reset (counted only with SBCE_ESTEP_COUNT=1).
int sbce_debug_estep_pair(unsigned long long* out, int reset) {
    if (!reset && !out) return SBCE_EINVAL;
    return hip_rc(estep_debug_pair(out, reset));
}

int sbce_ser(const sbce_dims* d, const void* x_dest, const void* x_d_true, double* ser_out,
             void* hip_stream) {
    clear_stale_error();
    Problem pb;
    if (!make_problem(d, pb) || !x_dest || !x_d_true || !ser_out) return SBCE_EINVAL;
    if (pb.B == 0) return SBCE_OK;
    return hip_rc(launch_ser(pb, (const cd*)x_dest, (const cd*)x_d_true, ser_out,
                             (hipStream_t)hip_stream));
}

int sbce_gauss_expand(const sbce_dims* d, const void* theta, void* h_out, void* hip_stream) {
    clear_stale_error();
    Problem pb;
    if (!make_problem(d, pb) || !theta || !h_out || !aligned16(theta) || !aligned16(h_out))
        return SBCE_EINVAL;
    if (pb.B == 0) return SBCE_OK;
    return hip_rc(launch_gauss_expand(pb, (const cd*)theta, (cd*)h_out, (hipStream_t)hip_stream));
}

int sbce_nmse(const sbce_dims* d, const void* theta, const void* h_true, double* nmse_out,
              void* hip_stream) {
    clear_stale_error();
    Problem pb;
    if (!make_problem(d, pb) || !theta || !h_true || !nmse_out) return SBCE_EINVAL;
    if (pb.B == 0) return SBCE_OK;
    return hip_rc(launch_nmse(pb, (const cd*)theta, (const cd*)h_true, nmse_out,
                              (hipStream_t)hip_stream));
}

}  // extern "C"
