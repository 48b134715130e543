#!/usr/bin/env python3
"""Benchmark: EM-iterations/s of the MI355X EM semi-blind channel estimator.

Metric (BASELINE.json): EM-iterations/sec (whole node) on Nt=Nr=4, N_RIS=64,
T_p=16, T_d=256, 16-QAM (BASELINE configs[1]: 1000 Monte-Carlo trials x 20 EM
iterations per GPU), SNR 20 dB, exact soft E-step, float64.

A "step" = one full estimator call (``sbce_em``: 20 EM iterations, E-step +
M-step) over the whole per-GPU batch of trials, inputs resident in HBM.
value = (trials on all ranks x EM iterations x steps) / max-over-ranks time.

Multi-GPU (``torchrun --nproc-per-node N``): Monte-Carlo trials shard across
ranks (each rank its own trials, weak scaling, no data-path collective); the
only collective is ONE all-reduce (RCCL) of the per-rank NMSE accumulators
after the timed region, as in the reference's Monte-Carlo average
(Proposed_method_NMSEvsTp.py:176).

Also reported (one JSON line on rank 0):
  roofline      the M-step (the dominant phase per EM iteration; "kernels" lists the
                launches it consists of) timed live with HIP events on the launch
                stream: algorithmic flops per launch / time, peak = FP64
                rate of MI355X; traffic from the committed rocprofv3 PMC summary.
                The E-step (a tree search + MFMA sweep of the listed remainder) is
                reported next to it (estep_roofline: time, where the symbols were
                resolved, hypotheses covered per second).
  cpu_baseline  the build's vectorised float64 NumPy port of the same
                algorithm (oracle/em_reduced.py) on a bounded sample of the
                same workload, on this host's cores (rank 0, N=1 only).
"""
import argparse
import ctypes
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

FP64_PEAK_TFLOPS = 78.6      # MI355X FP64 vector (= FP64 matrix); half the guide's 157.3 TF FP32
# FP64 MFMA rate measured on the box with operands that change every iteration (DESIGN.md §8
# item 6, tools/ubench/): reported beside the datasheet peak, never used as "peak"
FP64_MFMA_MEASURED_TFLOPS = 46.0
HBM_PEAK_GBS = 8000.0

CONFIGS = {
    # name: (n_tx, n_rx, N_RIS, T_p, T_d, M, trials per GPU, EM iterations)
    "cfg1": (4, 4, 64, 16, 256, 16, 1000, 20),
    "plumbing": (2, 2, 16, 16, 50, 4, 10, 10),
    # BASELINE configs[2]: 10k trials over 8 GPUs; PM_beta list E-step r = 1
    "cfg2": (8, 8, 256, 32, 1024, 16, 1250, 5),
    # BASELINE configs[3]: T_p unstated -> 16, 16-QAM assumed (SURVEY §8 sizes table)
    "cfg4": (4, 4, 1024, 16, 512, 16, 100, 5),
}
# E-step (mode, partition_r) and M-step solve of each workload.  cfg 2 / cfg 4 have
# L > T_d + T_p (rank-deficient normal equations at high SNR): they use the minimum-norm
# solve, np.linalg.lstsq of PM.py:108 (include/sbce.h SBCE_SOLVE_MINNORM).
ESTEP = {"cfg1": ("soft", 0, "chol"), "plumbing": ("soft", 0, "chol"),
         "cfg2": ("pm_soft", 1, "lstsq"), "cfg4": ("soft", 0, "lstsq")}
# BASELINE configs[4]: the SNR x T_d grid of "Proposed method/all_detectorsvsTd.py" (constants
# :345-363: 2x2, N_RIS = 15, T_p = 20, itera = 5, partition_r = 1; driver :371-405: its five EMs
# per T_d point, each with the oracle early stop on the true h and the np.linalg.solve M-step),
# 64-QAM, 20 SNR x 8 T_d points.  The reference sweeps T_d = 15..90 in steps of 15 (:346); the
# grid's 8 points continue that list to 120.  SNR -> varn = power / 10^(SNR/10) with power = the
# 64-QAM symbol energy 42 (SNR/all_Detectors.py:351-354 uses its constellation's power the same way).
GRID = {"cfg5": dict(n_tx=2, n_rx=2, N=15, T_p=20, T_d=(15, 30, 45, 60, 75, 90, 105, 120),
                     SNR=tuple(float(s) for s in range(-5, 35, 2)), M=64, trials=64, iters=5,
                     power=42.0, partition_r=1,
                     detectors=("pm_soft", "hard", "zf", "mmse", "soft"))}


def metric_name(n_tx, N, T_p, T_d):
    """BASELINE.json's metric string, on the workload actually run (cfg 1 gives it verbatim)."""
    return (f"EM-iterations/sec (whole node) + NMSE@SNR; Nt=Nr={n_tx}, N_RIS={N}, "
            f"Tp={T_p} Td={T_d}")


# kernels of one E-step / M-step launch sequence (rocprofv3 names, tools/pmc_summary.py keys)
ESTEP_KERNELS = ["estep_tree_kernel", "estep_bfs_kernel", "estep_pair_kernel", "estep_bounds_kernel", "estep_prep_kernel",
                 "estep_mfma_kernel"]
MSTEP_KERNELS = ["pilot_factor_kernel", "pilot_rhs_kernel", "rbuild_herm_kernel", "rbuild_kernel", "rhs_lds_kernel",
                 "rhs_dma_kernel", "rhs_kernel", "diag_tol_kernel", "panel_update2_kernel",
                 "panel_factor_kernel", "backsub_kernel", "backsub4_kernel"]
MSTEP_KERNELS_LARGE = ["pilot_factor_kernel", "pilot_rhs_kernel", "rbuild_herm_kernel",
                       "rbuild_wide_kernel", "rhs_kernel", "rhs_dma_kernel", "rhs_lds_kernel",
                       "diag_tol_kernel", "chol_mfma_kernel", "tile_inverse_kernel",
                       "tile_gemm_kernel", "tile_herk_kernel", "dvec_kernel", "act_kernel",
                       "backdiag_kernel", "backupd_kernel",
                       # the minimum-norm solve (csrc/minnorm.hip)
                       "lanczos_tol_kernel", "gram_kernel", "gram_tol_kernel", "ghb_kernel",
                       "fwddiag_kernel", "fwdupd_kernel", "gz_kernel", "mn_gate_kernel"]
# launched exactly once per full M-step (the divisor of the phase's PMC totals for kernels launched
# several times per M-step; the pilot factorisation runs once per EM run, so its bytes are spread
# over the run's M-steps)
MSTEP_ANCHORS = ["diag_tol_kernel", "lanczos_tol_kernel"]   # once per full M-step solve
# the L <= 512 Cholesky solve's launches (csrc/chol.hip; diag_tol_kernel runs once per M-step)
CHOL_KERNELS = ["diag_tol_kernel", "panel_update2_kernel", "panel_factor_kernel", "backsub4_kernel",
                "backsub_kernel"]
CHOL_ANCHORS = ["diag_tol_kernel"]


def chol_flops_per_trial(L, n_rx, g3=True):
    """Cholesky of the L x L Hermitian R plus the forward / back substitutions with n_rx
    right-hand sides, as executed: (4/3) L^3 real flops of complex MACs (8 flops each), of which
    the MFMA tile products run as three real MFMAs per complex product instead of four (G3: 3/4),
    and 8 n_rx L^2 for the two triangular solves."""
    return (4.0 / 3.0) * L ** 3 * (0.75 if g3 else 1.0) + 8.0 * n_rx * L * L


def minnorm_flops_per_trial(L, n_rx, act, refined):
    """The minimum-norm solve (csrc/minnorm.hip) as executed for a trial whose rank-cut
    factorisation reached the active extent `act` (columns past it are never touched): Lanczos
    (4 Hermitian mat-vecs, 8 L^2 each), the left-looking factorisation of act columns over L rows
    (8 (L a^2/2 - a^3/3), four real MFMAs per complex product), C = G^H G on the active extent
    and its Cholesky (three real MFMAs per complex product: x 3/4), G^H b and G z (8 n_rx (L a -
    a^2/2) each), four triangular passes with C's factor (4 n_rx a^2 each); the refinement step
    (refined = 1) adds two of each product with G and four more passes."""
    a = float(act)
    fac = 8.0 * (L * a * a / 2 - a ** 3 / 3)
    gram = 0.75 * 8.0 * (L * a * a / 2 - a ** 3 / 3)
    cfac = 0.75 * (4.0 / 3.0) * a ** 3
    gmul = 8.0 * n_rx * (L * a - a * a / 2)
    tri = 4.0 * n_rx * a * a
    return (32.0 * L * L + fac + gram + cfac + 2 * gmul + 4 * tri
            + refined * (4 * gmul + 4 * tri))


def panel_factor_mfma_per_trial(L, pw=32, nb=16):
    """FP64 MFMAs (16x16x4) one trial's panel_factor_kernel launches issue under the wide schedule
    (csrc/chol.hip, three MFMAs per complex product): per 32-column panel with n 16-row tiles,
    the TRSM against D_A of tiles 1.. (12 + 8 for the fused y update), the in-panel update of their
    B parts (12), the TRSM against D_B of tiles 2.. (20), and for odd panels the rank-32
    pre-update of every tile (2 halves x 8 k-steps x 3; tile 0 one half)."""
    total = 0
    for j in range((L + pw - 1) // pw):
        n = (L - j * pw + nb - 1) // nb
        total += max(n - 1, 0) * (20 + 12) + max(n - 2, 0) * 20
        if j & 1:
            total += max(n - 1, 0) * 48 + 24
    return total


def chol_bytes_per_trial(L, n_rx):
    """Minimal HBM bytes of the solve: R's lower triangle read once and the factor written once
    (16 B complex each), read once more by the back substitution, B^H read, theta written."""
    return 16.0 * (3 * L * (L + 1) / 2 + 2 * L * n_rx)


def rbuild_flops_per_trial_iter(n_tx, N, T_p, T_d):
    """R build as executed: R[(p,a),(q,b)] = sum_t w_t S_t[a][b] (w = psi_p conj(psi_q)) over the
    P(P+1)/2 pairs p >= q; S_t Hermitian holds n_tx^2 real numbers, so per (pair, symbol) the
    complex w meets n_tx^2 reals: 2 n_tx^2 real MACs.  2 P^2 n_tx^2 (T_d + T_p) flops, half of
    SURVEY §8d's complex count 4 P^2 n_tx^2 (T_d + T_p)."""
    P = N + 1
    return 2 * P * P * n_tx * n_tx * (T_d + T_p)


def rbuild_bytes_per_trial_iter(n_tx, N, T_p, T_d):
    """R build HBM bytes, each tensor once: psi of every symbol (data + factored pilots), the
    moments S_t (pilot x' x'^H), R's lower triangle written."""
    P = N + 1
    L = P * n_tx
    return 16 * ((T_d + T_p) * P + (T_d + T_p) * n_tx * n_tx + L * (L + 1) // 2)


def mstep_flops_per_trial_iter(n_tx, n_rx, N, T_p, T_d, survey=False):
    """M-step work: R build (executed Hermitian form, rbuild_flops_per_trial_iter; survey=True:
    SURVEY §8d's 4 P^2 n_tx^2 (T_d + T_p)), B^H 8 n_rx L (T_d + T_p), Cholesky (4/3) L^3,
    triangular solves 8 n_rx L^2.  The min-norm solve's extra work (Lanczos, C = G^H G and its
    Cholesky, minnorm.hip) is not counted: for the lstsq workloads this is a lower bound."""
    P = N + 1
    L = P * n_tx
    rb = 4 * P * P * n_tx * n_tx * (T_d + T_p) if survey else rbuild_flops_per_trial_iter(n_tx, N, T_p, T_d)
    return rb + 8 * n_rx * L * (T_d + T_p) + 4 * L ** 3 / 3 + 8 * n_rx * L * L


def mstep_bytes_per_trial_iter(n_tx, n_rx, N, T_p, T_d):
    """Minimal HBM bytes of one M-step per trial: R written once and read once (Hermitian
    half), psi / moments / pilots read once, theta written."""
    P = N + 1
    L = P * n_tx
    return 16 * (L * L + T_d * P + T_d * (n_tx + n_tx * n_tx) + T_p * L + L * n_rx)


def estep_flops_per_trial_iter(n_tx, n_rx, T_d, M):
    """Minimal data-independent E-step work: every one of the T_d*M^n_tx hypotheses
    needs its distance d = a_i + g_k - 2 Re(p_i^H q_k): 2*n_rx real FMAs (4*n_rx flop)
    + 1 add + 1 compare.  Exp/accumulate work is data dependent (skipped for
    hypotheses below e^-50 of the running maximum) and not counted."""
    return T_d * (M ** n_tx) * (4 * n_rx + 2)


def estep_bytes_per_trial_iter(n_tx, n_rx, P, T_d):
    """Minimal HBM bytes of one E-step per trial: y_d, psi_d, theta read once,
    moments written once (complex128)."""
    K = P * n_tx * n_rx
    return 16 * (T_d * n_rx + T_d * P + K + T_d * (n_tx + n_tx * n_tx))


def load_pmc_traffic(path):
    try:
        with open(path) as f:
            return json.load(f)
    except (OSError, ValueError):
        return None


def estep_issued(args, config, trials):
    """Issued FP64 flops of one E-step (tools/sq_issued.sh: SQ instruction counters of the same
    launches, 64 lanes x VALU FP64 ops + 512 x MFMA_MOPS_F64), or None when the summary is absent
    or was taken on another configuration / batch."""
    sq = load_pmc_traffic(args.sq or os.path.join(ROOT, "profiles", f"sq_{config}_latest.json"))
    if not sq or sq.get("config") != config or sq.get("trials") != trials:
        return None
    return sq.get("issued_fp64_flops_per_estep")


def kernel_traffic(pmc, kernel):
    """HBM bytes of ONE launch of `kernel` from a PMC summary, or None."""
    k = (pmc or {}).get("kernels", {}).get(kernel)
    if not k or not k["launches_fetch"] or not k["launches_write"]:
        return None
    return k["fetch_bytes_total"] / k["launches_fetch"] + k["write_bytes_total"] / k["launches_write"]


# kernels launched exactly once per phase execution: their bytes are taken per launch (the bench
# also launches the build kernels alone for its phase timings, so their launch counts exceed the
# phase's); every other kernel of a phase is averaged over the phase's anchor launches
ONCE_PER_PHASE = {"rbuild_herm_kernel", "rbuild_kernel", "rbuild_wide_kernel", "rhs_dma_kernel",
                  "rhs_lds_kernel", "rhs_kernel", "diag_tol_kernel", "backsub4_kernel",
                  "backsub3_kernel", "backsub2_kernel", "backsub_kernel", "lanczos_tol_kernel",
                  "gram_kernel", "gram_tol_kernel", "mn_gate_kernel"}


def phase_traffic(pmc, kernels, anchor):
    """HBM bytes of ONE phase execution from a PMC summary (tools/pmc_summary.py): for a kernel
    launched once per phase (ONCE_PER_PHASE) its average FETCH / WRITE bytes per launch, for the
    others (the panel and tile launches, several per phase) their totals divided by the launches
    of the phase's once-per-phase anchor kernel (the first name in `anchor` the summary holds);
    None without an anchor."""
    ks = (pmc or {}).get("kernels", {})
    anc = next((ks[a] for a in anchor if a in ks), None)
    if not anc or not anc["launches_fetch"] or not anc["launches_write"]:
        return None
    tot = 0.0
    for k, e in ks.items():
        if k not in kernels:
            continue
        if k in ONCE_PER_PHASE:
            tot += e["fetch_bytes_total"] / max(e["launches_fetch"], 1)
            tot += e["write_bytes_total"] / max(e["launches_write"], 1)
        else:
            tot += e["fetch_bytes_total"] / anc["launches_fetch"]
            tot += e["write_bytes_total"] / anc["launches_write"]
    return tot


def host_threads():
    """Threads a NumPy port can use here: the affinity set, capped by OMP_NUM_THREADS (BLAS;
    16 on the GPU box).  NumPy's elementwise work itself is single-threaded."""
    threads = os.environ.get("OMP_NUM_THREADS")
    cores = len(os.sched_getaffinity(0))
    if threads and threads.isdigit():
        cores = min(cores, int(threads))
    return cores


def hypotheses_per_symbol(mode, n_tx, M, part_r=0):
    """Hypotheses the reference's E-step loop visits per data symbol: every one of M^n_tx for the
    exact / log-max EMs, the M^(p+1) list of the PM detectors (p = int(partition_r / log2 M),
    PMd/PM.py:74-92)."""
    if mode.startswith("pm"):
        return float(M) ** (int(part_r / np.log2(M)) + 1)
    return float(M) ** n_tx


def cpu_baseline(cfg, varn, seed, iters=2, mode="soft", part_r=0):
    """Oracle port (vectorised float64 NumPy reduced form, or the PM list oracle) on
    1 trial x `iters` EM iterations of the same configuration: ~10-30 s of CPU work."""
    import importlib
    from oracle.em_reduced import em_reduced
    from oracle.pm import em_pm
    pkg = importlib.import_module(
        "semi-blind-channel-estimation-for-mimo-ris-communication-system-using-em-algo_amd")
    n_tx, n_rx, N, T_p, T_d, M, _, _ = cfg
    b = pkg.signal_model.synthetic_batch(1, n_tx, n_rx, N, T_p, T_d, M, varn, seed=seed + 12345)
    t0 = time.perf_counter()
    if mode.startswith("pm"):
        em_pm(b["y_d"][0], b["y_p"][0], b["u_p"][0], b["psi_d"][0].T, varn, iters,
              b["theta0"][0], n_tx, n_rx, part_r, b["cons"], soft=mode == "pm_soft")
    else:
        aps = pkg.qam.all_possible_symbols(b["cons"], n_tx)
        em_reduced(b["y_d"][0], b["y_p"][0], b["u_p"][0], b["psi_d"][0].T, aps, varn, iters,
                   b["theta0"][0], mode=mode)
    dt = time.perf_counter() - t0
    threads = os.environ.get("OMP_NUM_THREADS")
    return {"value": iters / dt, "unit": "EM-iterations/s", "cores": host_threads(),
            "kind": "port",
            "sample": f"1 trial x {iters} EM iterations of the same config, "
                      f"{'oracle/pm.py' if mode.startswith('pm') else 'oracle/em_reduced.py'} "
                      f"(NumPy float64, BLAS threads={threads or 'default'}), {dt:.2f} s"}


def cpu_baseline_reference_structured(cfg, varn, seed, budget_s=20.0, mode="soft", part_r=0):
    """the reference's own loop structure (oracle/em_loop.py: dense Kronecker
    regressor Z_{t,j} per hypothesis, K x K accumulation of every hypothesis, LAPACK solve on the
    K x K system -- PMd/Proposed_method_NMSEvsTp.py:50-83 in float64 instead of mpmath) timed at
    the plumbing shape (BASELINE configs[0]: 2x2, N_RIS = 16, T_p = 16, T_d = 50, 4-QAM), then
    extrapolated to the bench workload with the loop's O(T_d J K^2) cost model, J = the
    hypotheses the workload's E-step visits per symbol (hypotheses_per_symbol: M^n_tx exact,
    the PM list M^(p+1) for the PM workloads, whose loop PMd/PM.py:79-104 accumulates every list
    member the same way)."""
    import importlib
    from oracle.em_loop import em_loop
    pkg = importlib.import_module(
        "semi-blind-channel-estimation-for-mimo-ris-communication-system-using-em-algo_amd")
    pn_tx, pn_rx, pN, pT_p, pT_d, pM = 2, 2, 16, 16, 50, 4
    b = pkg.signal_model.synthetic_batch(1, pn_tx, pn_rx, pN, pT_p, pT_d, pM, varn,
                                         seed=seed + 777)
    Y_d = [y[:, None] for y in b["y_d"][0]]
    Y_p = [y[:, None] for y in b["y_p"][0]]
    Z_p = [np.kron(u[None], np.eye(pn_rx)) for u in b["u_p"][0]]
    aps = pkg.qam.all_possible_symbols(b["cons"], pn_tx)
    args = (Y_d, Y_p, pT_d, pT_p, Z_p, b["psi_d"][0].T, aps, pM, varn)
    t0 = time.perf_counter()
    n = 0
    while True:
        em_loop(*args, 1, b["theta0"][0], skip_zero=False)
        n += 1
        if time.perf_counter() - t0 > budget_s / 4 or n >= 20:
            break
    t_plumb = (time.perf_counter() - t0) / n

    def work(n_tx, n_rx, N, T_d, J):
        return T_d * J * ((N + 1) * n_tx * n_rx) ** 2

    n_tx, n_rx, N, T_p, T_d, M, _, _ = cfg
    J = hypotheses_per_symbol(mode, n_tx, M, part_r)
    ratio = work(n_tx, n_rx, N, T_d, J) / work(pn_tx, pn_rx, pN, pT_d, float(pM) ** pn_tx)
    t_cfg = t_plumb * ratio
    threads = os.environ.get("OMP_NUM_THREADS")
    return {"value": 1.0 / t_cfg, "unit": "EM-iterations/s", "cores": host_threads(),
            "kind": "port",
            "sample": (f"oracle/em_loop.py (reference loop structure, float64) at the plumbing "
                       f"shape 2x2 N_RIS=16 T_p=16 T_d=50 4-QAM: {t_plumb:.3f} s per "
                       f"trial-iteration ({n} timed); extrapolated by T_d J K^2 with J = {J:.6g} "
                       f"hypotheses per symbol ({mode} E-step): {ratio:.3g}x, {t_cfg:.3g} s per "
                       f"trial-iteration of this workload; NumPy elementwise work single-threaded, "
                       f"BLAS threads={threads or 'default'} (cores = the BLAS thread cap)")}


def rank_envs(n, port, base=None):
    """Environments of the N ranks of a single-node run (torchrun's variables): rank r drives
    GPU r, rendezvous on 127.0.0.1:port."""
    base = dict(os.environ if base is None else base)
    return [dict(base, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                 GROUP_RANK="0", MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
            for r in range(n)]


def _free_port():
    import socket
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def launch_ranks(n, argv, timeout=None):
    """`bench.py --gpus N` started without WORLD_SIZE: start N rank processes of this same
    script as CHILDREN (one per GPU, torchrun's environment), wait for all, return the worst exit
    code.  Called before this process touches the GPU; the parent never execs.  Rank 0 prints
    the JSON line (children inherit stdout)."""
    import subprocess
    port = _free_port()
    procs = [subprocess.Popen([sys.executable, os.path.abspath(__file__), *argv], env=env)
             for env in rank_envs(n, port)]
    codes = []
    try:
        for p in procs:
            codes.append(p.wait(timeout=timeout))
    finally:
        for p in procs:
            if p.poll() is None:
                p.kill()
                p.wait()
    bad = [c for c in codes if c != 0]
    return bad[0] if bad else 0


def parse_args(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=None,
                    help="GPUs of this node (one rank each).  Without WORLD_SIZE and N > 1 the "
                         "ranks are started here; under torchrun it must equal WORLD_SIZE")
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--config", default="cfg1", choices=sorted(CONFIGS) + sorted(GRID))
    ap.add_argument("--grid-batch", choices=["point", "snr"], default="snr",
                    help="cfg5: one sbce_em per (T_d, SNR, detector) ('point') or per (T_d, "
                         "detector) with the SNR axis batched through per-trial noise variances "
                         "('snr', default)")
    ap.add_argument("--trials", type=int, default=None, help="trials per GPU")
    ap.add_argument("--iters", type=int, default=None, help="EM iterations per step")
    ap.add_argument("--snr", type=float, default=20.0)
    ap.add_argument("--mode", default=None, choices=["soft", "hard", "pm", "pm_soft"],
                    help="E-step (default: the workload's, ESTEP)")
    ap.add_argument("--partition-r", type=int, default=None)
    ap.add_argument("--seed", type=int, default=0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--kernel-reps", type=int, default=5)
    ap.add_argument("--roofline-only", action="store_true",
                    help="cfg5: only the roofline launches (the largest T_d point's E-steps and "
                         "M-step), no grid steps -- for the PMC passes of tools/profile_cfg5.sh")
    ap.add_argument("--graphs", type=int, default=1,
                    help="cfg5: each sbce_em call replayed as one captured HIP graph (1, default) "
                         "or launched eagerly (0)")
    ap.add_argument("--hw-queues", type=int, default=None,
                    help="GPU_MAX_HW_QUEUES for this process (HIP's default 4) when the "
                         "environment does not set it; at most 32")
    ap.add_argument("--enqueue", choices=("serial", "threads"), default="serial",
                    help="cfg5: the grid's calls enqueued by this thread, interleaved over the "
                         "streams (serial), or by one host thread per stream (threads)")
    ap.add_argument("--schedule", choices=("lpt", "rr"), default="lpt",
                    help="cfg5: calls onto streams longest-first to the least loaded (lpt, by each "
                         "call's measured time) or round robin in grid order (rr)")
    ap.add_argument("--streams", type=int, default=None,
                    help="sub-batches on concurrent HIP streams per GPU (default: 3 at cfg1, 4 for the cfg5 grid's calls, else 1)")
    ap.add_argument("--rccl-init", choices=["lazy", "eager"], default="lazy",
                    help="multi-rank runs: create the RCCL communicator at its first collective "
                         "(after the timed region; default) or at process-group init")
    ap.add_argument("--dist-at-world1", action="store_true",
                    help="initialise torch.distributed (RCCL) even for one rank (A/B of the "
                         "multi-rank schedule on a one-GPU box)")
    ap.add_argument("--selftest", action="store_true",
                    help="CPU plumbing self-test (gloo, no GPU, no estimator work): the launcher, "
                         "barriers, max-over-ranks timing and the accumulator all-reduce only")
    ap.add_argument("--pmc", default=None,
                    help="PMC summary (default: profiles/pmc_<config>_latest.json)")
    ap.add_argument("--sq", default=None,
                    help="issued-work SQ summary of the E-step (tools/sq_issued.sh; default: "
                         "profiles/sq_<config>_latest.json)")
    return ap.parse_args(argv)


def check_world(args, env=None):
    """World size of this process and the --gpus consistency rule; raises SystemExit(2) when
    --gpus disagrees with the launcher's WORLD_SIZE."""
    env = os.environ if env is None else env
    world = int(env.get("WORLD_SIZE", "1"))
    if args.gpus is not None and args.gpus != world:
        print(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={world}: the run would not measure "
              f"{args.gpus} GPUs", file=sys.stderr)
        raise SystemExit(2)
    return world


class Ranks:
    """Process-group plumbing of a run: host-side (gloo) barriers and the max-over-ranks clock,
    so that nothing of RCCL exists while the timed region runs unless --rccl-init eager; the
    Monte-Carlo accumulators go through ONE RCCL all-reduce afterwards."""

    def __init__(self, args, world):
        self.world = world
        self.rank = int(os.environ.get("RANK", "0"))
        self.local = int(os.environ.get("LOCAL_RANK", "0"))
        self.dist = None
        self.cpu = None
        self.selftest = args.selftest
        use_dist = world > 1 or args.dist_at_world1
        if not args.selftest:
            import torch
            torch.cuda.set_device(self.local)
        if use_dist:
            import torch
            import torch.distributed as dist
            self.dist = dist
            if args.selftest:
                dist.init_process_group("gloo")
                self.cpu = None
            else:
                kw = ({"device_id": torch.device("cuda", self.local)}
                      if args.rccl_init == "eager" else {})
                dist.init_process_group("nccl", **kw)
                self.cpu = dist.new_group(backend="gloo")

    def barrier(self):
        if self.dist is not None:
            self.dist.barrier(group=self.cpu)
        if not self.selftest:
            import torch
            torch.cuda.synchronize()

    def max_time(self, t):
        if self.dist is None:
            return t
        import torch
        v = torch.tensor([t], dtype=torch.float64)
        self.dist.all_reduce(v, op=self.dist.ReduceOp.MAX, group=self.cpu)
        return float(v.item())

    def allreduce_sum(self, t):
        """The Monte-Carlo accumulators: RCCL over xGMI (gloo in the self-test)."""
        if self.dist is not None:
            self.dist.all_reduce(t, op=self.dist.ReduceOp.SUM)
        return t

    def close(self):
        if self.dist is not None:
            self.dist.destroy_process_group()


def selftest(args, ranks):
    """--selftest: the multi-rank code path with a fixed host-side step instead of the estimator
    (CPU tests of the launcher; never a measurement)."""
    import torch
    B, iters = 8, 2
    for _ in range(args.warmup):
        time.sleep(0.01)
    ranks.barrier()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        time.sleep(0.01)
    ranks.barrier()
    elapsed = ranks.max_time(time.perf_counter() - t0)
    acc = ranks.allreduce_sum(torch.tensor([0.5 * B * (ranks.rank + 1), float(B)],
                                           dtype=torch.float64))
    if ranks.rank == 0:
        print(json.dumps({"metric": "selftest (plumbing only, no estimator work)",
                          "value": ranks.world * B * iters * args.steps / elapsed,
                          "unit": "EM-iterations/s", "n_gpus": ranks.world, "steps": args.steps,
                          "warmup": args.warmup, "ms_per_step": elapsed / args.steps * 1e3,
                          "higher_is_better": True, "scaling": "weak", "vs_baseline": None,
                          "dtype": "none", "data": "selftest",
                          "config": {"workload": "selftest", "parallelism": f"trials-sharded x{ranks.world}"},
                          "nmse_mean": float(acc[0] / acc[1]),
                          "trials_total": int(acc[1].item())}), flush=True)
    ranks.close()


def grid_cpu_baseline(g, seed, td=60, snr=15.0):
    """cfg5 CPU baseline: the oracle restatements of the five EMs (oracle/em_reduced.py exact and
    log-max, oracle/detectors.py ZF / MMSE, oracle/pm.py soft PM list) on ONE trial at one grid
    point (T_d = 60, 15 dB), every EM for all `iters` iterations (no early stop): EM-iterations/s
    of the five EMs together."""
    import importlib
    from oracle.em_reduced import em_reduced
    from oracle.detectors import em_detector
    from oracle.pm import em_pm
    pkg = importlib.import_module(
        "semi-blind-channel-estimation-for-mimo-ris-communication-system-using-em-algo_amd")
    n_tx, n_rx = g["n_tx"], g["n_rx"]
    varn = float(pkg.signal_model.snr_to_varn(snr, g["power"]))
    b = pkg.signal_model.synthetic_batch(1, n_tx, n_rx, g["N"], g["T_p"], td, g["M"], varn,
                                         seed=seed + 4242, pinv="scipy")
    a = (b["y_d"][0], b["y_p"][0], b["u_p"][0], b["psi_d"][0].T)
    aps = pkg.qam.all_possible_symbols(b["cons"], n_tx)
    it = g["iters"]
    t0 = time.perf_counter()
    em_pm(*a, varn, it, b["theta0"][0], n_tx, n_rx, g["partition_r"], b["cons"], soft=True)
    em_reduced(*a, aps, varn, it, b["theta0"][0], mode="hard")
    for kind in ("zf", "mmse"):
        em_detector(*a, aps, varn, it, b["theta0"][0], n_tx, n_rx, kind)
    em_reduced(*a, aps, varn, it, b["theta0"][0])
    dt = time.perf_counter() - t0
    threads = os.environ.get("OMP_NUM_THREADS")
    return {"value": 5 * it / dt, "unit": "EM-iterations/s", "cores": host_threads(), "kind": "port",
            "sample": f"1 trial at T_d={td}, SNR {snr:g} dB: the five EMs (oracle/pm.py soft PM r=1, "
                      f"oracle/em_reduced.py log-max and exact, oracle/detectors.py ZF and MMSE), "
                      f"{it} iterations each without early stop (NumPy float64, BLAS "
                      f"threads={threads or 'default'}), {dt:.2f} s"}


def grid_roofline(args, g, engines, k_last, torch):
    """cfg5 roofline: every detector's E-step and the M-step at the largest T_d point (the grid's
    costliest launches; the SNR axis batched, B = trials x 20), timed alone with HIP events on the
    launch stream at theta = h (the converged regime the oracle early stop leaves most trials in).
    The dominant launch (the exact soft E-step) is priced at its data-independent enumeration work,
    estep_flops_per_trial_iter: T_d M^n_tx (4 n_rx + 2) flop per trial, against the FP64 peak (the
    tree / BFS passes run on the FP64 VALU, the tile sweep on FP64 MFMA: 78.6 TF/s either way)."""
    n_tx, n_rx, N, M = g["n_tx"], g["n_rx"], g["N"], g["M"]
    P = N + 1
    stream = torch.cuda.current_stream()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)

    def timed(fn):
        fn()
        torch.cuda.synchronize()
        e0.record(stream)
        for _ in range(args.kernel_reps):
            fn()
        e1.record(stream)
        torch.cuda.synchronize()
        return e0.elapsed_time(e1) / args.kernel_reps

    phases, B, T_d, soft_eng = {}, None, None, None
    for di, k, js, eng in engines:
        det = g["detectors"][di]
        if k != k_last or f"estep_{det}" in phases:
            continue
        eng.theta.copy_(eng.h)
        phases[f"estep_{det}"] = timed(eng.estep)
        B, T_d = eng.B, eng.T_d
        if det == "soft":
            soft_eng = eng
    if soft_eng is not None:
        phases["mstep"] = timed(soft_eng.mstep)
    pmc = load_pmc_traffic(args.pmc or os.path.join(ROOT, "profiles", f"pmc_{args.config}_latest.json"))
    pmc_ok = bool(pmc and pmc.get("config") == args.config and pmc.get("trials") == B)
    ms = phases.get("estep_soft")
    enum_flops = estep_flops_per_trial_iter(n_tx, n_rx, T_d, M) * B
    issued = estep_issued(args, args.config, B)
    flops = issued if issued else enum_flops
    algo = estep_bytes_per_trial_iter(n_tx, n_rx, P, T_d) * B
    traffic = phase_traffic(pmc, ESTEP_KERNELS, ESTEP_KERNELS) if pmc_ok else None
    ach = flops / (ms * 1e-3) / 1e12 if ms else None
    roof = {"bound": "mfma", "pipe": "FP64 (VALU tree / BFS passes + MFMA tile sweep)",
            "phase": "exact soft E-step (the grid's dominant launch)", "kernels": ESTEP_KERNELS,
            "point": {"T_d": T_d, "trials": B, "theta": "h (converged regime)"},
            "ms": ms, "achieved": ach, "peak": FP64_PEAK_TFLOPS, "unit": "TFLOP/s",
            "frac": ach / FP64_PEAK_TFLOPS if ach else None, "flops_per_launch": flops,
            "flops_note": ("FP64 work the launch's kernels ISSUE (SQ counters, "
                           "profiles/sq_cfg5_latest.json: 64 lanes x VALU FP64 ops + 512 x "
                           "MFMA_MOPS_F64)" if issued else
                           "data-independent enumeration work T_d M^n_tx (4 n_rx + 2) per trial; "
                           "the pruned search issues less"),
            "enumeration_flops_per_launch": enum_flops,
            "enumeration_equivalent_tflops": enum_flops / (ms * 1e-3) / 1e12 if ms else None,
            "traffic": traffic, "algorithmic_bytes": algo,
            "traffic_ratio": traffic / algo if traffic else None,
            "hbm_frac_algorithmic": algo / (ms * 1e-3) / 1e9 / HBM_PEAK_GBS if ms else None}
    return {"roofline": roof, "phases": {k: v for k, v in phases.items()}}


def grid_main(args, ranks, pkg):
    """--config cfg5: one step = the whole SNR x T_d grid, five detector EMs per point, `trials`
    Monte-Carlo trials per point on every rank.  Calls are spread over 4 HIP streams (--streams),
    each a captured HIP graph (--graphs), longest first onto the least loaded stream (--schedule
    lpt).  value =
    trial-iterations EXECUTED (the oracle early stop ends a trial's EM; iters_done) / time."""
    import torch
    g = dict(GRID[args.config])
    if args.trials:
        g["trials"] = args.trials
    if args.iters:
        g["iters"] = args.iters
    world, rank = ranks.world, ranks.rank
    n_tx, n_rx, N, T_p, M, B, iters = (g[k] for k in ("n_tx", "n_rx", "N", "T_p", "M", "trials",
                                                        "iters"))
    T_D, SNR, dets = g["T_d"], g["SNR"], g["detectors"]
    if args.roofline_only:
        T_D = T_D[-1:]
    varns = [float(v) for v in pkg.signal_model.snr_to_varn(SNR, g["power"])]
    ns, nt, nd = len(SNR), len(T_D), len(dets)
    engines = []                     # (detector index, T_d index, SNR indices, engine)
    for k, td in enumerate(T_D):
        # h_initial with scipy.linalg.pinv's cut, as all_detectorsvsTd.py:341 has it (T_p = 20 >
        # N_RIS = 15: the DFT pilot phases repeat; numpy's 1e-15 cut would give theta_0 ~ 1e13)
        pts = [pkg.signal_model.synthetic_batch(B, n_tx, n_rx, N, T_p, td, M, vn, pinv="scipy",
                                                seed=(args.seed * 1000003 + rank) * 1000 + k * 50 + j)
               for j, vn in enumerate(varns)]
        if args.grid_batch == "snr":
            groups = [(list(range(ns)), {key: np.concatenate([p[key] for p in pts])
                                         for key in ("y_d", "y_p", "psi_d", "u_p", "theta0", "h")},
                       np.repeat(np.asarray(varns), B))]
        else:
            groups = [([j], pts[j], varns[j]) for j in range(ns)]
        for js, batch, vn in groups:
            batch = dict(batch, cons=pts[0]["cons"])
            for di, det in enumerate(dets):
                eng = pkg.EMEngine(batch, vn, mode=det, solve="chol", early_stop=True,
                                   partition_r=g["partition_r"] if det == "pm_soft" else 0)
                engines.append((di, k, js, eng))
        del pts
    torch.cuda.synchronize()
    streams = [torch.cuda.Stream() for _ in range(args.streams or 4)]
    cur = torch.cuda.current_stream()
    graphs = None
    if args.graphs and not args.roofline_only:
        # every sbce_em call as one captured HIP graph (EMEngine.capture): the grid's 40 calls
        # launch ~4 kernels per iteration each, and eagerly the host enqueue sets the pace
        for _, _, _, eng in engines:
            eng.run(iters)                       # first launches load the code objects
        torch.cuda.synchronize()
        graphs = [eng.capture(iters) for _, _, _, eng in engines]
        torch.cuda.synchronize()
    # which stream runs which call: round robin in grid order, or longest-first onto the least
    # loaded stream (LPT) by each call's time measured alone (one untimed replay each)
    order = [[i for i in range(len(engines)) if i % len(streams) == s] for s in range(len(streams))]
    call_ms = None
    if args.schedule == "lpt":
        call_ms = []
        for i, (_, _, _, eng) in enumerate(engines):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(cur)
            if graphs is None:
                eng.run(iters)
            else:
                graphs[i].replay()
            e1.record(cur)
            torch.cuda.synchronize()
            call_ms.append(e0.elapsed_time(e1))
        load = [0.0] * len(streams)
        order = [[] for _ in streams]
        for i in sorted(range(len(engines)), key=lambda i: -call_ms[i]):
            s_min = min(range(len(streams)), key=lambda s: load[s])
            order[s_min].append(i)
            load[s_min] += call_ms[i]

    pool = None
    if args.enqueue == "threads":
        from concurrent.futures import ThreadPoolExecutor
        pool = ThreadPoolExecutor(len(streams))

    def enqueue(st, o):                  # one stream's calls (a host thread of its own)
        for i in o:
            if graphs is None:
                engines[i][3].run(iters, stream=st)
            else:
                with torch.cuda.stream(st):
                    graphs[i].replay()

    def step():
        ev = torch.cuda.Event()
        ev.record(cur)
        for st in streams:
            st.wait_event(ev)
        if pool is not None:
            for f in [pool.submit(enqueue, st, o) for st, o in zip(streams, order)]:
                f.result()
            for st in streams:
                cur.wait_stream(st)
            return
        # calls are issued interleaved over the streams (the host enqueue never starves one)
        for r in range(max(len(o) for o in order)):
            for st, o in zip(streams, order):
                if r >= len(o):
                    continue
                i = o[r]
                if graphs is None:
                    engines[i][3].run(iters, stream=st)
                else:
                    with torch.cuda.stream(st):
                        graphs[i].replay()
        for st in streams:
            cur.wait_stream(st)

    if args.roofline_only:
        roof = grid_roofline(args, g, engines, len(T_D) - 1, torch)
        if rank == 0:
            print(json.dumps({"roofline_only": args.config, "roofline": roof}), flush=True)
        ranks.close()
        return
    for _ in range(args.warmup):
        step()
    ranks.barrier()
    t0 = time.perf_counter()
    host = 0.0                        # host time inside step(): the enqueue of the grid's launches
    for _ in range(args.steps):
        th = time.perf_counter()
        step()
        host += time.perf_counter() - th
    torch.cuda.synchronize()
    ranks.barrier()
    elapsed = ranks.max_time(time.perf_counter() - t0)

    # executed trial-iterations of one step (every step repeats the same EMs from theta_0)
    done = torch.stack([eng.iters_done.sum() for _, _, _, eng in engines]).sum().to(torch.float64)
    nominal = float(B * iters * ns * nt * nd)
    # the one collective: [sum NMSE, count] of every (detector, T_d, SNR) point + executed its
    acc = torch.zeros(nd * nt * ns * 2 + 1, dtype=torch.float64, device="cuda")
    for di, k, js, eng in engines:
        nm = eng.nmse().view(len(js), B)
        for jj, j in enumerate(js):
            base = ((di * nt + k) * ns + j) * 2
            acc[base] += nm[jj].sum()
            acc[base + 1] += B
    acc[-1] = done
    ranks.allreduce_sum(acc)
    a = acc[:-1].view(nd, nt, ns, 2).cpu().numpy()
    mean = a[..., 0] / a[..., 1]
    executed = float(acc[-1].item())
    flagged = sum(int((eng.status != 0).sum().item()) for _, _, _, eng in engines)
    roof = grid_roofline(args, g, engines, len(T_D) - 1, torch)   # overwrites theta: after NMSE
    line = {
        "metric": metric_name(n_tx, N, T_p, f"{T_D[0]}..{T_D[-1]}") + " (SNR x T_d grid, five EMs)",
        "value": executed * args.steps / elapsed,
        "unit": "EM-iterations/s",
        "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
        "ms_per_step": elapsed / args.steps * 1e3,
        "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "f64",
        "data": "synthetic (Rayleigh channels, 64-QAM, uniform RIS phases, CN noise; numpy Generator)",
        "config": {"workload": args.config, "n_tx": n_tx, "n_rx": n_rx, "N_RIS": N, "T_p": T_p,
                   "T_d": list(T_D), "snr_db": list(SNR), "snr_power": g["power"], "M": M,
                   "trials_per_point_per_gpu": B, "em_iters": iters, "detectors": list(dets),
                   "partition_r": g["partition_r"], "solve": "chol", "early_stop": "oracle (h)",
                   "grid_batch": args.grid_batch, "sbce_em_calls_per_step": len(engines),
                   "streams_per_gpu": len(streams), "hip_graphs": graphs is not None,
                   "schedule": args.schedule, "enqueue": args.enqueue,
                   "call_ms_sum": None if call_ms is None else float(sum(call_ms)),
                   "parallelism": f"trials-sharded x{world}"},
        "value_note": ("value counts the trial-iterations the EMs executed (each EM stops at the "
                       "reference's oracle criterion, all_detectorsvsTd.py:87-89 etc.); "
                       f"nominal {nominal * world:.0f} per step (all {iters} iterations), executed "
                       f"{executed:.0f}"),
        "executed_iterations_per_step": executed,
        "host_enqueue_ms_per_step": host / args.steps * 1e3,
        "nominal_iterations_per_step": nominal * world,
        "nmse_grid_mean": {det: float(np.mean(mean[di])) for di, det in enumerate(dets)},
        "nmse_at_max_td": {det: [float(v) for v in mean[di, -1]] for di, det in enumerate(dets)},
        "status_flagged_trials": flagged,
        "roofline": roof["roofline"],
        "phases_at_max_td": roof["phases"],
    }
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        line["cpu_baseline"] = grid_cpu_baseline(g, args.seed)
    if rank == 0:
        print(json.dumps(line), flush=True)
    ranks.close()


def main(argv=None):
    argv = sys.argv[1:] if argv is None else argv
    args = parse_args(argv)
    if "WORLD_SIZE" not in os.environ and args.gpus is not None and args.gpus > 1:
        # no launcher: start one rank per GPU as child processes (nothing here has touched
        # the GPU yet) and exit with their status
        raise SystemExit(launch_ranks(args.gpus, argv))
    world_env = check_world(args)
    if args.selftest:
        ranks = Ranks(args, world_env)
        return selftest(args, ranks)
    # 3 sub-batch streams: with the default stream they fill HIP's 4 hardware queues per process
    # (GPU_MAX_HW_QUEUES, the box's default).  Measured at cfg1: 1 stream 325k EM-it/s, 2 330k,
    # 3 335k; 4 streams on 4 queues 276k (two sub-batches share a queue and run back to back), and
    # with the queue count raised to 8 / 12 for 4 / 6 streams 294k / 280k.  Multi-rank runs keep
    # the same schedule: the RCCL communicator (and its streams) is created lazily at the
    # accumulator all-reduce after the timed region.
    nstreams = args.streams if args.streams is not None else (3 if args.config == "cfg1" else 1)
    if args.hw_queues is None and args.config in GRID:
        # the grid's latency-bound calls: 4 streams on 8 hardware queues measured best on one box
        # (16.06 ms vs 17.07-17.42 with 3 on the default 4; profiles/r06/cfg5_streams/)
        args.hw_queues = 8
    if args.hw_queues and "GPU_MAX_HW_QUEUES" not in os.environ:
        # hardware queues per process: read once by the HIP runtime, so before torch loads it
        os.environ["GPU_MAX_HW_QUEUES"] = str(args.hw_queues)
    import torch
    import __graft_entry__ as ge
    pkg = ge.package()
    ranks = Ranks(args, world_env)
    world, rank = ranks.world, ranks.rank
    if args.config in GRID:
        return grid_main(args, ranks, pkg)

    cfg = list(CONFIGS[args.config])
    if args.trials:
        cfg[6] = args.trials
    if args.iters:
        cfg[7] = args.iters
    n_tx, n_rx, N, T_p, T_d, M, B, iters = cfg
    mode, part_r, solve = ESTEP[args.config]
    mode = args.mode or mode
    part_r = part_r if args.partition_r is None else args.partition_r
    varn = float(pkg.signal_model.snr_to_varn(args.snr))

    # ---- synthetic inputs for this rank's trials, resident in HBM before timing ----
    batch = pkg.signal_model.synthetic_batch(B, n_tx, n_rx, N, T_p, T_d, M, varn,
                                             seed=args.seed * 1000003 + rank)
    eng = pkg.EMEngine(batch, varn, mode=mode, partition_r=part_r, solve=solve, streams=nstreams)
    del batch
    torch.cuda.synchronize()

    for _ in range(args.warmup):
        eng.run(iters)
    ranks.barrier()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        eng.run(iters)
    torch.cuda.synchronize()
    ranks.barrier()
    elapsed = ranks.max_time(time.perf_counter() - t0)

    # ---- the one collective: Monte-Carlo NMSE accumulators (sum NMSE, count) ----
    nm = eng.nmse()
    acc = torch.stack([nm.sum(), torch.tensor(float(B), dtype=torch.float64, device="cuda")])
    ranks.allreduce_sum(acc)
    nmse_mean = float(acc[0] / acc[1])
    # SBCE_STATUS_NONHPD only: the PILOT / DETECTOR bits are informational
    nonhpd = int(((eng.status & pkg._lib.SBCE_STATUS_NONHPD) != 0).sum().item())
    status_bits = {name: int(((eng.status & bit) != 0).sum().item())
                   for name, bit in (("pilot", pkg._lib.SBCE_STATUS_PILOT),
                                     ("detector", pkg._lib.SBCE_STATUS_DETECTOR),
                                     ("rank_near_cut", pkg._lib.SBCE_STATUS_RANK),
                                     ("debug", pkg._lib.SBCE_STATUS_DEBUG))}

    # ---- dominant-kernel timing: E-step launches with HIP events on the launch stream ----
    stream = torch.cuda.current_stream()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    eng.estep()
    e0.record(stream)
    for _ in range(args.kernel_reps):
        eng.estep()
    e1.record(stream)
    torch.cuda.synchronize()
    estep_ms = e0.elapsed_time(e1) / args.kernel_reps
    # FP64 MFMAs the exact E-step actually issued at this theta (its exact column-tile
    # bounds skip provably negligible tiles): one counted launch outside the timed loops
    mfma_issued = None
    sphere = None
    lib = pkg._lib.load_ab()          # the counters live in the A/B build (eng.lib inside debug_env)
    if mode in ("soft", "hard") and hasattr(lib, "sbce_debug_estep_mfma"):
        import ctypes
        cnt = ctypes.c_ulonglong(0)
        sph = (ctypes.c_ulonglong * 3)()
        with pkg._lib.debug_env(SBCE_ESTEP_COUNT="1"):
            npair = ctypes.c_ulonglong(0)
            lib.sbce_debug_estep_mfma(None, 1)
            lib.sbce_debug_estep_sphere(None, 1)
            lib.sbce_debug_estep_pair(None, 1)
            eng.estep()
            torch.cuda.synchronize()
            lib.sbce_debug_estep_mfma(ctypes.byref(cnt), 0)
            lib.sbce_debug_estep_sphere(sph, 0)
            lib.sbce_debug_estep_pair(ctypes.byref(npair), 0)
        mfma_issued = int(cnt.value)
        nsym = float(B * T_d)
        # where the symbols' posteriors were computed: single surviving
        # path in the tree pass, breadth-first enumeration, factorised weights (the listed
        # symbols of a wide posterior), or the MFMA tile sweep
        sphere = {"single_path": sph[2] / nsym, "enumerated": sph[0] / nsym,
                  "factorised": npair.value / nsym, "swept": (sph[1] - npair.value) / nsym}
    e0.record(stream)
    for _ in range(args.kernel_reps):
        eng.mstep()
    e1.record(stream)
    torch.cuda.synchronize()
    mstep_ms = e0.elapsed_time(e1) / args.kernel_reps
    # the min-norm solve's per-trial extent / rank / refinement, read from the workspace of the
    # M-step just timed (the R-build timings below overwrite R, where G lives)
    rk = eng.minnorm_rank() if solve == "lstsq" else None

    # ---- dominant kernel: the R build (rbuild_herm_kernel, n_tx in {4, 8}) timed alone ----
    rb_ms = None
    if n_tx in (4, 8):
        eng.mstep_phase(0)                       # pilot factorisation (once per EM run)
        torch.cuda.synchronize()
        e0.record(stream)
        for _ in range(args.kernel_reps):
            eng.mstep_phase(1)
        e1.record(stream)
        torch.cuda.synchronize()
        rb_ms = e0.elapsed_time(e1) / args.kernel_reps

    # ---- the Cholesky's own launches by HIP events between them (sbce_debug_chol_timing) ----
    chol_launch = None
    if n_tx * (N + 1) <= 512 and solve == "chol":
        fn = eng.lib.sbce_debug_chol_timing
        fn.restype = ctypes.c_int
        out6 = (ctypes.c_double * 6)()
        torch.cuda.synchronize()
        if fn(1, None) == 0:                     # 512 events: up to 18 M-steps at cfg1
            for _ in range(min(args.kernel_reps, 16)):
                eng.mstep()
            torch.cuda.synchronize()
            if fn(0, out6) == 0 and out6[4] > 0:
                chol_launch = [v / min(args.kernel_reps, 16) for v in out6]

    # ---- the Cholesky solve alone: whole M-step minus its build (R and B^H, phase 2) ----
    build_ms = None
    if n_tx * (N + 1) <= 512 and solve == "chol":
        e0.record(stream)
        for _ in range(args.kernel_reps):
            eng.mstep_phase(2)
        e1.record(stream)
        torch.cuda.synchronize()
        build_ms = e0.elapsed_time(e1) / args.kernel_reps

    P = N + 1
    pmc = load_pmc_traffic(args.pmc or os.path.join(ROOT, "profiles", f"pmc_{args.config}_latest.json"))
    pmc_ok = bool(pmc and pmc.get("config") == args.config and pmc.get("trials") == B)
    # large-L workloads (every kernel per trial, grids over the batch): a PMC summary taken at
    # fewer trials (tools/r06_cfg2.sh: 256) is scaled by the batch -- stated in the line
    pmc_scale = 1.0
    if (not pmc_ok and pmc and pmc.get("config") == args.config and pmc.get("trials")
            and n_tx * P > 512):
        pmc_ok, pmc_scale = True, B / float(pmc["trials"])

    def traffic_of(kernels, anchor):
        t = phase_traffic(pmc, kernels, anchor) if pmc_ok else None
        return t * pmc_scale if t else t

    mflops = mstep_flops_per_trial_iter(n_tx, n_rx, N, T_p, T_d) * B
    mn_stats = None
    if solve == "lstsq":
        # the min-norm factorisation stops at R's numerical rank (left-looking, minnorm.hip):
        # priced per trial at the extent it reached (the last timed M-step's workspace)
        L_ = (N + 1) * n_tx
        mn = sum(minnorm_flops_per_trial(L_, n_rx, int(a_), int(r_)) for a_, _, r_ in rk)
        mflops = (rbuild_flops_per_trial_iter(n_tx, N, T_p, T_d) + 8 * n_rx * L_ * (T_d + T_p)) * B + mn
        mn_stats = {"extent_mean": float(rk[:, 0].mean()), "rank_mean": float(rk[:, 1].mean()),
                    "rank_min": int(rk[:, 1].min()), "rank_max": int(rk[:, 1].max()),
                    "refined_trials": int(rk[:, 2].sum()), "minnorm_flops_per_launch": mn}
    mbytes = mstep_bytes_per_trial_iter(n_tx, n_rx, N, T_p, T_d) * B
    m_kern = MSTEP_KERNELS_LARGE if n_tx * P > 512 else MSTEP_KERNELS
    m_traffic = traffic_of(m_kern, MSTEP_ANCHORS)
    m_ach = mflops / (mstep_ms * 1e-3) / 1e12
    mstep_roof = {"bound": "mfma", "pipe": "FP64 MFMA v_mfma_f64_16x16x4f64 (+ FP64 VALU)",
                  "phase": "M-step", "solve": solve, "kernels": m_kern, "ms": mstep_ms,
                  "achieved": m_ach, "peak": FP64_PEAK_TFLOPS, "unit": "TFLOP/s",
                  "frac": m_ach / FP64_PEAK_TFLOPS, "flops_per_launch": mflops,
                  "flops_survey_formula": mstep_flops_per_trial_iter(n_tx, n_rx, N, T_p, T_d,
                                                                     survey=True) * B,
                  "traffic": m_traffic, "algorithmic_bytes": mbytes,
                  "traffic_ratio": m_traffic / mbytes if m_traffic else None,
                  "hbm_frac_algorithmic": mbytes / (mstep_ms * 1e-3) / 1e9 / HBM_PEAK_GBS,
                  "measured_pipe_tflops": FP64_MFMA_MEASURED_TFLOPS,
                  "frac_of_measured_pipe": m_ach / FP64_MFMA_MEASURED_TFLOPS}
    if pmc_scale != 1.0:
        mstep_roof["traffic_note"] = (f"PMC summary of {pmc['trials']} trials scaled by "
                                      f"{pmc_scale:g} to the {B}-trial batch")
    if solve == "lstsq":
        mstep_roof["minnorm"] = mn_stats
        mstep_roof["note"] = ("flops: the R and B^H build plus the min-norm solve priced per trial at "
                              "the active extent its rank-cut factorisation reached "
                              "(bench.minnorm_flops_per_trial, sbce_debug_minnorm_rank)")
    rb_roof = None
    if rb_ms is not None:
        rflops = rbuild_flops_per_trial_iter(n_tx, N, T_p, T_d) * B
        rbytes = rbuild_bytes_per_trial_iter(n_tx, N, T_p, T_d) * B
        r_traffic = kernel_traffic(pmc, "rbuild_herm_kernel") if pmc_ok else None
        r_traffic = r_traffic * pmc_scale if r_traffic else r_traffic
        r_ach = rflops / (rb_ms * 1e-3) / 1e12
        rb_roof = {"bound": "mfma", "kernel": "rbuild_herm_kernel",
                   "pipe": "FP64 MFMA v_mfma_f64_16x16x4f64", "ms": rb_ms,
                   "achieved": r_ach, "peak": FP64_PEAK_TFLOPS, "unit": "TFLOP/s",
                   "frac": r_ach / FP64_PEAK_TFLOPS, "flops_per_launch": rflops,
                   "traffic": r_traffic, "algorithmic_bytes": rbytes,
                   "traffic_ratio": r_traffic / rbytes if r_traffic else None,
                   "measured_pipe_tflops": FP64_MFMA_MEASURED_TFLOPS,
                   "frac_of_measured_pipe": r_ach / FP64_MFMA_MEASURED_TFLOPS}
    chol_roof = None
    if build_ms is not None:
        L_ = n_tx * P
        c_ms = mstep_ms - build_ms
        cflops = chol_flops_per_trial(L_, n_rx) * B
        cbytes = chol_bytes_per_trial(L_, n_rx) * B
        c_traffic = traffic_of(CHOL_KERNELS, CHOL_ANCHORS)
        c_ach = cflops / (c_ms * 1e-3) / 1e12
        chol_roof = {"bound": "mfma", "phase": "Cholesky solve (batched panels + back substitution)",
                     "kernels": CHOL_KERNELS, "ms": c_ms, "how": "M-step minus its R / B^H build, "
                     "both timed with HIP events on the launch stream",
                     "achieved": c_ach, "peak": FP64_PEAK_TFLOPS, "unit": "TFLOP/s",
                     "frac": c_ach / FP64_PEAK_TFLOPS, "flops_per_launch": cflops,
                     "traffic": c_traffic, "algorithmic_bytes": cbytes,
                     "traffic_ratio": c_traffic / cbytes if c_traffic else None,
                     "hbm_GBps_traffic": c_traffic / (c_ms * 1e-3) / 1e9 if c_traffic else None,
                     "frac_of_measured_pipe": c_ach / FP64_MFMA_MEASURED_TFLOPS}
        if chol_launch:
            # panel_factor_kernel's own line: its launches of one M-step (HIP events around each
            # launch on the launch stream), priced at the MFMAs it issues (2048 flop each)
            f_ms, f_n = chol_launch[1], chol_launch[4]
            pflops = panel_factor_mfma_per_trial(L_) * 2048.0 * B
            p_traffic = kernel_traffic(pmc, "panel_factor_kernel") if pmc_ok else None
            p_ach = pflops / (f_ms * 1e-3) / 1e12
            chol_roof["panel_factor"] = {
                "kernel": "panel_factor_kernel", "bound": "mfma", "launches": f_n, "ms": f_ms,
                "flops_per_mstep": pflops, "achieved": p_ach, "peak": FP64_PEAK_TFLOPS,
                "unit": "TFLOP/s", "frac": p_ach / FP64_PEAK_TFLOPS,
                "frac_of_measured_pipe": p_ach / FP64_MFMA_MEASURED_TFLOPS,
                "traffic_per_mstep": p_traffic * f_n if p_traffic else None,
                "note": "MFMA work only; the two diagonal-block chains per launch are FP64 VALU / "
                        "LDS latency (DESIGN section 3.5)"}
            chol_roof["launch_ms"] = {"panel_update2": chol_launch[0], "panel_factor": f_ms,
                                      "back_substitution": chol_launch[2],
                                      "launches": {"panel_update2": chol_launch[3],
                                                   "panel_factor": f_n,
                                                   "back_substitution": chol_launch[5]}}
    if mode in ("soft", "hard"):
        flops = estep_flops_per_trial_iter(n_tx, n_rx, T_d, M) * B
        algo_bytes = estep_bytes_per_trial_iter(n_tx, n_rx, P, T_d) * B
        # executed work: the MFMAs issued (16x16x4 f64 = 2048 flop each); the full
        # enumeration's flops are reported next to it ("enumeration_*")
        executed = mfma_issued * 2048 if mfma_issued is not None else flops
        # the E-step is a search (tree pass, enumeration, sweep of the listed remainder): its
        # time is set by per-symbol latency, not a pipe's peak; reported for reference
        issued = estep_issued(args, args.config, B)
        e_ach = issued / (estep_ms * 1e-3) / 1e12 if issued else None
        estep_roof = {"bound": "fp64 issue" if issued else "latency",
                      "pipe": "FP64 VALU tree search + FP64 MFMA sweep",
                      "phase": "E-step", "kernels": ESTEP_KERNELS, "ms": estep_ms,
                      "issued_fp64_flops_per_launch": issued,
                      "achieved": e_ach, "peak": FP64_PEAK_TFLOPS, "unit": "TFLOP/s",
                      "frac": e_ach / FP64_PEAK_TFLOPS if e_ach else None,
                      "issued_note": ("FP64 work the E-step's kernels issue (SQ counters, "
                                      "profiles/sq_<config>_latest.json: 64 lanes x VALU FP64 ops + "
                                      "512 x MFMA_MOPS_F64 per launch) / its live time"),
                      "sphere_pass": sphere,
                      "traffic": traffic_of(ESTEP_KERNELS, ESTEP_KERNELS),
                      "sweep_mfma_flops_per_launch": executed,
                      "enumeration_flops_per_launch": flops,
                      "hypotheses_per_s": B * T_d * float(M) ** n_tx / (estep_ms * 1e-3),
                      "algorithmic_bytes": algo_bytes,
                      "hbm_GBps_algorithmic": algo_bytes / (estep_ms * 1e-3) / 1e9,
                      "hbm_frac_algorithmic": algo_bytes / (estep_ms * 1e-3) / 1e9 / HBM_PEAK_GBS}
    else:
        estep_roof = None
    # the roofline object: the dominant kernel (the R build) when it runs alone; otherwise the
    # M-step phase
    roofline = rb_roof if rb_roof is not None and n_tx * P <= 512 else mstep_roof

    value = world * B * iters * args.steps / elapsed
    line = {
        "metric": metric_name(n_tx, N, T_p, T_d),
        "value": value,
        "unit": "EM-iterations/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": elapsed / args.steps * 1e3,
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "f64",
        "data": "synthetic (Rayleigh channels, 16-QAM, uniform RIS phases, CN noise; numpy Generator)",
        "config": {"workload": args.config, "n_tx": n_tx, "n_rx": n_rx, "N_RIS": N, "T_p": T_p,
                   "T_d": T_d, "M": M, "trials_per_gpu": B, "em_iters": iters,
                   "snr_db": args.snr, "estep": mode, "partition_r": part_r, "solve": solve,
                   "parallelism": f"trials-sharded x{world}",
                   "streams_per_gpu": len(eng.subs) or 1,
                   "rccl_init": args.rccl_init if ranks.dist is not None else None},
        "schedule": (f"per GPU: {len(eng.subs)} contiguous sub-batches of the {B} trials, one sbce_em "
                     f"each on its own HIP stream (bitwise the same theta as one call); kernels_ms "
                     f"and the rooflines time whole-batch launches alone" if eng.subs else
                     "one sbce_em call per GPU"),
        "nmse_mean": nmse_mean,
        "nmse_note": ("at cfg 1 / 20 dB the EM moves the pilot-only theta_0 (NMSE ~0.93) to NMSE "
                      "~9 within ~4 iterations; the 20-iteration trajectory is pinned to the float64 "
                      "oracle (tests/golden/cfg1_traj.npz), which is validated against the reference "
                      "em() itself at this kernel shape for 2 iterations (cfg1_kernel.npz)"
                      if args.config == "cfg1" else None),
        "nonhpd_trials": nonhpd,
        "status_trials": status_bits,
        "kernels_ms": {"estep": estep_ms, "mstep_build_plus_solve": mstep_ms},
        "roofline": roofline,
        "rbuild_roofline": rb_roof,
        "mstep_roofline": mstep_roof,
        "chol_roofline": chol_roof,
        "estep_roofline": estep_roof,
    }
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        line["cpu_baseline"] = cpu_baseline(cfg, varn, args.seed,
                                            iters=2 if args.config in ("cfg1", "plumbing") else 1,
                                            mode=mode, part_r=part_r)
        line["cpu_baseline_reference_structured"] = cpu_baseline_reference_structured(
            cfg, varn, args.seed, mode=mode, part_r=part_r)
    if rank == 0:
        print(json.dumps(line), flush=True)
    ranks.close()


if __name__ == "__main__":
    main()
