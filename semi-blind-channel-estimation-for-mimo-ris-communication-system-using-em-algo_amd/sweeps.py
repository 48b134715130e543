"""Monte-Carlo sweep drivers: the reference's entry-point scripts, running the GPU
estimator with every trial of a sweep point batched into ONE sbce_em call.

  nmse_vs_tp   "Proposed method/Proposed_method_NMSEvsTp.py":133-176
  nmse_vs_td   "Proposed method/Proposed_method_NMSEvsTd.py":121-157
  nmse_vs_snr  "Proposed method/SNR/all_Detectors.py":331-395 (its five EMs: PM r=1, log-max,
               ZF, MMSE, exact)
  ser_vs_snr   "Proposed method/SER/log_max_SER.py":124-167 (log-max EM decisions)
  nmse_vs_tp_superimposed  "Parallel/ParallelProtocol_Tp.py":106-136 (superimposed pilots)
  nmse_vs_tp_gaussian      "Proposed method/MIMO_Gaussian_proposed.py":158-177 (Gaussian prior)
  nmse_grid_detectors      "Proposed method/all_detectorsvsTd.py":345-405 (five EMs per T_d
                           point), extended over an SNR axis (BASELINE configs[4])
  llf_vs_iteration         "Proposed method/IterationsvsLLF.py":119-157 (LLF per EM iteration)

Data generation (host, NumPy):
  replay=True   the reference's exact legacy-RandomState call order after
                np.random.seed(seed) (trials generated sequentially, so every rank
                replays the whole stream and keeps its own trials);
  replay=False  per-trial numpy Generators seeded (seed, trial): statistical parity,
                no sequential dependence (large sweeps / many GPUs).
Multi-GPU: when torch.distributed is initialised, trials are sharded
(distributed.shard) and the per-point accumulators are all-reduced ONCE at the end.
"""
import numpy as np

from . import signal_model as sm
from .distributed import Accumulators, shard
from .em import em_batch, ser_batch, gauss_expand_batch, nmse_batch, _GAUSS_CONS
from .qam import qam_constellation


def _dist():
    try:
        import torch.distributed as dist
        if dist.is_available() and dist.is_initialized():
            return dist, dist.get_world_size(), dist.get_rank()
    except ImportError:
        pass
    return None, 1, 0


def _trial_rng(seed, trial):
    return np.random.RandomState(np.random.SeedSequence([seed, trial]).generate_state(1)[0])


def _pack(trials, P):
    """Stack per-trial dicts into the batch-major C-ABI arrays."""
    return dict(
        y_d=np.stack([t["Y_d"] for t in trials]),
        y_p=np.stack([t["Y_p"] for t in trials]),
        psi_d=np.stack([t["Psi_d"].T for t in trials]),
        u_p=np.stack([t["U_p"] for t in trials]),
        theta0=np.stack([t["h0"] for t in trials]),
        h=np.stack([t["h"] for t in trials]),
    )


def _nmse(theta, h):
    return np.sum(np.abs(theta - h) ** 2, axis=1) / np.sum(np.abs(h) ** 2, axis=1)


def _run_points(points, cons, varns, itera, mode, acc, dist):
    for pt, (trials, varn) in enumerate(zip(points, varns)):
        if not trials:
            continue
        b = _pack(trials, None)
        r = em_batch(b["y_d"], b["y_p"], b["psi_d"], b["u_p"], cons, varn, itera, b["theta0"],
                     mode=mode)
        acc.add(pt, _nmse(r["theta"], b["h"]))
    return acc


def nmse_vs_tp(T_p=(4, 12, 20, 28, 36, 40), T_d=50, N=32, n_rx=4, n_tx=4, itera=3, monte_iter=1,
               M=4, varn=0.1, seed=0, replay=True, mode="soft", varh=1.0):
    """Mean NMSE per pilot length (PMd/Proposed_method_NMSEvsTp.py:154-176).

    Reference draw order per trial: channelMatrix, symbols(T_d), pilotSymbols(max T_p),
    then for each T_p: irsMatrix (T_d uniform draws), receivedSignals (noise)."""
    dist, world, rank = _dist()
    mine = set(shard(monte_iter, world, rank).tolist())
    points = [[] for _ in T_p]
    if replay:
        np.random.seed(seed)
    for i in range(monte_iter):
        rs = None if replay else _trial_rng(seed, i)
        if not replay and i not in mine:
            continue
        h = sm.channel_matrix(n_tx, n_rx, N, varh, rs=rs)
        X_d, _ = sm.symbols(n_tx, M, T_d, rs=rs)
        X_p = sm.pilot_symbols(n_tx, M, max(T_p), rs=rs)
        for k, tp in enumerate(T_p):
            Ptp, Ptd = sm.irs_matrix(tp, T_d, N, rs=rs)
            Ptd = sm.insert_direct(Ptd)
            Y_p, Y_d, U_p, _, h0 = sm.received_signals(tp, T_d, Ptp, Ptd, n_rx, n_tx, X_d, X_p[:tp],
                                                       h, varn, rs=rs)
            if i in mine:
                points[k].append(dict(Y_d=Y_d, Y_p=Y_p, Psi_d=Ptd, U_p=U_p, h0=h0, h=h))
    acc = Accumulators(len(T_p))
    _run_points(points, qam_constellation(M), [varn] * len(T_p), itera, mode, acc, dist)
    acc.allreduce(dist)
    return np.asarray(T_p), acc.mean_nmse()


def nmse_vs_td(T_d=(20, 30, 40, 50, 60, 70, 80, 90, 100), T_p=16, N=32, n_rx=2, n_tx=2, itera=3,
               monte_iter=1, M=4, varn=0.1, seed=0, replay=True, mode="soft", varh=1.0,
               variant="pmd"):
    """Mean NMSE per data length (PMd/Proposed_method_NMSEvsTd.py:140-157; C-order h, :15).

    Reference draw order per trial: channelMatrix, pilotSymbols(T_p), then for each T_d:
    symbols(T_d), irsMatrix, receivedSignals.
    variant='root': the root-level Proposed_method_NMSEvsTd.py -- the same draw order, N x T_p
    DFT pilot phases over T_p plus a ones row (:81-86, :95), deterministic (N+1) x T_d DFT data
    phases over T_d (:92-94, no RNG draw: signal_model.irs_matrix(data='dft_td')) and the EM
    started from theta = 0 (:46, em_zero_init)."""
    if variant not in ("pmd", "root"):
        raise ValueError(variant)
    root = variant == "root"
    dist, world, rank = _dist()
    mine = set(shard(monte_iter, world, rank).tolist())
    points = [[] for _ in T_d]
    if replay:
        np.random.seed(seed)
    for i in range(monte_iter):
        rs = None if replay else _trial_rng(seed, i)
        if not replay and i not in mine:
            continue
        h = sm.channel_matrix(n_tx, n_rx, N, varh, order="C", rs=rs)
        X_p = sm.pilot_symbols(n_tx, M, T_p, rs=rs)
        for k, td in enumerate(T_d):
            X_d, _ = sm.symbols(n_tx, M, td, rs=rs)
            if root:
                Ptp, Ptd = sm.irs_matrix(T_p, td, N, pilot="dft_tp", data="dft_td", rs=rs)
                Ptp = sm.insert_direct(Ptp)
            else:
                Ptp, Ptd = sm.irs_matrix(T_p, td, N, rs=rs)
            Ptd = sm.insert_direct(Ptd)
            Y_p, Y_d, U_p, _, h0 = sm.received_signals(T_p, td, Ptp, Ptd, n_rx, n_tx, X_d, X_p, h,
                                                       varn, rs=rs, with_initial=not root)
            if root:
                h0 = np.zeros(len(h), dtype=complex)
            if i in mine:
                points[k].append(dict(Y_d=Y_d, Y_p=Y_p, Psi_d=Ptd, U_p=U_p, h0=h0, h=h))
    acc = Accumulators(len(T_d))
    _run_points(points, qam_constellation(M), [varn] * len(T_d), itera, mode, acc, dist)
    acc.allreduce(dist)
    return np.asarray(T_d), acc.mean_nmse()


def gen_snr(SNR=(-5, 0, 5, 10, 15, 20), T_d=50, T_p=12, N=10, n_rx=2, n_tx=2, monte_iter=15, M=4,
            power=10.0, seed=0, replay=True, varh=1.0, keep=None):
    """Synthetic data of PMd/SNR/all_Detectors.py:362-370 in the reference draw order:
    per trial channelMatrix, symbols, pilotSymbols, irsMatrix once, then per SNR
    receivedSignals.  Returns (points, varns): points[k] = list of per-trial dicts."""
    varns = sm.snr_to_varn(SNR, power)
    keep = set(range(monte_iter)) if keep is None else set(keep)
    points = [[] for _ in SNR]
    if replay:
        np.random.seed(seed)
    for i in range(monte_iter):
        rs = None if replay else _trial_rng(seed, i)
        if not replay and i not in keep:
            continue
        h = sm.channel_matrix(n_tx, n_rx, N, varh, rs=rs)
        X_d, _ = sm.symbols(n_tx, M, T_d, rs=rs)
        X_p = sm.pilot_symbols(n_tx, M, T_p, rs=rs)
        Ptp, Ptd = sm.irs_matrix(T_p, T_d, N, rs=rs)
        Ptd = sm.insert_direct(Ptd)
        for k in range(len(SNR)):
            Y_p, Y_d, U_p, _, h0 = sm.received_signals(T_p, T_d, Ptp, Ptd, n_rx, n_tx, X_d, X_p, h,
                                                       varns[k], rs=rs)
            if i in keep:
                points[k].append(dict(Y_d=Y_d, Y_p=Y_p, Psi_d=Ptd, U_p=U_p, h0=h0, h=h,
                                      X_d=np.stack([x.reshape(-1) for x in X_d])))
    return points, varns


# The five EMs of the NMSE-vs-SNR figure, PMd/SNR/all_Detectors.py:372-377, in the script's call
# order: (E-step mode, reference EM, oracle early stop on the true h as THIS script has it, plot
# label :396-401).  Unlike all_detectorsvsTd.py (DETECTORS below, every EM stops), only em_pm
# stops here (:234-236); em_zf's stop is commented out (:125-127); em_mmse, em_ml, em have none.
SNR_DETECTORS = {
    "pm_soft": ("em_pm :170-240 (posterior-weighted list, partition_r_1 = 1)", True,
                "Soft decision-PM r =1"),
    "hard": ("em_ml :132-167 (log-max)", False, "log-max"),
    "zf": ("em_zf :92-130", False, "Zero forcing"),
    "mmse": ("em_mmse :53-90", False, "MMSE"),
    "soft": ("em :242-274 (exact posterior)", False, "Exact"),
}


def _snr_groups(points, varns, batch_snr):
    """The sbce_em calls of an SNR axis: with batch_snr ONE call over the trials of every SNR
    point (per-trial noise variances, include/sbce.h sbce_ptrs.varn_t), else one call per point.
    Yields (SNR indices, trials per index, packed batch, varn scalar or (B,) array)."""
    live = [k for k, t in enumerate(points) if t]
    if not live:
        return
    if batch_snr and len(live) > 1:
        trials = [t for k in live for t in points[k]]
        vt = np.concatenate([np.full(len(points[k]), varns[k]) for k in live])
        yield live, [len(points[k]) for k in live], _pack(trials, None), vt
    else:
        for k in live:
            yield [k], [len(points[k])], _pack(points[k], None), varns[k]


def nmse_vs_snr(SNR=(-5, 0, 5, 10, 15, 20), T_d=50, T_p=12, N=10, n_rx=2, n_tx=2, itera=5,
                monte_iter=15, M=4, power=10.0, seed=0, replay=True, modes=tuple(SNR_DETECTORS),
                varh=1.0, partition_r=1, return_status=False, batch_snr=True):
    """Mean NMSE per SNR of the five EMs of PMd/SNR/all_Detectors.py (driver :362-395; varn =
    power / 10^(SNR/10), :351-354): em_pm (r = 1), em_ml, em_zf, em_mmse and the exact em, each
    with that script's own early-stop pattern (SNR_DETECTORS) and np.linalg.solve M-step.

    One batched sbce_em per detector over this rank's trials of EVERY SNR point (per-trial noise
    variances; batch_snr=False: one call per (SNR point, detector), the same results); the
    accumulators of every (detector, SNR) point are all-reduced ONCE at the end.  Returns (SNR, {mode: curve});
    with return_status also {mode: (len(SNR),) count of trials whose status word is non-zero
    (e.g. SBCE_STATUS_DETECTOR: the reference's nearest_symbol_ecul would raise IndexError)}."""
    dist, world, rank = _dist()
    mine = shard(monte_iter, world, rank).tolist()
    points, varns = gen_snr(SNR, T_d, T_p, N, n_rx, n_tx, monte_iter, M, power, seed, replay,
                            varh, keep=mine)
    cons = qam_constellation(M)
    nm, ns = len(modes), len(SNR)
    acc = Accumulators(nm * ns, n_extra=1)
    for ks, counts, b, vn in _snr_groups(points, varns, batch_snr):
        for mi, mode in enumerate(modes):
            stop = SNR_DETECTORS[mode][1]
            r = em_batch(b["y_d"], b["y_p"], b["psi_d"], b["u_p"], cons, vn, itera,
                         b["theta0"], mode=mode,
                         partition_r=partition_r if mode.startswith("pm") else 0,
                         h_true=b["h"] if stop else None)
            err, flag = _nmse(r["theta"], b["h"]), (r["status"] != 0).astype(float)[:, None]
            off = np.cumsum([0] + counts)
            for k, o0, o1 in zip(ks, off[:-1], off[1:]):
                acc.add(mi * ns + k, err[o0:o1], extra_values=flag[o0:o1])
    acc.allreduce(dist)                   # the sweep's only collective
    mean = acc.mean_nmse().reshape(nm, ns)
    curves = {mode: mean[mi] for mi, mode in enumerate(modes)}
    if return_status:
        flagged = acc.extra[:, 0].reshape(nm, ns)
        return np.asarray(SNR), curves, {mode: flagged[mi] for mi, mode in enumerate(modes)}
    return np.asarray(SNR), curves


def gen_ser(SNR=(-5, 0, 5, 10, 15, 20), T_d=50, T_p=20, N=30, n_rx=2, n_tx=2, monte_iter=75, M=4,
            power=10.0, seed=0, replay=True, varh=1.0, keep=None):
    """Synthetic data of PMd/SER/log_max_SER.py:150-160 in the reference draw order: per
    trial channelMatrix, symbols(T_d), irsMatrix (pilot phases (N+1) x T_p with a zero last
    row; ones row inserted into the data phases), pilotSymbols, then per SNR
    receivedSignals."""
    varns = sm.snr_to_varn(SNR, power)
    keep = set(range(monte_iter)) if keep is None else set(keep)
    points = [[] for _ in SNR]
    if replay:
        np.random.seed(seed)
    for i in range(monte_iter):
        rs = None if replay else _trial_rng(seed, i)
        if not replay and i not in keep:
            continue
        h = sm.channel_matrix(n_tx, n_rx, N, varh, rs=rs)
        X_d, _ = sm.symbols(n_tx, M, T_d, rs=rs)
        Ptp, Ptd = sm.irs_matrix(T_p, T_d, N, pilot="dft_n", rs=rs)
        Ptd = sm.insert_direct(Ptd)
        X_p = sm.pilot_symbols(n_tx, M, T_p, rs=rs)
        for k in range(len(SNR)):
            Y_p, Y_d, U_p, _, h0 = sm.received_signals(T_p, T_d, Ptp, Ptd, n_rx, n_tx, X_d, X_p, h,
                                                       varns[k], rs=rs)
            if i in keep:
                points[k].append(dict(Y_d=Y_d, Y_p=Y_p, Psi_d=Ptd, U_p=U_p, h0=h0, h=h,
                                      X_d=np.stack([x.reshape(-1) for x in X_d])))
    return points, varns


def ser_vs_snr(SNR=(-5, 0, 5, 10, 15, 20), T_d=50, T_p=20, N=30, n_rx=2, n_tx=2, itera=5,
               monte_iter=75, M=4, power=10.0, seed=0, replay=True, varh=1.0):
    """SER per SNR of the log-max EM's last-iteration decisions (PMd/SER/log_max_SER.py:
    constants :124-147, driver :150-167).  Returns (SNR, ser_reference, ser_elementwise,
    nmse): ser_reference is the script's own expression (:162, a (T_d, n_tx, n_tx)
    broadcast count), ser_elementwise the per-symbol-entry error rate.

    Reference draw order per trial: channelMatrix, symbols(T_d), irsMatrix (ones row
    inserted, pilot phases (N+1) x T_p with a zero last row), pilotSymbols, then per SNR
    receivedSignals (gen_ser)."""
    dist, world, rank = _dist()
    mine = shard(monte_iter, world, rank).tolist()
    points, varns = gen_ser(SNR, T_d, T_p, N, n_rx, n_tx, monte_iter, M, power, seed, replay,
                            varh, keep=mine)
    acc = Accumulators(len(SNR), n_extra=2)
    cons = qam_constellation(M)
    for pt, trials in enumerate(points):
        if not trials:
            continue
        b = _pack(trials, None)
        r = em_batch(b["y_d"], b["y_p"], b["psi_d"], b["u_p"], cons, varns[pt], itera,
                     b["theta0"], mode="hard", return_decisions=True)
        x_true = np.stack([t["X_d"] for t in trials])
        s_ref, s_el = ser_batch(r["x_dest"], x_true)
        acc.add(pt, _nmse(r["theta"], b["h"]), extra_values=np.stack([s_ref, s_el], axis=1))
    acc.allreduce(dist)
    ser = acc.mean_extra()
    return np.asarray(SNR), ser[:, 0], ser[:, 1], acc.mean_nmse()


def gen_superimposed(T_p=(4, 8, 12, 16, 20, 24, 28, 32, 36, 40), T_d=50, N=32, n_rx=8, n_tx=1,
                     monte_iter=50, M=16, varn=0.1, seed=0, replay=True, varh=1.0, keep=None):
    """Data of Parallel/ParallelProtocol_Tp.py:114-122 in the reference draw order: per
    trial channelMatrix (C-order h, :10-16), symbols(T_d); per T_p irsMatrix(T, N)
    ((N+1) x T DFT, deterministic), pilotSymbols, dataPilotSymbols (zero-padded sum),
    receivedSignals (one noise draw per symbol)."""
    keep = set(range(monte_iter)) if keep is None else set(keep)
    points = [[] for _ in T_p]
    if replay:
        np.random.seed(seed)
    for i in range(monte_iter):
        rs = None if replay else _trial_rng(seed, i)
        if not replay and i not in keep:
            continue
        h = sm.channel_matrix(n_tx, n_rx, N, varh, order="C", rs=rs)
        X_d, _ = sm.symbols(n_tx, M, T_d, rs=rs)
        for k, tp in enumerate(T_p):
            T = max(T_d, tp)
            Psi = sm.dft_phases(N + 1, T, T)
            X_p = sm.pilot_symbols(n_tx, M, tp, rs=rs)
            xd = np.zeros((T, n_tx), dtype=complex)
            xp = np.zeros((T, n_tx), dtype=complex)
            xd[:T_d] = np.stack([x.reshape(-1) for x in X_d])
            xp[:tp] = np.stack([x.reshape(-1) for x in X_p])
            X = xd + xp
            _, Y, _, _, _ = sm.received_signals(0, T, Psi[:, :0], Psi, n_rx, n_tx, list(X), [], h,
                                                varn, rs=rs, with_initial=False)
            if i in keep:
                points[k].append(dict(Y=Y, Psi=Psi, X_sup=xp, h=h))
    return points


def nmse_vs_tp_superimposed(T_p=(4, 8, 12, 16, 20, 24, 28, 32, 36, 40), T_d=50, N=32, n_rx=8,
                            n_tx=1, itera=20, monte_iter=50, M=16, varn=0.1, seed=0, replay=True,
                            varh=1.0):
    """Mean NMSE per pilot length of the superimposed-pilot protocol
    (Parallel/ParallelProtocol_Tp.py:106-136; NMSE :129)."""
    dist, world, rank = _dist()
    mine = shard(monte_iter, world, rank).tolist()
    points = gen_superimposed(T_p, T_d, N, n_rx, n_tx, monte_iter, M, varn, seed, replay, varh,
                              keep=mine)
    acc = Accumulators(len(T_p))
    cons = qam_constellation(M)
    for k, trials in enumerate(points):
        if not trials:
            continue
        L = (N + 1) * n_tx
        B = len(trials)
        r = em_batch(np.stack([t["Y"] for t in trials]), np.zeros((B, 0, n_rx), dtype=complex),
                     np.stack([t["Psi"].T for t in trials]), np.zeros((B, 0, L), dtype=complex),
                     cons, varn, itera, np.zeros((B, L * n_rx), dtype=complex), mode="soft",
                     x_sup=np.stack([t["X_sup"] for t in trials]))
        acc.add(k, _nmse(r["theta"], np.stack([t["h"] for t in trials])))
    acc.allreduce(dist)
    return np.asarray(T_p), acc.mean_nmse()


def gen_gaussian(T_p=(8, 12, 16, 20, 24, 28, 32, 36, 40), T_d=50, N=32, n_rx=2, n_tx=2,
                 monte_iter=1, varn=0.1, varx=1.0, seed=0, replay=True, varh=1.0, keep=None):
    """Data of MIMO_Gaussian_proposed.py:160-169 in the reference draw order: per trial
    channelMatrix1 and symbols(n_tx, T_d, varx); per T_p irsMatrix (N x T_p DFT + T_d
    uniform phase draws), pilotSymbols, received_proposed (one noise draw per symbol).
    Reduced form: u_p = psi_p (x) x_p, y = H z = H_r u, h_initial = Y_p pinv(Z_p) reduced."""
    keep = set(range(monte_iter)) if keep is None else set(keep)
    points = [[] for _ in T_p]
    if replay:
        np.random.seed(seed)
    for i in range(monte_iter):
        rs = None if replay else _trial_rng(seed, i)
        if not replay and i not in keep:
            continue
        h = sm.gaussian_channel(varh, N, n_rx, n_tx, rs=rs)
        X_d = sm.gaussian_symbols(n_tx, T_d, varx, rs=rs)
        for k, tp in enumerate(T_p):
            Ptp, Ptd = sm.irs_matrix(tp, T_d, N, pilot="dft_n", rs=rs)
            Ptp = Ptp[:N]
            X_p = sm.gaussian_symbols(n_tx, tp, varx, rs=rs)
            Y_p, Y_d, U_p, _, h0 = sm.received_signals(tp, T_d, Ptp, Ptd, n_rx, n_tx, X_d.T,
                                                       X_p.T, h, varn, rs=rs)
            if i in keep:
                points[k].append(dict(Y_d=Y_d, Y_p=Y_p, U_p=U_p, Psi_d=Ptd, h0=h0, h=h))
    return points


def nmse_vs_tp_gaussian(T_p=(8, 12, 16, 20, 24, 28, 32, 36, 40), T_d=50, N=32, n_rx=2, n_tx=2,
                        itera=3, monte_iter=1, varn=0.1, varx=1.0, seed=0, replay=True,
                        varh=1.0):
    """Mean NMSE per pilot length of the Gaussian-prior EM (MIMO_Gaussian_proposed.py:
    158-177): trace(|(H_hat - H)^H (H_hat - H)|) / ||H||^2 (:173) on the full n_rx x Q
    matrices, H_hat = the reference-format expansion of the device estimate."""
    dist, world, rank = _dist()
    mine = shard(monte_iter, world, rank).tolist()
    points = gen_gaussian(T_p, T_d, N, n_rx, n_tx, monte_iter, varn, varx, seed, replay, varh,
                          keep=mine)
    acc = Accumulators(len(T_p))
    for k, trials in enumerate(points):
        if not trials:
            continue
        d = _pack(trials, N)
        r = em_batch(d["y_d"], d["y_p"], d["psi_d"], d["u_p"], _GAUSS_CONS, varn, itera + 1,
                     d["theta0"], mode="gauss", varx=varx, solve="drop", return_device=True)
        Hh = gauss_expand_batch(r["theta"], n_tx, n_rx, return_device=True)
        Hf = np.stack([sm.full_gaussian_channel(h, n_rx).reshape(-1) for h in d["h"]])
        acc.add(k, nmse_batch(Hh.reshape(len(trials), -1), Hf).cpu().numpy())
    acc.allreduce(dist)
    return np.asarray(T_p), acc.mean_nmse()


# (E-step mode, reference EM of all_detectorsvsTd.py, its plot label :407-411)
DETECTORS = {
    "pm_soft": ("em_pm :176-249 (posterior-weighted list, partition_r)", "Soft decision-PM"),
    "hard": ("em_ml :135-173 (log-max)", "Non - Superimposed log-max"),
    "zf": ("em_zf :95-133", "Zero forcing"),
    "mmse": ("em_mmse :54-93", "MMSE"),
    "soft": ("em :260-295 (exact posterior)", "Non - Superimposed"),
}


def gen_detectors(T_d=(15, 30, 45, 60, 75, 90), SNR=None, T_p=20, N=15, n_rx=2, n_tx=2,
                  monte_iter=1, M=4, varn=0.1, power=10.0, seed=0, replay=True, varh=1.0,
                  keep=None):
    """Data of PMd/all_detectorsvsTd.py:371-382 in its draw order: per trial channelMatrix,
    pilotSymbols(T_p); per T_d point symbols(T_d), irsMatrix (pilot phases (N+1) x T_p DFT
    with a zero last row, T_d uniform data-phase columns), the ones row inserted, then
    receivedSignals (h_initial by scipy.linalg.pinv, :341) -- once with the script's varn
    (SNR=None), or once per SNR point in SNR order (the grid extension of BASELINE
    configs[4]; varn = power / 10^(SNR/10), SNR/all_Detectors.py:351-354).  Returns (points[k_td][k_snr] = trial dicts, varns)."""
    varns = [float(varn)] if SNR is None else [float(v) for v in sm.snr_to_varn(SNR, power)]
    keep = set(range(monte_iter)) if keep is None else set(keep)
    points = [[[] for _ in varns] for _ in T_d]
    if replay:
        np.random.seed(seed)
    for i in range(monte_iter):
        rs = None if replay else _trial_rng(seed, i)
        if not replay and i not in keep:
            continue
        h = sm.channel_matrix(n_tx, n_rx, N, varh, rs=rs)
        X_p = sm.pilot_symbols(n_tx, M, T_p, rs=rs)
        for k, td in enumerate(T_d):
            X_d, _ = sm.symbols(n_tx, M, td, rs=rs)
            Ptp, Ptd = sm.irs_matrix(T_p, td, N, pilot="dft_n", rs=rs)
            Ptd = sm.insert_direct(Ptd)
            for j, vn in enumerate(varns):
                Y_p, Y_d, U_p, _, h0 = sm.received_signals(T_p, td, Ptp, Ptd, n_rx, n_tx, X_d,
                                                           X_p, h, vn, rs=rs, pinv="scipy")
                if i in keep:
                    points[k][j].append(dict(Y_d=Y_d, Y_p=Y_p, Psi_d=Ptd, U_p=U_p, h0=h0, h=h))
    return points, varns


def nmse_grid_detectors(T_d=(15, 30, 45, 60, 75, 90), SNR=None, T_p=20, N=15, n_rx=2, n_tx=2,
                        itera=5, monte_iter=1, M=4, varn=0.1, power=10.0, partition_r=1, seed=0,
                        replay=True, detectors=tuple(DETECTORS), early_stop=True, varh=1.0,
                        batch_snr=True):
    """Mean NMSE of the five EMs of PMd/all_detectorsvsTd.py (:384-405) per T_d point, and
    per SNR point when SNR is given (BASELINE configs[4]: 20 SNR x 8 T_d, 64-QAM).

    One batched sbce_em per (T_d, detector) over this rank's trials of every SNR point (per-trial
    noise variances; batch_snr=False: one per (T_d, SNR, detector), the same results); every EM
    keeps the script's oracle early stop on the true h (:87-89, :128-130, :169-171, :243-245,
    :291-293) unless early_stop=False, and its np.linalg.solve M-step (SBCE_SOLVE_CHOL).
    The accumulators of the whole grid are all-reduced once.  Returns (T_d, SNR or None,
    {detector: (len(T_d), len(SNR or [varn])) mean NMSE})."""
    dist, world, rank = _dist()
    mine = shard(monte_iter, world, rank).tolist()
    points, varns = gen_detectors(T_d, SNR, T_p, N, n_rx, n_tx, monte_iter, M, varn, power, seed,
                                  replay, varh, keep=mine)
    cons = qam_constellation(M)
    nd, nt, ns = len(detectors), len(T_d), len(varns)
    acc = Accumulators(nd * nt * ns)
    for k in range(nt):
        for js, counts, b, vn in _snr_groups(points[k], varns, batch_snr):
            off = np.cumsum([0] + counts)
            for di, det in enumerate(detectors):
                r = em_batch(b["y_d"], b["y_p"], b["psi_d"], b["u_p"], cons, vn, itera,
                             b["theta0"], mode=det, partition_r=partition_r if det == "pm_soft" else 0,
                             h_true=b["h"] if early_stop else None)
                nm = _nmse(r["theta"], b["h"])
                for j, o0, o1 in zip(js, off[:-1], off[1:]):
                    acc.add((di * nt + k) * ns + j, nm[o0:o1])
    acc.allreduce(dist)
    mean = acc.mean_nmse().reshape(nd, nt, ns)
    return (np.asarray(T_d), None if SNR is None else np.asarray(SNR),
            {det: mean[di] for di, det in enumerate(detectors)})


def gen_llf(T_d=50, T_p=4, N=32, n_rx=2, n_tx=2, monte_iter=3, M=4, varn=0.1, seed=0,
            replay=True, varh=1.0, keep=None):
    """Data of PMd/IterationsvsLLF.py:140-149 in its draw order per trial: channelMatrix
    (row-major flatten of h, :16), symbols(T_d), irsMatrix (pilot phases N x T_p DFT over N, :90-92), ones rows inserted into
    the pilot and data phases (:144-145), pilotSymbols, receivedSignals."""
    keep = set(range(monte_iter)) if keep is None else set(keep)
    trials = []
    if replay:
        np.random.seed(seed)
    for i in range(monte_iter):
        rs = None if replay else _trial_rng(seed, i)
        if not replay and i not in keep:
            continue
        h = sm.channel_matrix(n_tx, n_rx, N, varh, order="C", rs=rs)
        X_d, _ = sm.symbols(n_tx, M, T_d, rs=rs)
        Ptp, Ptd = sm.irs_matrix(T_p, T_d, N, pilot="dft_n", rs=rs)
        Ptp = sm.insert_direct(Ptp[:N])
        Ptd = sm.insert_direct(Ptd)
        X_p = sm.pilot_symbols(n_tx, M, T_p, rs=rs)
        Y_p, Y_d, U_p, _, h0 = sm.received_signals(T_p, T_d, Ptp, Ptd, n_rx, n_tx, X_d, X_p, h,
                                                   varn, rs=rs)
        if i in keep:
            trials.append(dict(Y_d=Y_d, Y_p=Y_p, Psi_d=Ptd, U_p=U_p, h0=h0, h=h,
                               X_d=np.stack([x.reshape(-1) for x in X_d])))
    return trials


def llf_vs_iteration(T_d=50, T_p=4, N=32, n_rx=2, n_tx=2, itera=5, monte_iter=3, M=4, varn=0.1,
                     seed=0, replay=True, varh=1.0):
    """Mean log-likelihood per EM iteration (PMd/IterationsvsLLF.py:139-154): the exact EM
    (:45-77) with the script's genie LLF (:76: un-squared norms, Z_d from the TRUE data
    symbols), averaged over trials (gen_llf data).  Returns (iterations, mean LLF, mean final
    NMSE)."""
    dist, world, rank = _dist()
    trials = gen_llf(T_d, T_p, N, n_rx, n_tx, monte_iter, M, varn, seed, replay, varh,
                     keep=shard(monte_iter, world, rank).tolist())
    acc = Accumulators(1, n_iters=itera)
    if trials:
        b = _pack(trials, None)
        r = em_batch(b["y_d"], b["y_p"], b["psi_d"], b["u_p"], qam_constellation(M), varn, itera,
                     b["theta0"], mode="soft", x_d_true=np.stack([t["X_d"] for t in trials]))
        acc.add(0, _nmse(r["theta"], b["h"]), llf_values=r["llf"])
    acc.allreduce(dist)
    return np.arange(itera), acc.mean_llf()[0], float(acc.mean_nmse()[0])
