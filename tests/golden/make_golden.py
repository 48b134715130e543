"""Generate the golden fixtures under tests/golden/ by running the REFERENCE's own
estimator functions in this (CPU) container.

This script is test infrastructure. It reads /root/reference (read-only) as the
oracle of record and is never run on the GPU box; only the .npz files it writes
travel. Nothing here is imported by the product package.

How the reference is loaded:
  * every reference script runs a Monte-Carlo sweep and ``plt.show()`` at module
    top level, so only its ``import`` and ``def`` statements are executed
    (``ast`` filter), into a namespace pre-seeded with the module globals the
    functions read (``N``, ``n_tx``, ``beta_min``/``beta_max``, ``qamCons``,
    ``Z_d``, ``h``);
  * ``gmpy2`` is not installed: ``gmpy2.exp`` is bound to ``mpmath.exp`` (both
    return a 53-bit-mantissa number with unbounded exponent);
  * ``Proposed method/QAM.py`` uses the NumPy aliases removed in NumPy 2
    (``np.int``/``np.float``/``np.complex``): they are restored as the builtins.
  * ``sys.dont_write_bytecode`` keeps ``__pycache__`` out of the reference tree.

Synthetic data for every case is produced by the reference's own helpers
(``channelMatrix``, ``symbols``, ``pilotSymbols``, ``irsMatrix``,
``receivedSignals``) in the reference's own RNG call order after
``np.random.seed(seed)``, so the fixtures also pin the build's signal-model
replay (``signal_model.py``).

Usage:  python tests/golden/make_golden.py [case ...]     (default: all cases)
"""
import ast
import contextlib
import io
import os
import sys
import time
from multiprocessing import Pool

sys.dont_write_bytecode = True
os.environ.setdefault("MPLBACKEND", "Agg")

import numpy as np  # noqa: E402

REF = "/root/reference"
PMD = os.path.join(REF, "Proposed method")
OUT = os.path.dirname(os.path.abspath(__file__))


def _shim_env():
    import mpmath
    for name, typ in (("int", int), ("float", float), ("complex", complex)):
        if not hasattr(np, name):
            setattr(np, name, typ)
    sys.modules.setdefault("gmpy2", mpmath)
    if PMD not in sys.path:
        sys.path.insert(0, PMD)


def load_defs(path, **globs):
    """Execute only the import/def statements of a reference script."""
    _shim_env()
    src = open(path).read()
    tree = ast.parse(src, filename=path)
    keep = [n for n in tree.body
            if isinstance(n, (ast.Import, ast.ImportFrom, ast.FunctionDef))]
    mod = ast.Module(body=keep, type_ignores=[])
    ns = {"__name__": "refdefs", "np": np}
    ns.update(globs)
    with contextlib.redirect_stdout(io.StringIO()):
        exec(compile(mod, path, "exec"), ns)
    return ns


def nmse(theta, h):
    theta = np.asarray(theta).reshape(-1)
    return float(np.sum(np.abs(theta - h) ** 2) / np.sum(np.abs(h) ** 2))


def quiet(fn, *a):
    with contextlib.redirect_stdout(io.StringIO()):
        return fn(*a)


def _gen_northstar(ns, seed, N, n_tx, n_rx, T_d, T_p, M, varn):
    """PMd/Proposed_method_NMSEvsTp.py call order (:155-163)."""
    np.random.seed(seed)
    h = quiet(ns["channelMatrix"], n_tx, n_rx, N, 1)
    X_d, aps = ns["symbols"](n_tx, M, T_d)[:2]
    X_p = ns["pilotSymbols"](n_tx, M, T_p)
    Ptp, Ptd = ns["irsMatrix"](T_p, T_d, N, 0, 1)
    Ptd = np.insert(Ptd, 0, np.ones((1, T_d), dtype="complex128"), axis=0)
    Y_p, Y_d, Z_p, Z_d, h0 = ns["receivedSignals"](T_p, T_d, Ptp, Ptd, n_rx, n_tx,
                                                   X_d, X_p, h, varn, M)
    return dict(h=h, X_d=X_d, aps=aps, X_p=X_p, Ptp=Ptp, Ptd=Ptd, Y_p=Y_p, Y_d=Y_d,
                Z_p=Z_p, Z_d=Z_d, h0=h0)


def _pack(d, **extra):
    """Store the inputs in array form (lists of per-symbol arrays are stacked)."""
    out = dict(
        h=np.asarray(d["h"]),
        X_d=np.stack(d["X_d"])[..., 0],
        X_p=np.stack(d["X_p"])[..., 0],
        aps=np.asarray(d["aps"]),
        Ptp=np.asarray(d["Ptp"]),
        Ptd=np.asarray(d["Ptd"]),
        Y_p=np.stack(d["Y_p"])[..., 0],
        Y_d=np.stack(d["Y_d"])[..., 0],
        Z_p=np.stack(d["Z_p"]),
        h0=np.asarray(d["h0"]).reshape(-1),
    )
    out.update(extra)
    return out


def _cons(M):
    _shim_env()
    import QAM as qp  # reference's vendored komm QAM, Proposed method/QAM.py:246-336
    return np.asarray(qp.QAModulation(M).constellation)


# ----------------------------------------------------------------------------- cases

def case_kat1(seed):
    """KAT-1: PMd/Proposed_method_NMSEvsTp.py helpers + em (:50-83)."""
    N, n_tx, n_rx, T_d, T_p, M, varn = 8, 2, 2, 40, 12, 4, 0.1
    ns = load_defs(os.path.join(PMD, "Proposed_method_NMSEvsTp.py"),
                   N=N, n_tx=n_tx, n_rx=n_rx, beta_min=0.0, beta_max=2 * np.pi)
    d = _gen_northstar(ns, seed, N, n_tx, n_rx, T_d, T_p, M, varn)
    res = {}
    for it in (1, 2):
        th = quiet(ns["em"], d["Y_d"], d["Y_p"], T_d, T_p, d["Z_p"], d["Ptd"], d["aps"],
                   M, varn, it, d["h0"])
        res[f"theta_it{it}"] = np.asarray(th).reshape(-1)
    extra = dict(res)
    extra["nmse_it2"] = nmse(res["theta_it2"], d["h"])
    extra["nmse_init"] = nmse(d["h0"], d["h"])
    if seed == 7:
        # same data through the LLF / hard-ML / PM variants
        ns_llf = load_defs(os.path.join(PMD, "IterationsvsLLF.py"), N=N,
                           beta_min=0.0, beta_max=2 * np.pi)
        th, llf = quiet(ns_llf["em"], d["Y_d"], d["Y_p"], T_d, T_p, d["Z_p"], d["Z_d"],
                        d["Ptd"], d["aps"], M, varn, 2, d["h0"], n_tx)
        extra["llf_soft_theta"] = np.asarray(th).reshape(-1)
        extra["llf_soft"] = np.asarray(llf).reshape(-1)
        ns_ml = load_defs(os.path.join(PMD, "ML_detecctor.py"), N=N, n_tx=n_tx,
                          Z_d=d["Z_d"], beta_min=0.0, beta_max=2 * np.pi)
        th, llf = quiet(ns_ml["em"], d["Y_d"], d["Y_p"], T_d, T_p, d["Z_p"], d["Ptd"],
                        d["aps"], M, varn, 2, d["h0"])
        extra["ml_theta"] = np.asarray(th).reshape(-1)
        extra["ml_llf"] = np.asarray(llf).reshape(-1)
        cons = _cons(M)
        ns_pm = load_defs(os.path.join(PMD, "PM.py"), N=N, beta_min=0.0,
                          beta_max=2 * np.pi)
        th = quiet(ns_pm["em_pm"], d["Y_d"], d["Y_p"], T_d, T_p, d["Z_p"], d["Ptd"],
                   d["aps"], M, varn, 3, d["h0"], d["h"], n_tx, 0, d["X_d"], cons)
        extra["pm_r0_theta"] = np.asarray(th).reshape(-1)
        ns_pmb = load_defs(os.path.join(PMD, "PM_beta.py"), N=N, qamCons=cons,
                           beta_min=0.0, beta_max=2 * np.pi)
        th = quiet(ns_pmb["em_pm"], d["Y_d"], d["Y_p"], T_d, T_p, d["Z_p"], d["Ptd"],
                   M, varn, 3, d["h0"], d["h"], n_tx, 1, d["X_d"], cons)
        extra["pmbeta_r1_theta"] = np.asarray(th).reshape(-1)
        ns_all = load_defs(os.path.join(PMD, "all_detectorsvsTd.py"), N=N, n_tx=n_tx,
                           qamCons=cons, h=d["h"], Z_d=d["Z_d"], beta_min=0.0,
                           beta_max=2 * np.pi)
        th = quiet(ns_all["em_zf"], d["Y_d"], d["Y_p"], T_d, T_p, d["Z_p"], d["Ptd"],
                   d["aps"], M, varn, 3, d["h0"], d["h"])
        extra["zf_theta"] = np.asarray(th).reshape(-1)
        th = quiet(ns_all["em_mmse"], d["Y_d"], d["Y_p"], T_d, T_p, d["Z_p"], d["Ptd"],
                   d["aps"], M, varn, 3, d["h0"], d["h"])
        extra["mmse_theta"] = np.asarray(th).reshape(-1)
    return f"kat1_s{seed}", _pack(d, N=N, n_tx=n_tx, n_rx=n_rx, T_d=T_d, T_p=T_p, M=M,
                                  varn=varn, seed=seed, **extra)


def case_kat2():
    """KAT-2: PMd/SNR/all_Detectors.py, em (:242-274), driver order :362-377."""
    N, n_tx, n_rx, T_d, T_p, M, itera = 10, 2, 2, 50, 12, 4, 5
    SNR = [-5, 0, 5, 10, 15, 20]
    varns = np.array([10 / np.power(10, s / 10) for s in SNR])
    ns = load_defs(os.path.join(PMD, "SNR", "all_Detectors.py"), N=N, n_tx=n_tx,
                   beta_min=0.0, beta_max=2 * np.pi)
    np.random.seed(0)
    h = quiet(ns["channelMatrix"], n_tx, n_rx, N, 1)
    X_d, aps, qamCons = ns["symbols"](n_tx, M, T_d)
    X_p = ns["pilotSymbols"](n_tx, M, T_p)
    Ptp, Ptd = ns["irsMatrix"](T_p, T_d, N, 0, 1)
    Ptd = np.insert(Ptd, 0, np.ones((1, T_d), dtype="complex128"), axis=0)
    Yps, Yds, h0s, thetas, thetas_ml, nm, nm_ml = [], [], [], [], [], [], []
    for k in range(len(SNR)):
        Y_p, Y_d, Z_p, Z_d, h0 = ns["receivedSignals"](T_p, T_d, Ptp, Ptd, n_rx, n_tx,
                                                        X_d, X_p, h, varns[k], M)
        th = quiet(ns["em"], Y_d, Y_p, T_d, T_p, Z_p, Ptd, aps, M, varns[k], itera, h0)
        thm = quiet(ns["em_ml"], Y_d, Y_p, T_d, T_p, Z_p, Ptd, aps, M, varns[k], itera, h0)
        Yps.append(np.stack(Y_p)[..., 0]); Yds.append(np.stack(Y_d)[..., 0])
        h0s.append(np.asarray(h0).reshape(-1))
        thetas.append(np.asarray(th).reshape(-1)); thetas_ml.append(np.asarray(thm).reshape(-1))
        nm.append(nmse(th, h)); nm_ml.append(nmse(thm, h))
    return "kat2_snr", dict(
        h=h, X_d=np.stack(X_d)[..., 0], X_p=np.stack(X_p)[..., 0], aps=aps, Ptp=Ptp,
        Ptd=Ptd, Z_p=np.stack(Z_p), Y_p=np.stack(Yps), Y_d=np.stack(Yds),
        h0=np.stack(h0s), theta=np.stack(thetas), theta_ml=np.stack(thetas_ml),
        nmse=np.array(nm), nmse_ml=np.array(nm_ml), snr=np.array(SNR), varn=varns,
        N=N, n_tx=n_tx, n_rx=n_rx, T_d=T_d, T_p=T_p, M=M, itera=itera, seed=0)


_SNR_DETS = ("pm", "ml", "zf", "mmse", "em")


def _kat2_driver_job(job):
    """One (trial, SNR point) of PMd/SNR/all_Detectors.py's driver: its five EMs in the order of
    :372-377, each with the script's own early-stop pattern (em_pm stops on the true h, :234-236;
    em_zf's stop is commented out, :125-127; em_mmse, em_ml and em have none)."""
    i, k, d, varn, N, n_tx, M, T_d, T_p, itera, partition_r = job
    ns = load_defs(os.path.join(PMD, "SNR", "all_Detectors.py"), N=N, n_tx=n_tx,
                   beta_min=0.0, beta_max=2 * np.pi, qamCons=d["cons"])
    common = (d["Y_d"], d["Y_p"], T_d, T_p, d["Z_p"], d["Ptd"])
    out = {}
    for det in _SNR_DETS:
        try:
            if det == "pm":
                th = quiet(ns["em_pm"], *common, M, varn, itera, d["h0"], d["h"], n_tx, partition_r,
                           d["X_d"], d["cons"])
            elif det == "ml":
                th = quiet(ns["em_ml"], *common, d["aps"], M, varn, itera, d["h0"])
            elif det == "zf":
                th = quiet(ns["em_zf"], *common, d["aps"], M, varn, itera, d["h0"], d["h"])
            elif det == "mmse":
                th = quiet(ns["em_mmse"], *common, d["aps"], M, varn, itera, d["h0"], d["h"])
            else:
                th = quiet(ns["em"], *common, d["aps"], M, varn, itera, d["h0"])
            out[det] = np.asarray(th, dtype=complex).reshape(-1)
        except IndexError:           # nearest_symbol_ecul's flat index past the table (:48-51)
            out[det] = None
    return i, k, out


def case_kat2_driver(monte_iter=3, seed=0):
    """PMd/SNR/all_Detectors.py's whole driver (:362-395) for `monte_iter` trials after
    np.random.seed(seed), with the script's own helpers, constants (:331-354) and all FIVE EMs
    of the NMSE-vs-SNR figure (em_pm r=1, em_ml, em_zf, em_mmse, em): per-trial thetas and
    NMSE (the script's trace expression, :382-387) and the averaged curves (:390-395).  Data
    are generated sequentially in the driver's draw order; the EM runs (mpmath, ~1 min each)
    are spread over worker processes."""
    N, n_tx, n_rx, T_d, T_p, M, itera, partition_r = 10, 2, 2, 50, 12, 4, 5, 1
    SNR = [-5, 0, 5, 10, 15, 20]
    varns = np.array([10 / np.power(10, s / 10) for s in SNR])
    ns = load_defs(os.path.join(PMD, "SNR", "all_Detectors.py"), N=N, n_tx=n_tx,
                   beta_min=0.0, beta_max=2 * np.pi)
    np.random.seed(seed)
    jobs, data = [], {}
    for i in range(monte_iter):
        h = quiet(ns["channelMatrix"], n_tx, n_rx, N, 1)
        X_d, aps, cons = ns["symbols"](n_tx, M, T_d)
        X_p = ns["pilotSymbols"](n_tx, M, T_p)
        Ptp, Ptd = ns["irsMatrix"](T_p, T_d, N, 0, 1)
        Ptd = np.insert(Ptd, 0, np.ones((1, T_d), dtype="complex128"), axis=0)
        data[f"h{i}"], data[f"X_d{i}"] = h, np.stack(X_d)[..., 0]
        data[f"X_p{i}"], data[f"Ptd{i}"] = np.stack(X_p)[..., 0], Ptd
        Z_p = None
        for k in range(len(SNR)):
            Y_p, Y_d, Z_p, Z_d, h0 = ns["receivedSignals"](T_p, T_d, Ptp, Ptd, n_rx, n_tx, X_d,
                                                            X_p, h, varns[k], M)
            data[f"Y_p{i}_{k}"], data[f"Y_d{i}_{k}"] = np.stack(Y_p)[..., 0], np.stack(Y_d)[..., 0]
            data[f"h0{i}_{k}"] = np.asarray(h0).reshape(-1)
            data[f"Z_p{i}"] = np.stack(Z_p)
            d = dict(Y_d=Y_d, Y_p=Y_p, Z_p=Z_p, Ptd=Ptd, h0=h0, h=h, X_d=X_d, aps=aps, cons=cons)
            jobs.append((i, k, d, varns[k], N, n_tx, M, T_d, T_p, itera, partition_r))
    import multiprocessing as mp_
    if mp_.current_process().daemon:
        results = [_kat2_driver_job(j) for j in jobs]
    else:
        with Pool(7) as pool:
            results = pool.map(_kat2_driver_job, jobs)
    nm = np.full((len(_SNR_DETS), monte_iter, len(SNR)), np.nan)
    for i, k, out in results:
        for di, det in enumerate(_SNR_DETS):
            if out[det] is None:
                continue
            data[f"{det}_theta{i}_{k}"] = out[det]
            e = out[det][:, None] - data[f"h{i}"][:, None]
            nm[di, i, k] = (np.trace(np.abs(e.conj().T @ e)) /
                            np.linalg.norm(data[f"h{i}"][:, None]) ** 2)
    data.update(nmse=nm, curve=np.average(nm, axis=1), dets=np.array(_SNR_DETS), snr=np.array(SNR),
                varn=varns, aps=aps, cons=cons, Ptp=Ptp, N=N, n_tx=n_tx,
                n_rx=n_rx, T_d=T_d, T_p=T_p, M=M, itera=itera, partition_r=partition_r,
                monte_iter=monte_iter, seed=seed)
    return "kat2_driver", data


def case_shape(name, N, n_tx, n_rx, T_d, T_p, M, varn, itera, seed):
    """Extra shapes through the north-star em (odd stream splits, 16/64-QAM)."""
    ns = load_defs(os.path.join(PMD, "Proposed_method_NMSEvsTp.py"),
                   N=N, n_tx=n_tx, n_rx=n_rx, beta_min=0.0, beta_max=2 * np.pi)
    d = _gen_northstar(ns, seed, N, n_tx, n_rx, T_d, T_p, M, varn)
    th = quiet(ns["em"], d["Y_d"], d["Y_p"], T_d, T_p, d["Z_p"], d["Ptd"], d["aps"], M,
               varn, itera, d["h0"])
    return name, _pack(d, N=N, n_tx=n_tx, n_rx=n_rx, T_d=T_d, T_p=T_p, M=M, varn=varn,
                       itera=itera, seed=seed, theta=np.asarray(th).reshape(-1),
                       nmse=nmse(th, d["h"]))


def case_root():
    """Root-level Proposed_method_NMSEvsTp.py: zero init, float path (:43-69),
    C-order h (:16), N x T_p DFT over T_p plus a ones row (:73-77, :129)."""
    N, n_tx, n_rx, T_d, T_p, M, varn, itera = 4, 2, 2, 10, 6, 4, 0.1, 3
    ns = load_defs(os.path.join(REF, "Proposed_method_NMSEvsTp.py"), N=N, n_tx=n_tx,
                   beta_min=0.0, beta_max=2 * np.pi)
    np.random.seed(3)
    h = quiet(ns["channelMatrix"], n_tx, n_rx, N, 1)
    X_d, aps = ns["symbols"](n_tx, M, T_d)
    Ptp, Ptd = ns["irsMatrix"](T_p, T_d, N, 0, 1)
    Ptp = np.insert(Ptp, 0, np.ones((1, T_p), dtype="complex128"), axis=0)
    Ptd = np.insert(Ptd, 0, np.ones((1, T_d), dtype="complex128"), axis=0)
    X_p = ns["pilotSymbols"](n_tx, M, T_p)
    Y_p, Y_d, Z_p, Z_d = ns["receivedSignals"](T_p, T_d, Ptp, Ptd, n_rx, n_tx, X_d, X_p,
                                               h, varn, M)
    th = quiet(ns["em"], Y_d, Y_p, T_d, T_p, Z_p, Ptd, aps, M, varn, itera)
    d = dict(h=h, X_d=X_d, aps=aps, X_p=X_p, Ptp=Ptp, Ptd=Ptd, Y_p=Y_p, Y_d=Y_d, Z_p=Z_p,
             h0=np.zeros(len(h), dtype=complex))
    return "root_tp", _pack(d, N=N, n_tx=n_tx, n_rx=n_rx, T_d=T_d, T_p=T_p, M=M,
                            varn=varn, itera=itera, seed=3,
                            theta=np.asarray(th).reshape(-1), nmse=nmse(th, h))


def case_root_td():
    """Root-level Proposed_method_NMSEvsTd.py: zero init (:44-47), C-order h (:25), N x T_p DFT
    over T_p plus a ones row (:81-86, :95) and DETERMINISTIC (N+1) x T_d DFT data phases over T_d
    (:92-94); per trial channelMatrix, pilotSymbols, then per T_d point symbols, irsMatrix,
    receivedSignals (:137-143).  Two T_d points of one trial."""
    N, n_tx, n_rx, T_p, M, varn, itera = 4, 1, 3, 6, 4, 0.1, 3
    T_ds = (8, 12)
    ns = load_defs(os.path.join(REF, "Proposed_method_NMSEvsTd.py"), N=N, n_tx=n_tx,
                   beta_min=0.0, beta_max=2 * np.pi)
    np.random.seed(5)
    h = quiet(ns["channelMatrix"], n_tx, n_rx, N, 1)
    X_p = ns["pilotSymbols"](n_tx, M, T_p)
    out = dict(h=h, X_p=X_p, h0=np.zeros(len(h), dtype=complex))
    for k, T_d in enumerate(T_ds):
        X_d, aps = ns["symbols"](n_tx, M, T_d)
        Ptp, Ptd = ns["irsMatrix"](T_p, T_d, N, 0, 1)
        Y_p, Y_d, Z_p, Z_d = ns["receivedSignals"](T_p, T_d, Ptp, Ptd, n_rx, n_tx, X_d, X_p,
                                                   h, varn, M)
        th = quiet(ns["em"], Y_d, Y_p, T_d, T_p, Z_p, Ptd, aps, M, varn, itera)
        out.update({f"X_d{k}": np.stack([x.reshape(-1) for x in X_d]), f"Ptd{k}": Ptd,
                    f"Y_d{k}": np.stack([y.reshape(-1) for y in Y_d]),
                    f"Y_p{k}": np.stack([y.reshape(-1) for y in Y_p]),
                    f"Z_p{k}": np.stack(Z_p), f"theta{k}": np.asarray(th).reshape(-1),
                    f"nmse{k}": nmse(th, h)})
        out["Ptp"], out["aps"] = Ptp, aps
    out["X_p"] = np.stack([x.reshape(-1) for x in X_p])
    return "root_td", dict(out, N=N, n_tx=n_tx, n_rx=n_rx, T_p=T_p, T_ds=np.array(T_ds), M=M,
                           varn=varn, itera=itera, seed=5)


def case_pm(name, N, n_tx, n_rx, T_d, T_p, M, varn, itera, seed, r_uniform, r_soft):
    """PM.em_pm (uniform list, lstsq) and PM_beta.em_pm (posterior list) on north-star data."""
    ns = load_defs(os.path.join(PMD, "Proposed_method_NMSEvsTp.py"),
                   N=N, n_tx=n_tx, n_rx=n_rx, beta_min=0.0, beta_max=2 * np.pi)
    d = _gen_northstar(ns, seed, N, n_tx, n_rx, T_d, T_p, M, varn)
    cons = _cons(M)
    ns_pm = load_defs(os.path.join(PMD, "PM.py"), N=N, beta_min=0.0, beta_max=2 * np.pi)
    th_u = quiet(ns_pm["em_pm"], d["Y_d"], d["Y_p"], T_d, T_p, d["Z_p"], d["Ptd"], d["aps"], M,
                 varn, itera, d["h0"], d["h"], n_tx, r_uniform, d["X_d"], cons)
    ns_pmb = load_defs(os.path.join(PMD, "PM_beta.py"), N=N, qamCons=cons, beta_min=0.0,
                       beta_max=2 * np.pi)
    th_s = quiet(ns_pmb["em_pm"], d["Y_d"], d["Y_p"], T_d, T_p, d["Z_p"], d["Ptd"], M, varn,
                 itera, d["h0"], d["h"], n_tx, r_soft, d["X_d"], cons)
    return name, _pack(d, N=N, n_tx=n_tx, n_rx=n_rx, T_d=T_d, T_p=T_p, M=M, varn=varn,
                       itera=itera, seed=seed, r_uniform=r_uniform, r_soft=r_soft,
                       pm_theta=np.asarray(th_u).reshape(-1),
                       pmbeta_theta=np.asarray(th_s).reshape(-1))


def case_det(name, N, n_tx, n_rx, T_d, T_p, M, varn, itera, seed):
    """all_detectorsvsTd.em_zf / em_mmse (off-by-one list channel, flattened-argmin
    nearest_symbol_ecul, oracle early stop) on north-star data."""
    ns = load_defs(os.path.join(PMD, "Proposed_method_NMSEvsTp.py"),
                   N=N, n_tx=n_tx, n_rx=n_rx, beta_min=0.0, beta_max=2 * np.pi)
    d = _gen_northstar(ns, seed, N, n_tx, n_rx, T_d, T_p, M, varn)
    cons = _cons(M)
    ns_all = load_defs(os.path.join(PMD, "all_detectorsvsTd.py"), N=N, n_tx=n_tx, qamCons=cons,
                       h=d["h"], Z_d=d["Z_d"], beta_min=0.0, beta_max=2 * np.pi)
    th_z = quiet(ns_all["em_zf"], d["Y_d"], d["Y_p"], T_d, T_p, d["Z_p"], d["Ptd"], d["aps"], M,
                 varn, itera, d["h0"], d["h"])
    th_m = quiet(ns_all["em_mmse"], d["Y_d"], d["Y_p"], T_d, T_p, d["Z_p"], d["Ptd"], d["aps"],
                 M, varn, itera, d["h0"], d["h"])
    return name, _pack(d, N=N, n_tx=n_tx, n_rx=n_rx, T_d=T_d, T_p=T_p, M=M, varn=varn,
                       itera=itera, seed=seed, zf_theta=np.asarray(th_z).reshape(-1),
                       mmse_theta=np.asarray(th_m).reshape(-1))


def case_ser():
    """PMd/SER/log_max_SER.py: log-max em (:51-84) returning the last iteration's argmax
    decisions X_dest, and the script's SER expression (:162), on the script's own data
    helpers and draw order (:150-160), one trial, two SNR points."""
    N, n_tx, n_rx, T_d, T_p, M, itera, SNR = 6, 2, 2, 30, 20, 4, 3, (0, 10)
    ns = load_defs(os.path.join(PMD, "SER", "log_max_SER.py"), N=N, n_tx=n_tx, n_rx=n_rx,
                   beta_min=0.0, beta_max=2 * np.pi, varh=1.0, amp=1)
    np.random.seed(5)
    h = quiet(ns["channelMatrix"], n_tx, n_rx, N, 1.0)
    X_d, aps = ns["symbols"](n_tx, M, T_d)
    Ptp, Ptd = ns["irsMatrix"](T_p, T_d, N, 0.0, 1)
    Ptd = np.insert(Ptd, 0, np.ones((1, T_d), dtype="complex128"), axis=0)
    X_p = ns["pilotSymbols"](n_tx, M, T_p)
    out = dict(N=N, n_tx=n_tx, n_rx=n_rx, T_d=T_d, T_p=T_p, M=M, itera=itera,
               snr=np.asarray(SNR), h=h, X_d=np.stack(X_d)[..., 0], aps=aps, Ptp=Ptp, Ptd=Ptd,
               X_p=np.stack(X_p)[..., 0])
    for k, snr in enumerate(SNR):
        varn = 10 / np.power(10, snr / 10)
        Y_p, Y_d, Z_p, Z_d, h0 = ns["receivedSignals"](T_p, T_d, Ptp, Ptd, n_rx, n_tx, X_d, X_p,
                                                       h, varn, M)
        ns["Z_d"] = Z_d                      # em's LLF line (:83) reads the global Z_d
        th, X_dest = quiet(ns["em"], Y_d, Y_p, T_d, T_p, Z_p, Ptd, aps, M, varn, itera, h0)
        ser = np.count_nonzero(np.array(X_d) - np.array(X_dest)) / (T_d * n_tx)
        out.update({f"varn{k}": varn, f"Y_p{k}": np.stack(Y_p)[..., 0],
                    f"Y_d{k}": np.stack(Y_d)[..., 0], f"Z_p{k}": np.stack(Z_p),
                    f"h0{k}": np.asarray(h0).reshape(-1), f"theta{k}": np.asarray(th).reshape(-1),
                    f"X_dest{k}": np.stack(X_dest)[:, 0, :], f"ser{k}": ser})
    return "ser_logmax", out


def case_superimposed():
    """Parallel/ParallelProtocol_Tp.py: superimposed data + pilot (dataPilotSymbols :41-53),
    soft EM with hypotheses x_j + x_p,t and no separate pilot block (em :63-86), zero
    initialisation, driver draw order :114-122; T_p shorter and longer than T_d."""
    N, n_tx, n_rx, T_d, M, varn, itera, T_ps = 4, 1, 4, 20, 16, 0.1, 3, (8, 30)
    ns = load_defs(os.path.join(REF, "Parallel", "ParallelProtocol_Tp.py"))
    np.random.seed(17)
    h = quiet(ns["channelMatrix"], n_tx, n_rx, N, 1.0)
    X_d, aps = ns["symbols"](n_tx, M, T_d)
    out = dict(N=N, n_tx=n_tx, n_rx=n_rx, T_d=T_d, M=M, varn=varn, itera=itera,
               T_ps=np.asarray(T_ps), h=np.asarray(h).reshape(-1), aps=aps,
               X_d=np.stack(X_d)[..., 0])
    for k, T_p in enumerate(T_ps):
        T = max(T_d, T_p)
        Psi = ns["irsMatrix"](T, N)
        X_p = ns["pilotSymbols"](n_tx, M, T_p)
        X = ns["dataPilotSymbols"](n_tx, X_p, X_d)
        Y, Z = ns["receivedSignals"](T, Psi, n_rx, n_tx, X, h, varn)
        th = quiet(ns["em"], Y, T, Z, X_d, X_p, T_p, T_d, n_tx, Psi, aps, M, varn, itera, N)
        out.update({f"Psi{k}": Psi, f"X_p{k}": np.stack(X_p)[..., 0], f"X{k}": X,
                    f"Y{k}": np.stack(Y)[..., 0], f"theta{k}": np.asarray(th).reshape(-1)})
    return "superimposed", out


def case_gaussian():
    """Proposed method/MIMO_Gaussian_proposed.py: Gaussian-prior EM (EM_Gaussian_proposed
    :56-89, run itera + 1 times) on the script's own generators (channelMatrix1, symbols,
    pilotSymbols, irsMatrix, received_proposed; driver order :160-170), n_rx = 1, 2, 3, and
    the script's own size (N = 32) for ONE iteration: past it the reference iteration
    diverges (NMSE ~1e6 after one step at these defaults) and is not reproducible."""
    out = {}
    for k, (N, n_tx, n_rx, T_d, T_p, varn, varx, itera, seed) in enumerate(
            [(4, 2, 2, 12, 8, 0.1, 1.0, 3, 31), (4, 2, 1, 12, 8, 0.1, 1.0, 3, 32),
             (3, 1, 3, 10, 6, 0.2, 1.0, 2, 33), (4, 2, 2, 12, 8, 0.1, 0.7, 2, 34),
             (32, 2, 2, 50, 8, 0.1, 1.0, 0, 35)]):
        ns = load_defs(os.path.join(PMD, "MIMO_Gaussian_proposed.py"),
                       beta_max=2 * np.pi)
        np.random.seed(seed)
        H = ns["channelMatrix1"](1.0, N, n_rx, n_tx)
        X_d = ns["symbols"](n_tx, T_d, varx)
        Ptp, Ptd = ns["irsMatrix"](T_p, T_d, N, 0.0, 1.0)
        X_p = ns["pilotSymbols"](n_tx, T_p, varx)
        y_p, y_d, z_p, z_d, H0 = ns["received_proposed"](T_p, T_d, Ptp, Ptd, n_rx, n_tx, X_d,
                                                         X_p, H, varn)
        Hh = quiet(ns["EM_Gaussian_proposed"], y_d, y_p, T_d, T_p, z_p, Ptd, varn, itera, H0,
                   varx, n_tx)
        out.update({f"dims{k}": np.array([N, n_tx, n_rx, T_d, T_p, itera]),
                    f"varn{k}": varn, f"varx{k}": varx, f"H{k}": H, f"X_d{k}": X_d,
                    f"X_p{k}": X_p, f"Ptp{k}": Ptp, f"Ptd{k}": Ptd,
                    f"Y_p{k}": np.stack(y_p)[..., 0], f"Y_d{k}": np.stack(y_d)[..., 0],
                    f"Z_p{k}": np.stack(z_p)[..., 0], f"H0{k}": H0, f"H_hat{k}": Hh})
    return "gaussian", out


def case_alldet(name, N, n_tx, n_rx, T_d, T_p, M, varn, itera, partition_r, seed):
    """PMd/all_detectorsvsTd.py at ONE T_d point of its sweep, with the script's own helpers in
    its driver's draw order (:371-382: channelMatrix, pilotSymbols, then per T_d symbols,
    irsMatrix, ones row, receivedSignals) and its five EMs (:384-388): em_pm (soft list,
    :176-249), em_ml (:135-173), em_zf (:95-133), em_mmse (:54-93), em (:260-295).  Every EM
    reads the global h for the oracle early stop."""
    ns = load_defs(os.path.join(PMD, "all_detectorsvsTd.py"), N=N, n_tx=n_tx,
                   beta_min=0.0, beta_max=2 * np.pi)
    np.random.seed(seed)
    h = quiet(ns["channelMatrix"], n_tx, n_rx, N, 1)
    X_p = ns["pilotSymbols"](n_tx, M, T_p)
    X_d, aps, cons = ns["symbols"](n_tx, M, T_d)
    Ptp, Ptd = ns["irsMatrix"](T_p, T_d, N, 0.0, 1)
    Ptd = np.insert(Ptd, 0, np.ones((1, T_d), dtype="complex128"), axis=0)
    Y_p, Y_d, Z_p, Z_d, h0 = ns["receivedSignals"](T_p, T_d, Ptp, Ptd, n_rx, n_tx, X_d, X_p, h,
                                                   varn, M)
    ns["h"] = h
    ns["qamCons"] = cons
    ns["Z_d"] = Z_d                      # em_mmse's LLF line (:91) reads the global Z_d
    common = (Y_d, Y_p, T_d, T_p, Z_p, Ptd)
    th = {
        "pm": quiet(ns["em_pm"], *common, M, varn, itera, h0, h, n_tx, partition_r, X_d, cons),
        "ml": quiet(ns["em_ml"], *common, aps, M, varn, itera, h0),
        "zf": quiet(ns["em_zf"], *common, aps, M, varn, itera, h0, h),
        "mmse": quiet(ns["em_mmse"], *common, aps, M, varn, itera, h0, h),
        "em": quiet(ns["em"], *common, aps, M, varn, itera, h0),
    }
    d = dict(h=h, X_d=X_d, aps=aps, X_p=X_p, Ptp=Ptp, Ptd=Ptd, Y_p=Y_p, Y_d=Y_d, Z_p=Z_p, h0=h0)
    extra = {f"{k}_theta": np.asarray(v).reshape(-1) for k, v in th.items()}
    extra.update({f"{k}_nmse": nmse(v, h) for k, v in th.items()})
    return name, _pack(d, N=N, n_tx=n_tx, n_rx=n_rx, T_d=T_d, T_p=T_p, M=M, varn=varn,
                       itera=itera, partition_r=partition_r, seed=seed, cons=cons, **extra)


def case_cfg1_kernel():
    """The BASELINE cfg-1 kernel instantiation (n_tx = n_rx = 4, 16-QAM: J = 65,536 hypotheses
    per symbol) through the north-star em (PMd/Proposed_method_NMSEvsTp.py:50-83, gmpy2 ->
    mpmath) at a size the mp-object reference finishes in minutes: N = 1, T_p = 8, T_d = 2,
    two iterations, a low SNR (varn = 3) so that the posterior weights are genuinely soft."""
    N, n_tx, n_rx, T_d, T_p, M, varn, itera, seed = 1, 4, 4, 2, 8, 16, 3.0, 2, 41
    ns = load_defs(os.path.join(PMD, "Proposed_method_NMSEvsTp.py"),
                   N=N, n_tx=n_tx, n_rx=n_rx, beta_min=0.0, beta_max=2 * np.pi)
    d = _gen_northstar(ns, seed, N, n_tx, n_rx, T_d, T_p, M, varn)
    res = {}
    for it in (1, itera):
        th = quiet(ns["em"], d["Y_d"], d["Y_p"], T_d, T_p, d["Z_p"], d["Ptd"], d["aps"],
                   M, varn, it, d["h0"])
        res[f"theta_it{it}"] = np.asarray(th).reshape(-1)
    return "cfg1_kernel", _pack(d, N=N, n_tx=n_tx, n_rx=n_rx, T_d=T_d, T_p=T_p, M=M, varn=varn,
                                itera=itera, seed=seed, **res)


def case_llf_driver():
    """PMd/IterationsvsLLF.py's own driver (:139-154) with its own helpers and draw order
    (channelMatrix, symbols, irsMatrix + ones rows, pilotSymbols, receivedSignals, em with
    the genie LLF :76) at reduced sizes: the per-trial LLF curves and the data."""
    N, n_tx, n_rx, T_d, T_p, M, varn, itera, monte_iter, seed = 8, 2, 2, 20, 4, 4, 0.1, 3, 2, 23
    ns = load_defs(os.path.join(PMD, "IterationsvsLLF.py"), N=N, n_tx=n_tx, n_rx=n_rx,
                   beta_min=0.0, beta_max=2 * np.pi)
    np.random.seed(seed)
    out = dict(N=N, n_tx=n_tx, n_rx=n_rx, T_d=T_d, T_p=T_p, M=M, varn=varn, itera=itera,
               monte_iter=monte_iter, seed=seed)
    for i in range(monte_iter):
        h = quiet(ns["channelMatrix"], n_tx, n_rx, N, 1)
        X_d, aps = ns["symbols"](n_tx, M, T_d)[:2]
        Ptp, Ptd = ns["irsMatrix"](T_p, T_d, N, 0.0, 1)
        Ptp = np.insert(Ptp, 0, np.ones((1, T_p), dtype="complex128"), axis=0)
        Ptd = np.insert(Ptd, 0, np.ones((1, T_d), dtype="complex128"), axis=0)
        X_p = ns["pilotSymbols"](n_tx, M, T_p)
        Y_p, Y_d, Z_p, Z_d, h0 = ns["receivedSignals"](T_p, T_d, Ptp, Ptd, n_rx, n_tx, X_d, X_p,
                                                       h, varn, M, N)
        th, llf = quiet(ns["em"], Y_d, Y_p, T_d, T_p, Z_p, Z_d, Ptd, aps, M, varn, itera, h0,
                        n_tx)
        out.update({f"h{i}": h, f"Y_d{i}": np.stack(Y_d)[..., 0], f"Y_p{i}": np.stack(Y_p)[..., 0],
                    f"theta{i}": np.asarray(th).reshape(-1),
                    f"llf{i}": np.asarray(llf, dtype=float).reshape(-1)})
    return "llf_driver", out


def case_qam():
    """Constellation tables of the vendored komm QAM (PMd/QAM.py:320-322)."""
    return "qam", {f"cons{M}": _cons(M) for M in (4, 16, 64, 256)}


CASES = {
    "qam": (case_qam, ()),
    # all_detectorsvsTd.py's own constants (:345-363) at its first T_d point
    "alldet_td15": (case_alldet, ("alldet_td15", 15, 2, 2, 15, 20, 4, 0.1, 5, 1, 3)),
    "cfg1_kernel": (case_cfg1_kernel, ()),
    "llf_driver": (case_llf_driver, ()),
    "pm_nt4": (case_pm, ("pm_nt4", 3, 4, 4, 24, 8, 4, 0.1, 3, 12, 0, 2)),
    "pm_nt3_m16": (case_pm, ("pm_nt3_m16", 4, 3, 3, 24, 10, 16, 0.3, 3, 13, 1, 1)),
    "ser_logmax": (case_ser, ()),
    "superimposed": (case_superimposed, ()),
    "gaussian": (case_gaussian, ()),
    "det_nt3": (case_det, ("det_nt3", 4, 3, 4, 30, 10, 4, 0.2, 3, 21)),
    "det_nt2_m16": (case_det, ("det_nt2_m16", 5, 2, 3, 30, 12, 16, 0.3, 3, 22)),
    "kat1_s7": (case_kat1, (7,)),
    "kat1_s11": (case_kat1, (11,)),
    "kat2_snr": (case_kat2, ()),
    "kat2_driver": (case_kat2_driver, ()),
    "root_tp": (case_root, ()),
    "root_td": (case_root_td, ()),
    "nt4_m4": (case_shape, ("nt4_m4", 3, 4, 4, 16, 8, 4, 0.1, 2, 5)),
    "nt3_m4": (case_shape, ("nt3_m4", 3, 3, 2, 10, 8, 4, 0.2, 2, 9)),
    "nt1_m16": (case_shape, ("nt1_m16", 5, 1, 3, 20, 6, 16, 0.3, 3, 4)),
    "nt2_m16": (case_shape, ("nt2_m16", 4, 2, 2, 12, 8, 16, 0.5, 2, 6)),
    "nt2_m64": (case_shape, ("nt2_m64", 3, 2, 2, 6, 10, 64, 1.0, 2, 8)),
}


def run(name):
    fn, args = CASES[name]
    t0 = time.time()
    key, arrays = fn(*args)
    np.savez_compressed(os.path.join(OUT, key + ".npz"), **arrays)
    return key, time.time() - t0


if __name__ == "__main__":
    names = sys.argv[1:] or list(CASES)
    if len(names) == 1:                  # in-process: a case may use its own worker pool
        print("%s: %.1fs" % run(names[0]), flush=True)
        sys.exit(0)
    with Pool(min(len(names), 7)) as pool:
        for key, dt in pool.imap_unordered(run, names):
            print(f"{key}: {dt:.1f}s", flush=True)
