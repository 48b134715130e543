#!/usr/bin/env python3
"""Min-norm trials flagged SBCE_STATUS_RANK at full BASELINE cfg 2 size vs numpy.linalg.lstsq
(the reference's solve, "Proposed method/PM.py":108) on the device's own normal equations.

Runs the cfg-2 workload (8x8, N_RIS = 256, T_p = 32, T_d = 1024, 16-QAM, PM_beta r = 1 E-step,
20 dB) for `--iters` EM iterations, then one more E-step + min-norm M-step through the staged
entry points (sbce_estep, sbce_mstep) so that R and B^H of that M-step come back to the host.
For every flagged trial (and a few clean ones) reports theta's relative error against lstsq,
the NMSE of both, and R's eigenvalues around lstsq's cut eps K lambda_max.
Usage: python tools/rank_study.py --trials 64 --iters 1 --out gpurun_out/rank.json
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--trials", type=int, default=64)
    ap.add_argument("--iters", type=int, nargs="+", default=[1])
    ap.add_argument("--seed", type=int, default=0)
    ap.add_argument("--clean", type=int, default=2, help="unflagged trials compared too")
    ap.add_argument("--max-flagged", type=int, default=8)
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    import __graft_entry__ as ge
    from oracle.em_reduced import mstep_lstsq, nmse
    pkg = ge.package()
    pkg._lib.use_ab()       # the A/B build: SBCE_* switches, counters, clocks
    n_tx, n_rx, N, T_p, T_d, M = 8, 8, 256, 32, 1024, 16
    varn = float(pkg.signal_model.snr_to_varn(20.0))
    b = pkg.signal_model.synthetic_batch(a.trials, n_tx, n_rx, N, T_p, T_d, M, varn, seed=a.seed)
    out = {"trials": a.trials, "runs": []}
    for iters in a.iters:
        out["runs"].append(study(pkg, b, varn, iters, a, mstep_lstsq, nmse, n_tx, n_rx))
    if a.out:
        with open(a.out, "w") as f:
            json.dump(out, f, indent=1)


def study(pkg, b, varn, iters, a, mstep_lstsq, nmse, n_tx, n_rx):
    th = b["theta0"]
    if iters:
        r = pkg.em_batch(b["y_d"], b["y_p"], b["psi_d"], b["u_p"], b["cons"], varn, iters, th,
                         mode="pm_soft", partition_r=1, solve="lstsq")
        th = r["theta"]
    m, S = pkg.estep_batch(b["y_d"], b["psi_d"], b["cons"], th, varn, n_tx, "pm_soft",
                           partition_r=1)
    thd, R, rhs, st = pkg.mstep_batch(b["y_d"], b["y_p"], b["psi_d"], b["u_p"], b["cons"], m, S,
                                      varn, solve="lstsq")
    RANK = pkg._lib.SBCE_STATUS_RANK
    flagged = [i for i in range(a.trials) if st[i] & RANK]
    clean = [i for i in range(a.trials) if not st[i] & RANK][:a.clean]
    L = R.shape[1]
    K = L * n_rx
    eps = np.finfo(float).eps
    out = {"iters_before": iters, "flagged": len(flagged), "flagged_trials": flagged, "cases": []}
    print(f"after {iters} iterations: {len(flagged)} of {a.trials} trials flagged RANK", flush=True)
    for i in flagged[:a.max_flagged] + clean:
        t0 = time.time()
        th_ls, rank = mstep_lstsq(R[i], rhs[i])
        ev = np.linalg.eigvalsh(R[i])
        cut = eps * K * ev[-1]
        k = np.searchsorted(ev, cut)
        near = (ev[max(k - 3, 0):k + 3] / cut).tolist()
        e = float(np.abs(thd[i] - th_ls).max() / np.abs(th_ls).max())
        n_dev, n_ls = nmse(thd[i], b["h"][i]), nmse(th_ls, b["h"][i])
        x = np.conj(thd[i]).reshape(L, n_rx)
        x0 = np.conj(th_ls).reshape(L, n_rx)
        res, res0 = np.linalg.norm(R[i] @ x - rhs[i]), np.linalg.norm(R[i] @ x0 - rhs[i])
        c = {"trial": i, "flagged": bool(st[i] & RANK), "status": int(st[i]), "rank_lstsq": rank,
             "theta_rel_err": e, "nmse_dev": n_dev, "nmse_lstsq": n_ls,
             "nmse_rel_dev": abs(n_dev / n_ls - 1), "norm_dev": float(np.linalg.norm(thd[i])),
             "norm_lstsq": float(np.linalg.norm(th_ls)), "residual_dev": float(res),
             "residual_lstsq": float(res0), "eig_over_cut_near_cut": near,
             "kept_cond": float(ev[-1] / ev[ev > cut].min()), "secs": time.time() - t0}
        out["cases"].append(c)
        print(json.dumps(c), flush=True)
    return out


if __name__ == "__main__":
    main()
