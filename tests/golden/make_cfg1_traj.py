#!/usr/bin/env python3
"""Golden trajectories at BASELINE cfg 1 (Nt = Nr = 4, N_RIS = 64, T_p = 16, T_d = 256,
16-QAM, SNR 20 dB, exact soft E-step): the float64 oracle (oracle/em_reduced.py, pinned to
the reference's own em() by tests/golden/make_golden.py's fixtures) run for 20 EM iterations
on the first trials of bench.py's synthetic batch (signal_model.synthetic_batch(1000, ...,
seed=0)).  Writes tests/golden/cfg1_traj.npz: per-iteration NMSE and the final theta.

    OMP_NUM_THREADS=2 python tests/golden/make_cfg1_traj.py [n_trials] [workers]
"""
import importlib
import os
import sys
from multiprocessing import Pool

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
PKG = "semi-blind-channel-estimation-for-mimo-ris-communication-system-using-em-algo_amd"
CFG = dict(n_tx=4, n_rx=4, N=64, T_p=16, T_d=256, M=16, snr=20.0, itera=20, B=1000, seed=0)


def batch():
    pkg = importlib.import_module(PKG)
    varn = float(pkg.signal_model.snr_to_varn(CFG["snr"]))
    b = pkg.signal_model.synthetic_batch(CFG["B"], CFG["n_tx"], CFG["n_rx"], CFG["N"], CFG["T_p"],
                                         CFG["T_d"], CFG["M"], varn, seed=CFG["seed"])
    return pkg, b, varn


def run(i):
    from oracle.em_reduced import em_reduced, nmse
    pkg, b, varn = batch()
    aps = pkg.qam.all_possible_symbols(b["cons"], CFG["n_tx"])
    th, trace = em_reduced(b["y_d"][i], b["y_p"][i], b["u_p"][i], b["psi_d"][i].T, aps, varn,
                           CFG["itera"], b["theta0"][i], return_trace=True)
    traj = [nmse(b["theta0"][i], b["h"][i])] + [nmse(t, b["h"][i]) for t in trace]
    print(f"trial {i}: NMSE {traj[0]:.4f} -> {traj[-1]:.4f}", flush=True)
    return np.array(traj), th


if __name__ == "__main__":
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 8
    workers = int(sys.argv[2]) if len(sys.argv) > 2 else 4
    with Pool(workers) as p:
        res = p.map(run, range(n))
    np.savez_compressed(os.path.join(ROOT, "tests", "golden", "cfg1_traj.npz"),
                        nmse=np.stack([r[0] for r in res]), theta=np.stack([r[1] for r in res]),
                        **{k: v for k, v in CFG.items()})
