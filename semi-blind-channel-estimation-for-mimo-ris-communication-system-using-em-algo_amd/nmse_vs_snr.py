#!/usr/bin/env python3
"""NMSE vs SNR — entry point of "Proposed method/SNR/all_Detectors.py" (constants :331-354,
driver :362-395): its five EMs (PM r=1, log-max, ZF, MMSE, exact) on the MI355X."""
import argparse

from _cli import init_distributed, package, report  # noqa: E402


def main():
    ap = argparse.ArgumentParser(description=__doc__)
    ap.add_argument("--SNR", type=float, nargs="+", default=[-5, 0, 5, 10, 15, 20])
    ap.add_argument("--T-d", type=int, default=50)
    ap.add_argument("--T-p", type=int, default=12)
    ap.add_argument("--N", type=int, default=10)
    ap.add_argument("--n-rx", type=int, default=2)
    ap.add_argument("--n-tx", type=int, default=2)
    ap.add_argument("--itera", type=int, default=5)
    ap.add_argument("--monte-iter", type=int, default=15)
    ap.add_argument("--M", type=int, default=4)
    ap.add_argument("--power", type=float, default=10.0)
    ap.add_argument("--seed", type=int, default=0)
    ap.add_argument("--partition-r", type=int, default=1)
    ap.add_argument("--detectors", nargs="+", default=None,
                    help="subset of pm_soft hard zf mmse soft (default: all five)")
    ap.add_argument("--no-replay", action="store_true")
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    init_distributed()
    pkg = package()
    x, curves = pkg.sweeps.nmse_vs_snr(tuple(a.SNR), a.T_d, a.T_p, a.N, a.n_rx, a.n_tx, a.itera,
                                       a.monte_iter, a.M, a.power, a.seed, replay=not a.no_replay,
                                       modes=tuple(a.detectors or pkg.sweeps.SNR_DETECTORS),
                                       partition_r=a.partition_r)
    labels = {k: v[2] for k, v in pkg.sweeps.SNR_DETECTORS.items()}
    report("SNR", x, {labels[k]: v for k, v in curves.items()}, a.out,
           "Proposed method with detectors")


if __name__ == "__main__":
    main()
