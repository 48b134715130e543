#!/usr/bin/env python3
"""NMSE vs SNR — entry point of "Proposed method/SNR/all_Detectors.py" (constants :331-354,
driver :362-395): exact EM ('Exact') and log-max EM, on the MI355X."""
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
    ap.add_argument("--no-replay", action="store_true")
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    init_distributed()
    pkg = package()
    x, curves = pkg.sweeps.nmse_vs_snr(tuple(a.SNR), a.T_d, a.T_p, a.N, a.n_rx, a.n_tx, a.itera,
                                       a.monte_iter, a.M, a.power, a.seed, replay=not a.no_replay)
    report("SNR", x, {"Exact": curves["soft"], "log-max": curves["hard"]}, a.out,
           "Proposed method with detectors")


if __name__ == "__main__":
    main()
