#!/usr/bin/env python3
"""NMSE vs T_p of the Gaussian-prior EM — entry point of
"Proposed method/MIMO_Gaussian_proposed.py" (constants :140-155, driver :158-186), on the
MI355X."""
import argparse

from _cli import init_distributed, package, report  # noqa: E402


def main():
    ap = argparse.ArgumentParser(description=__doc__)
    ap.add_argument("--T-p", type=int, nargs="+", default=[8, 12, 16, 20, 24, 28, 32, 36, 40])
    ap.add_argument("--T-d", type=int, default=50)
    ap.add_argument("--N", type=int, default=32)
    ap.add_argument("--n-rx", type=int, default=2)
    ap.add_argument("--n-tx", type=int, default=2)
    ap.add_argument("--itera", type=int, default=3)
    ap.add_argument("--monte-iter", type=int, default=1)
    ap.add_argument("--varn", type=float, default=0.1)
    ap.add_argument("--varx", type=float, default=1.0)
    ap.add_argument("--seed", type=int, default=0)
    ap.add_argument("--no-replay", action="store_true")
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    init_distributed()
    pkg = package()
    x, nm = pkg.sweeps.nmse_vs_tp_gaussian(tuple(a.T_p), a.T_d, a.N, a.n_rx, a.n_tx, a.itera,
                                           a.monte_iter, a.varn, a.varx, a.seed,
                                           replay=not a.no_replay)
    report("T_p", x, {"Proposed method": nm}, a.out, "Proposed method and Gaussian method - Exact")


if __name__ == "__main__":
    main()
