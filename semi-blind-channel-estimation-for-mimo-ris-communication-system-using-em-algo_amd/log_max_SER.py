#!/usr/bin/env python3
"""SER vs SNR of the log-max EM — entry point of "Proposed method/SER/log_max_SER.py"
(constants :124-147, driver :150-167), on the MI355X.  Prints both the script's own SER
expression (:162) and the element-wise symbol error rate."""
import argparse

from _cli import init_distributed, package, report  # noqa: E402


def main():
    ap = argparse.ArgumentParser(description=__doc__)
    ap.add_argument("--SNR", type=float, nargs="+", default=[-5, 0, 5, 10, 15, 20])
    ap.add_argument("--T-d", type=int, default=50)
    ap.add_argument("--T-p", type=int, default=20)
    ap.add_argument("--N", type=int, default=30)
    ap.add_argument("--n-rx", type=int, default=2)
    ap.add_argument("--n-tx", type=int, default=2)
    ap.add_argument("--itera", type=int, default=5)
    ap.add_argument("--monte-iter", type=int, default=75)
    ap.add_argument("--M", type=int, default=4)
    ap.add_argument("--power", type=float, default=10.0)
    ap.add_argument("--seed", type=int, default=0)
    ap.add_argument("--no-replay", action="store_true")
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    init_distributed()
    pkg = package()
    x, ser_ref, ser_el, _ = pkg.sweeps.ser_vs_snr(tuple(a.SNR), a.T_d, a.T_p, a.N, a.n_rx, a.n_tx,
                                                  a.itera, a.monte_iter, a.M, a.power, a.seed,
                                                  replay=not a.no_replay)
    report("SNR", x, {"Log-Max (script SER)": ser_ref, "Log-Max (element SER)": ser_el}, a.out,
           "Proposed method - ML detector", ylabel="SER", logy=True)


if __name__ == "__main__":
    main()
