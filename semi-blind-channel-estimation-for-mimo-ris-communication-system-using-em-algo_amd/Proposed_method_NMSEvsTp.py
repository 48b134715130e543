#!/usr/bin/env python3
"""NMSE vs pilot length T_p — entry point of "Proposed method/Proposed_method_NMSEvsTp.py"
(constants :133-149) with the EM (:50-83) on the MI355X.  Defaults = the reference's.

  python <pkg>/Proposed_method_NMSEvsTp.py --monte-iter 10
  torchrun --nproc-per-node 8 <pkg>/Proposed_method_NMSEvsTp.py --monte-iter 1000 --no-replay
"""
import argparse

from _cli import init_distributed, package, report  # noqa: E402


def main():
    ap = argparse.ArgumentParser(description=__doc__)
    ap.add_argument("--T-d", type=int, default=50)
    ap.add_argument("--T-p", type=int, nargs="+", default=[4, 12, 20, 28, 36, 40])
    ap.add_argument("--N", type=int, default=32)
    ap.add_argument("--n-rx", type=int, default=4)
    ap.add_argument("--n-tx", type=int, default=4)
    ap.add_argument("--itera", type=int, default=3)
    ap.add_argument("--monte-iter", type=int, default=1)
    ap.add_argument("--M", type=int, default=4)
    ap.add_argument("--varn", type=float, default=0.1)
    ap.add_argument("--seed", type=int, default=0)
    ap.add_argument("--no-replay", action="store_true", help="per-trial RNG instead of the "
                    "reference's sequential legacy-RandomState stream")
    ap.add_argument("--out", default=None, help=".npz (+ .png) output")
    a = ap.parse_args()
    init_distributed()
    pkg = package()
    x, nm = pkg.sweeps.nmse_vs_tp(tuple(a.T_p), a.T_d, a.N, a.n_rx, a.n_tx, a.itera, a.monte_iter,
                                  a.M, a.varn, a.seed, replay=not a.no_replay)
    report("T_p", x, {"Proposed method": nm}, a.out, "proposed method")


if __name__ == "__main__":
    main()
