#!/usr/bin/env python3
"""NMSE vs data length T_d — entry point of "Proposed method/Proposed_method_NMSEvsTd.py"
(constants :121-136, C-order channel vec :15) with the EM (:44-76) on the MI355X.
--variant root: the root-level Proposed_method_NMSEvsTd.py instead (deterministic DFT data
phases :92-94, zero-initialised EM :46, its constants :121-136: n_rx = 8, n_tx = 1, itera = 20)."""
import argparse

from _cli import init_distributed, package, report  # noqa: E402


def main():
    ap = argparse.ArgumentParser(description=__doc__)
    ap.add_argument("--T-p", type=int, default=16)
    ap.add_argument("--T-d", type=int, nargs="+", default=[20, 30, 40, 50, 60, 70, 80, 90, 100])
    ap.add_argument("--N", type=int, default=32)
    ap.add_argument("--n-rx", type=int, default=None)
    ap.add_argument("--n-tx", type=int, default=None)
    ap.add_argument("--itera", type=int, default=None)
    ap.add_argument("--variant", choices=("pmd", "root"), default="pmd")
    ap.add_argument("--monte-iter", type=int, default=1)
    ap.add_argument("--M", type=int, default=4)
    ap.add_argument("--varn", type=float, default=0.1)
    ap.add_argument("--seed", type=int, default=0)
    ap.add_argument("--no-replay", action="store_true")
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    dflt = dict(n_rx=8, n_tx=1, itera=20) if a.variant == "root" else dict(n_rx=2, n_tx=2, itera=3)
    for k, v in dflt.items():
        if getattr(a, k) is None:
            setattr(a, k, v)
    init_distributed()
    pkg = package()
    x, nm = pkg.sweeps.nmse_vs_td(tuple(a.T_d), a.T_p, a.N, a.n_rx, a.n_tx, a.itera, a.monte_iter,
                                  a.M, a.varn, a.seed, replay=not a.no_replay,
                                  variant=a.variant)
    report("T_d", x, {"Proposed method - Exact": nm}, a.out, "Proposed method - Exact")


if __name__ == "__main__":
    main()
