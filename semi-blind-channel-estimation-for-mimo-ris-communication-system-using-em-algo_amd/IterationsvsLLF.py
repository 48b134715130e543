#!/usr/bin/env python3
"""Log-likelihood vs EM iteration -- entry point of "Proposed method/IterationsvsLLF.py"
(constants :119-135, driver :139-154): the exact EM with the script's genie LLF (:76),
averaged over Monte-Carlo trials, on the MI355X."""
import argparse

from _cli import init_distributed, package, report  # noqa: E402


def main():
    ap = argparse.ArgumentParser(description=__doc__)
    ap.add_argument("--T-d", type=int, default=50)
    ap.add_argument("--T-p", type=int, default=4)
    ap.add_argument("--N", type=int, default=32)
    ap.add_argument("--n-rx", type=int, default=2)
    ap.add_argument("--n-tx", type=int, default=2)
    ap.add_argument("--itera", type=int, default=5)
    ap.add_argument("--monte-iter", type=int, default=3)
    ap.add_argument("--M", type=int, default=4)
    ap.add_argument("--varn", type=float, default=0.1)
    ap.add_argument("--seed", type=int, default=0)
    ap.add_argument("--no-replay", action="store_true")
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    init_distributed()
    pkg = package()
    it, llf, nm = pkg.sweeps.llf_vs_iteration(a.T_d, a.T_p, a.N, a.n_rx, a.n_tx, a.itera,
                                              a.monte_iter, a.M, a.varn, a.seed,
                                              replay=not a.no_replay)
    report("iter", it, {"Proposed method": llf}, a.out, "Proposed method with DFT for pilots",
           ylabel="LLF", logy=False)


if __name__ == "__main__":
    main()
