#!/usr/bin/env python3
"""NMSE of the five detector EMs vs T_d (and SNR) -- entry point of
"Proposed method/all_detectorsvsTd.py" (constants :345-363, driver :371-405): soft-decision PM
list EM, log-max EM, ZF, MMSE and the exact EM, on the MI355X.  With --SNR the sweep becomes
the SNR x T_d grid of BASELINE configs[4] (e.g. 20 SNR points, 8 T_d points, --M 64)."""
import argparse

from _cli import init_distributed, package, report  # noqa: E402


def main():
    ap = argparse.ArgumentParser(description=__doc__)
    ap.add_argument("--T-d", type=int, nargs="+", default=[15, 30, 45, 60, 75, 90])
    ap.add_argument("--SNR", type=float, nargs="+", default=None,
                    help="SNR grid in dB (default: the script's single varn)")
    ap.add_argument("--T-p", type=int, default=20)
    ap.add_argument("--N", type=int, default=15)
    ap.add_argument("--n-rx", type=int, default=2)
    ap.add_argument("--n-tx", type=int, default=2)
    ap.add_argument("--itera", type=int, default=5)
    ap.add_argument("--monte-iter", type=int, default=1)
    ap.add_argument("--M", type=int, default=4)
    ap.add_argument("--varn", type=float, default=0.1)
    ap.add_argument("--power", type=float, default=10.0)
    ap.add_argument("--partition-r", type=int, default=1)
    ap.add_argument("--seed", type=int, default=0)
    ap.add_argument("--no-replay", action="store_true")
    ap.add_argument("--no-early-stop", action="store_true")
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    init_distributed()
    pkg = package()
    td, snr, curves = pkg.sweeps.nmse_grid_detectors(
        tuple(a.T_d), None if a.SNR is None else tuple(a.SNR), a.T_p, a.N, a.n_rx, a.n_tx,
        a.itera, a.monte_iter, a.M, a.varn, a.power, a.partition_r, a.seed,
        replay=not a.no_replay, early_stop=not a.no_early_stop)
    labels = {k: v[1] for k, v in pkg.sweeps.DETECTORS.items()}
    if snr is None:
        report("T_d", td, {labels[k]: v[:, 0] for k, v in curves.items()}, a.out,
               "Proposed method with detectors")
    else:
        for j, s in enumerate(snr):
            print(f"SNR {s:g} dB")
            report("T_d", td, {labels[k]: v[:, j] for k, v in curves.items()},
                   None if a.out is None else a.out.replace(".npz", f"_snr{s:g}.npz"),
                   f"Proposed method with detectors, SNR {s:g} dB")


if __name__ == "__main__":
    main()
