"""GPU tier: per-trial noise variances (include/sbce.h sbce_ptrs.varn_t, ABI 6).

One sbce_em call carrying the trials of several SNR points must give every trial exactly what a
call with dims.varn = that trial's varn gives: the E-step kernels derive the posterior constants
(1/varn^2, the 50 varn^2 skip bound, the 0.1 varn^2 ridge) per trial in the host's operation
order, so theta, the early-stop iteration and the status word are BITWISE those of the per-point
calls.  This is what lets the sweep drivers (sweeps.nmse_vs_snr, sweeps.nmse_grid_detectors) and
bench.py --config cfg5 batch a whole SNR axis into one call (SNR/all_Detectors.py:351-354,
all_detectorsvsTd.py:371-405).
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _points(sbce, snrs, B, n_tx, n_rx, N, T_p, T_d, M, power, seed):
    return [sbce.signal_model.synthetic_batch(B, n_tx, n_rx, N, T_p, T_d, M,
                                              float(sbce.signal_model.snr_to_varn(s, power)),
                                              seed=seed + 17 * j)
            for j, s in enumerate(snrs)]


def _cat(pts, key):
    return np.concatenate([p[key] for p in pts])


def _check_modes(sbce, pts, modes, itera, llf=False):
    vt = np.concatenate([np.full(len(p["h"]), p["varn"]) for p in pts])
    for mode, pr in modes:
        kw = dict(mode=mode, partition_r=pr, h_true=_cat(pts, "h"))
        if llf:
            kw["x_d_true"] = _cat(pts, "x_d")
        one = sbce.em_batch(_cat(pts, "y_d"), _cat(pts, "y_p"), _cat(pts, "psi_d"),
                            _cat(pts, "u_p"), pts[0]["cons"], vt, itera, _cat(pts, "theta0"), **kw)
        o = 0
        for p in pts:
            B = len(p["h"])
            kw1 = dict(mode=mode, partition_r=pr, h_true=p["h"])
            if llf:
                kw1["x_d_true"] = p["x_d"]
            r = sbce.em_batch(p["y_d"], p["y_p"], p["psi_d"], p["u_p"], p["cons"], p["varn"], itera,
                              p["theta0"], **kw1)
            assert np.array_equal(one["theta"][o:o + B], r["theta"]), (mode, p["varn"])
            assert np.array_equal(one["iters_done"][o:o + B], r["iters_done"]), mode
            assert np.array_equal(one["status"][o:o + B], r["status"]), mode
            if llf:
                assert np.array_equal(one["llf"][o:o + B], r["llf"]), mode
            o += B


def test_per_trial_varn_bitwise_2x2_64qam_five_detectors(sbce):
    """The cfg5 geometry (2x2, N_RIS = 15, T_p = 20, 64-QAM) at 0 / 15 / 30 dB: the five EMs of
    all_detectorsvsTd.py plus the uniform-weight PM list, early stop on h."""
    pts = _points(sbce, (0.0, 15.0, 30.0), 4, 2, 2, 15, 20, 60, 64, 42.0, seed=71)
    _check_modes(sbce, pts, [("soft", 0), ("hard", 0), ("pm_soft", 1), ("pm", 1), ("zf", 0),
                             ("mmse", 0)], itera=5)


def test_per_trial_varn_bitwise_4x4_16qam_all_estep_paths(sbce):
    """4x4 16-QAM (the cfg1 E-step kernels: tree pass, enumeration, factorised-weight pass, MFMA
    sweep) from -5 dB (wide posteriors: the pair pass and the sweep) to 25 dB (single paths),
    soft and hard, with the genie LLF."""
    pts = _points(sbce, (-5.0, 5.0, 25.0), 3, 4, 4, 12, 16, 64, 16, 10.0, seed=5)
    _check_modes(sbce, pts, [("soft", 0), ("hard", 0)], itera=3, llf=True)


def test_sweep_snr_batching_is_bitwise_neutral(sbce):
    """sweeps.nmse_grid_detectors with the SNR axis in one call per (T_d, detector) equals the
    per-point calls exactly (curves bitwise)."""
    args = ((15, 30), (0.0, 20.0), 20, 15, 2, 2, 5, 3, 64)
    _, _, a = sbce.sweeps.nmse_grid_detectors(*args, power=42.0, seed=9, batch_snr=True)
    _, _, b = sbce.sweeps.nmse_grid_detectors(*args, power=42.0, seed=9, batch_snr=False)
    for det in a:
        assert np.array_equal(a[det], b[det]), det
