"""GPU tier: the factorised-weight soft E-step (csrc/estep_pair.hip) that resolves the wide
posteriors of the cfg-1 geometry (n_tx = 4, 16-QAM) the sphere pass leaves to the tile sweep.
It must give the sweep's moments (and the oracle's) wherever it runs, take the listed symbols
at low SNR and hand the ones whose factor range it cannot represent back to the sweep."""
import ctypes

import numpy as np
import pytest

from oracle.em_reduced import estep_moments

pytestmark = pytest.mark.gpu


@pytest.fixture(autouse=True, scope="module")
def _torch_first():
    """torch must bring the HIP runtime up before the library's diagnostic entry points
    touch it (called first, they leave torch.cuda.is_available() False)."""
    import torch
    assert torch.cuda.is_available()
    torch.zeros(1, device="cuda")


def _run(sbce, b, th, varn, pair):
    lib = sbce._lib.load_ab()           # the counters live in the A/B build
    with sbce._lib.debug_env(SBCE_ESTEP_PAIR=pair, SBCE_ESTEP_COUNT="1"):
        lib.sbce_debug_estep_sphere(None, 1)
        lib.sbce_debug_estep_pair(None, 1)
        m, S = sbce.estep_batch(b["y_d"], b["psi_d"], b["cons"], th, varn, 4)
        sph = (ctypes.c_ulonglong * 3)()
        lib.sbce_debug_estep_sphere(sph, 0)
        npair = ctypes.c_ulonglong(0)
        lib.sbce_debug_estep_pair(ctypes.byref(npair), 0)
    return m, S, list(sph), npair.value


@pytest.mark.parametrize("n_rx,snr", [(4, -5), (4, 0), (4, 5), (4, 10), (4, 20), (5, 0),
                                      (8, -5), (8, 10)])
def test_pair_estep_matches_sweep(sbce, n_rx, snr):
    varn = float(sbce.signal_model.snr_to_varn(snr))
    b = sbce.signal_model.synthetic_batch(3, 4, n_rx, 16, 16, 96, 16, varn, seed=40 + snr + n_rx)
    scale = np.abs(b["cons"]).max() ** 2
    for th in (b["theta0"], b["h"] + 0.05 * b["theta0"] / np.abs(b["theta0"]).max()):
        m1, S1, sph, npair = _run(sbce, b, th, varn, "1")
        m0, S0, sph0, npair0 = _run(sbce, b, th, varn, "0")
        assert npair0 == 0
        assert sph == sph0                      # the sphere pass is unchanged
        listed = sph[1]
        assert npair <= listed
        if snr <= 0:
            # wide posteriors: every listed symbol is representable (D << 640)
            assert npair == listed, (npair, listed)
        assert np.abs(m1 - m0).max() < 1e-11 * scale, (snr, np.abs(m1 - m0).max())
        assert np.abs(S1 - S0).max() < 1e-11 * scale, (snr, np.abs(S1 - S0).max())
        # Hermitian second moments, diagonal real
        assert np.abs(S1 - np.conj(np.swapaxes(S1, -1, -2))).max() < 1e-12 * scale


@pytest.mark.parametrize("snr", [-5, 0])
def test_pair_estep_vs_oracle_cfg1_geometry(sbce, snr):
    """cfg-1 geometry (4 x 4, N_RIS = 64, 16-QAM) at low SNR, theta_0: the pass resolves the
    listed symbols and the moments equal the oracle's enumeration of all 65,536 hypotheses."""
    varn = float(sbce.signal_model.snr_to_varn(snr))
    b = sbce.signal_model.synthetic_batch(2, 4, 4, 64, 16, 24, 16, varn, seed=7 - snr)
    m, S, sph, npair = _run(sbce, b, b["theta0"], varn, "1")
    assert npair > 0 and npair == sph[1]
    aps = sbce.qam.all_possible_symbols(b["cons"], 4)
    scale = np.abs(b["cons"]).max() ** 2
    for i in range(2):
        m0, S0, _, _ = estep_moments(b["theta0"][i], b["y_d"][i], b["psi_d"][i].T, aps, varn)
        assert np.abs(m[i] - m0).max() < 1e-11 * scale
        assert np.abs(S[i] - S0).max() < 1e-11 * scale


def test_pair_estep_full_em_low_snr_vs_oracle(sbce):
    """Two EM iterations at 0 dB, cfg-1 geometry at reduced N and T_d: theta vs the oracle."""
    from oracle.em_reduced import em_reduced
    from conftest import rel
    varn = float(sbce.signal_model.snr_to_varn(0.0))
    b = sbce.signal_model.synthetic_batch(1, 4, 4, 8, 16, 48, 16, varn, seed=3)
    aps = sbce.qam.all_possible_symbols(b["cons"], 4)
    r = sbce.em_batch(b["y_d"], b["y_p"], b["psi_d"], b["u_p"], b["cons"], varn, 2, b["theta0"])
    th0 = em_reduced(b["y_d"][0], b["y_p"][0], b["u_p"][0], b["psi_d"][0].T, aps, varn, 2,
                     b["theta0"][0])
    assert rel(r["theta"][0], th0) < 1e-10


def _run_nt(sbce, b, th, varn, pair, n_tx):
    lib = sbce._lib.load_ab()           # the counters live in the A/B build
    with sbce._lib.debug_env(SBCE_ESTEP_PAIR=pair, SBCE_ESTEP_COUNT="1"):
        lib.sbce_debug_estep_pair(None, 1)
        m, S = sbce.estep_batch(b["y_d"], b["psi_d"], b["cons"], th, varn, n_tx)
        npair = ctypes.c_ulonglong(0)
        lib.sbce_debug_estep_pair(ctypes.byref(npair), 0)
    return m, S, npair.value


@pytest.mark.parametrize("n_rx,M,snr", [(2, 64, -5), (2, 64, 5), (2, 64, 15), (2, 64, 30),
                                        (3, 16, 0), (2, 4, -5), (4, 64, 10), (8, 16, 20)])
def test_fact2_estep_nt2_matches_sweep_and_oracle(sbce, n_rx, M, snr):
    """n_tx = 2 (BASELINE cfg 5: 2 x 2, N_RIS = 15, 64-QAM): the tree pass routes every symbol it
    does not resolve alone to estep_fact2_kernel -- the factorised tables (four 1-D and four K x K
    log tables, the (a1, b1) sum split into an a1 and a b1 sum) when the range D is representable,
    else the narrow-posterior path (lane = x0, the x1 within e^-50 in a box around h1^H r / g11);
    its moments equal the enumeration / sweep path's (SBCE_ESTEP_PAIR=0) and the oracle's
    enumeration of all M^2 hypotheses to 1e-11 max|c|^2, from -5 to 30 dB."""
    power = {4: 2.0, 16: 10.0, 64: 42.0}[M]          # the square QAM's mean symbol energy
    varn = float(sbce.signal_model.snr_to_varn(snr, power))
    b = sbce.signal_model.synthetic_batch(3, 2, n_rx, 15, 20, 60, M, varn, seed=60 + snr + n_rx,
                                          pinv="scipy")
    scale = np.abs(b["cons"]).max() ** 2
    aps = sbce.qam.all_possible_symbols(b["cons"], 2)
    for th in (b["theta0"], b["h"] + 0.05 * b["theta0"] / np.abs(b["theta0"]).max()):
        m1, S1, npair = _run_nt(sbce, b, th, varn, "1", 2)
        m0, S0, npair0 = _run_nt(sbce, b, th, varn, "0", 2)
        assert npair0 == 0
        if snr <= 5 and M >= 16:                   # (4-QAM, J = 16: the VALU E-step, no sphere pass)
            assert npair > 0
        assert np.abs(m1 - m0).max() < 1e-11 * scale, (snr, np.abs(m1 - m0).max())
        assert np.abs(S1 - S0).max() < 1e-11 * scale, (snr, np.abs(S1 - S0).max())
        mo, So, _, _ = estep_moments(th[0], b["y_d"][0], b["psi_d"][0].T, aps, varn)
        assert np.abs(m1[0] - mo).max() < 1e-11 * scale
        assert np.abs(S1[0] - So).max() < 1e-11 * scale


@pytest.mark.parametrize("n_rx,M,snr", [(2, 64, -5), (2, 64, 10), (2, 64, 30), (3, 16, 0),
                                        (4, 64, 20), (8, 16, 5)])
def test_hard2_estep_nt2_matches_enumeration_and_oracle(sbce, n_rx, M, snr):
    """n_tx = 2 log-max E-step (estep_hard2_kernel: lane = x_0, the best x_1 per axis with a
    rounding-guarded rival check, first minimum in table order): decisions identical to the
    enumeration path (SBCE_ESTEP_PAIR=0) and to the oracle's argmin over all M^2 hypotheses."""
    power = {4: 2.0, 16: 10.0, 64: 42.0}[M]
    varn = float(sbce.signal_model.snr_to_varn(snr, power))
    b = sbce.signal_model.synthetic_batch(3, 2, n_rx, 15, 20, 60, M, varn, seed=80 + snr + n_rx,
                                          pinv="scipy")
    aps = sbce.qam.all_possible_symbols(b["cons"], 2)
    lib = sbce._lib.load_ab()           # the counters live in the A/B build
    for th in (b["theta0"], b["h"] + 0.05 * b["theta0"] / np.abs(b["theta0"]).max()):
        out = {}
        for pair in ("1", "0"):
            with sbce._lib.debug_env(SBCE_ESTEP_PAIR=pair, SBCE_ESTEP_COUNT="1"):
                lib.sbce_debug_estep_pair(None, 1)
                m, S = sbce.estep_batch(b["y_d"], b["psi_d"], b["cons"], th, varn, 2, "hard")
                npair = ctypes.c_ulonglong(0)
                lib.sbce_debug_estep_pair(ctypes.byref(npair), 0)
            out[pair] = (m, S, npair.value)
        assert out["0"][2] == 0 and out["1"][2] > 0
        assert np.array_equal(out["1"][0], out["0"][0])
        assert np.array_equal(out["1"][1], out["0"][1])
        for i in range(3):
            mo, So, _, _ = estep_moments(th[i], b["y_d"][i], b["psi_d"][i].T, aps, varn, "hard")
            assert np.array_equal(out["1"][0][i], mo)
