"""CPU tier: the oracle (both faces) and the host-side signal model are pinned
against golden vectors produced by the reference's own functions
(tests/golden/make_golden.py, SURVEY.md §8c known-answer values)."""
import numpy as np
import pytest

from conftest import golden, rel
from oracle.em_loop import em_loop, llf_genie
from oracle.em_reduced import (em_reduced, u_from_zp, cons_from_aps, aps_from_cons, nmse,
                               estep_moments, mstep_build, mstep_solve)

SOFT_CASES = ["kat1_s7", "kat1_s11", "nt3_m4", "nt1_m16", "root_tp", "nt4_m4", "nt2_m16",
              "nt2_m64"]


def _run_reduced(d, mode="soft", itera=None):
    n_rx = int(d["n_rx"])
    it = itera or (int(d["itera"]) if "itera" in d else 2)
    return em_reduced(d["Y_d"], d["Y_p"], u_from_zp(d["Z_p"], n_rx), d["Ptd"], d["aps"],
                      float(d["varn"]), it, d["h0"], mode=mode, return_trace=True)


@pytest.mark.parametrize("case", SOFT_CASES)
def test_reduced_oracle_matches_reference_em(case):
    d = golden(case)
    th, _ = _run_reduced(d)
    ref = d["theta"] if "theta" in d else d["theta_it2"]
    assert rel(th, ref) < 1e-12


def test_kat1_known_answers():
    """seed 7 NMSE(theta0)=0.3124412991124182, NMSE(em)=7.765079093716e-02;
    seed 11 NMSE(em)=5.305423058721e-02."""
    d7, d11 = golden("kat1_s7"), golden("kat1_s11")
    assert abs(nmse(d7["h0"], d7["h"]) - 0.3124412991124182) < 1e-13
    assert abs(float(d7["nmse_it2"]) - 7.765079093716e-02) < 1e-13
    assert abs(float(d11["nmse_it2"]) - 5.305423058721e-02) < 1e-13
    th, tr = _run_reduced(d7)
    assert rel(tr[0], d7["theta_it1"]) < 1e-12
    assert abs(nmse(th, d7["h"]) / 7.765079093716e-02 - 1) < 1e-10


def test_loop_oracle_matches_reference():
    d = golden("kat1_s7")
    Y_d = [y[:, None] for y in d["Y_d"]]
    Y_p = [y[:, None] for y in d["Y_p"]]
    th = em_loop(Y_d, Y_p, 40, 12, list(d["Z_p"]), d["Ptd"], d["aps"], 4, float(d["varn"]), 2,
                 d["h0"])
    assert rel(th, d["theta_it2"]) < 1e-12
    thm = em_loop(Y_d, Y_p, 40, 12, list(d["Z_p"]), d["Ptd"], d["aps"], 4, float(d["varn"]), 2,
                  d["h0"], hard=True)
    assert rel(thm, d["ml_theta"]) < 1e-12


def test_hard_ml_and_llf_match_reference():
    """IterationsvsLLF.em and ML_detecctor.em on the KAT-1 seed-7 data."""
    d = golden("kat1_s7")
    n_rx, varn = 2, float(d["varn"])
    Ud = np.einsum("pt,ta->tpa", d["Ptd"], d["X_d"]).reshape(d["Y_d"].shape[0], -1)
    Zd = np.stack([np.kron(u[None], np.eye(n_rx)) for u in Ud])
    for mode, key_th, key_llf in (("soft", "llf_soft_theta", "llf_soft"),
                                  ("hard", "ml_theta", "ml_llf")):
        th, tr = _run_reduced(d, mode=mode, itera=2)
        assert rel(th, d[key_th]) < 1e-12
        llf = [llf_genie(t, d["Y_p"][..., None], d["Z_p"], d["Y_d"][..., None], Zd, 40, 12, 2, 4,
                         varn) for t in tr]
        assert rel(llf, d[key_llf]) < 1e-12


def test_kat2_nmse_vs_snr_curve():
    """KAT-2: PMd/SNR/all_Detectors.py em at SNR -5..20 dB (the north-star curve)."""
    k = golden("kat2_snr")
    Up = u_from_zp(k["Z_p"], 2)
    survey = [7.116100579890e-01, 4.735312842427e-01, 1.325647368276e-01, 2.408388722975e-01,
              5.924439598782e-02, 2.295354158055e-01]
    for i in range(6):
        th = em_reduced(k["Y_d"][i], k["Y_p"][i], Up, k["Ptd"], k["aps"], float(k["varn"][i]), 5,
                        k["h0"][i])
        assert rel(th, k["theta"][i]) < 1e-12
        assert abs(nmse(th, k["h"]) / k["nmse"][i] - 1) < 1e-10
        assert abs(k["nmse"][i] / survey[i] - 1) < 1e-10
        thm = em_reduced(k["Y_d"][i], k["Y_p"][i], Up, k["Ptd"], k["aps"], float(k["varn"][i]),
                         5, k["h0"][i], mode="hard")
        assert rel(thm, k["theta_ml"][i]) < 1e-12


def test_constellation_and_hypothesis_order(sbce):
    q = golden("qam")
    for M in (4, 16, 64, 256):
        assert np.array_equal(sbce.qam.qam_constellation(M), q[f"cons{M}"])
    assert sbce.qam.energy_per_symbol(16) == 10.0
    for case in ("kat1_s7", "nt2_m16", "nt3_m4", "nt4_m4"):
        d = golden(case)
        M, n_tx = int(d["M"]), int(d["n_tx"])
        cons = cons_from_aps(d["aps"], M)
        assert np.array_equal(cons, q[f"cons{M}"])
        assert np.array_equal(aps_from_cons(cons, n_tx), d["aps"])
        assert np.array_equal(sbce.qam.all_possible_symbols(cons, n_tx), d["aps"])


def test_signal_model_replays_reference_rng(sbce):
    """np.random.seed(s) + the north-star call order reproduces the reference's data."""
    sm = sbce.signal_model
    for case in ("kat1_s7", "nt3_m4", "nt2_m16"):
        d = golden(case)
        N, n_tx, n_rx = int(d["N"]), int(d["n_tx"]), int(d["n_rx"])
        T_d, T_p, M, varn = int(d["T_d"]), int(d["T_p"]), int(d["M"]), float(d["varn"])
        np.random.seed(int(d["seed"]))
        h = sm.channel_matrix(n_tx, n_rx, N, 1.0)
        X_d, aps = sm.symbols(n_tx, M, T_d)
        X_p = sm.pilot_symbols(n_tx, M, T_p)
        Ptp, Ptd = sm.irs_matrix(T_p, T_d, N)
        Ptd = sm.insert_direct(Ptd)
        Y_p, Y_d, U_p, U_d, h0 = sm.received_signals(T_p, T_d, Ptp, Ptd, n_rx, n_tx, X_d, X_p, h,
                                                     varn)
        assert np.array_equal(h, d["h"])
        assert np.array_equal(np.stack(X_d)[..., 0], d["X_d"])
        assert np.array_equal(np.stack(X_p)[..., 0], d["X_p"])
        assert np.array_equal(aps, d["aps"])
        assert np.array_equal(Ptd, d["Ptd"]) and np.array_equal(Ptp, d["Ptp"])
        assert rel(Y_p, d["Y_p"]) < 1e-14 and rel(Y_d, d["Y_d"]) < 1e-14
        assert rel(U_p, u_from_zp(d["Z_p"], n_rx)) == 0.0
        assert rel(h0, d["h0"]) < 1e-12


def test_root_variant_replay(sbce):
    """Root-level script: C-order h, N x T_p DFT over T_p plus a ones row (pilots drawn after
    the RIS phases)."""
    sm = sbce.signal_model
    d = golden("root_tp")
    N, n_tx, n_rx, T_d, T_p, M = 4, 2, 2, 10, 6, 4
    np.random.seed(3)
    h = sm.channel_matrix(n_tx, n_rx, N, 1.0, order="C")
    X_d, aps = sm.symbols(n_tx, M, T_d)
    Ptp, Ptd = sm.irs_matrix(T_p, T_d, N, pilot="dft_tp")
    Ptp, Ptd = sm.insert_direct(Ptp), sm.insert_direct(Ptd)
    X_p = sm.pilot_symbols(n_tx, M, T_p)
    Y_p, Y_d, U_p, _, _ = sm.received_signals(T_p, T_d, Ptp, Ptd, n_rx, n_tx, X_d, X_p, h, 0.1,
                                              with_initial=False)
    assert np.array_equal(h, d["h"])
    assert rel(Y_d, d["Y_d"]) < 1e-14 and rel(Y_p, d["Y_p"]) < 1e-14


def test_moments_are_consistent():
    """E-step moments: S Hermitian PSD with diag >= |m|^2; hard mode gives x x^H."""
    rng = np.random.default_rng(0)
    d = golden("nt2_m16")
    theta = d["h0"] + 0.1 * (rng.normal(size=d["h0"].shape) + 1j * rng.normal(size=d["h0"].shape))
    m, S, dmin, logZ = estep_moments(theta, d["Y_d"], d["Ptd"], d["aps"], float(d["varn"]))
    assert np.allclose(S, np.conj(np.transpose(S, (0, 2, 1))))
    for t in range(S.shape[0]):
        assert np.linalg.eigvalsh(S[t] - np.outer(m[t], np.conj(m[t]))).min() > -1e-12
    mh, Sh, _, _ = estep_moments(theta, d["Y_d"], d["Ptd"], d["aps"], float(d["varn"]), "hard")
    assert np.allclose(Sh, mh[:, :, None] * np.conj(mh[:, None, :]))


def test_reduced_normal_equations_equal_kronecker_form():
    """The commutation identity: (conj(R) (x) I, vec(B)) equals the reference's K x K
    sums sum w Z^H Z, sum w Z^H y built from dense Kronecker regressors."""
    d = golden("nt3_m4")
    n_rx, n_tx = int(d["n_rx"]), int(d["n_tx"])
    Up = u_from_zp(d["Z_p"], n_rx)
    m, S, _, _ = estep_moments(d["h0"], d["Y_d"], d["Ptd"], d["aps"], float(d["varn"]))
    R, rhs = mstep_build(Up, d["Y_p"], d["Ptd"], d["Y_d"], m, S)
    # dense reference-form sums with the same posterior
    aps = d["aps"]
    J = aps.shape[0]
    P, T = d["Ptd"].shape
    K = P * n_tx * n_rx
    A = np.zeros((K, K), complex)
    bvec = np.zeros((K, 1), complex)
    H = np.asarray(d["h0"])
    for t in range(T):
        psi = d["Ptd"][:, t]
        Zs = [np.kron(np.kron(psi[None], aps[j][None]), np.eye(n_rx)) for j in range(J)]
        dd = np.array([np.linalg.norm(d["Y_d"][t][:, None] - Z @ H[:, None]) ** 2 for Z in Zs])
        w = np.exp(-(dd - dd.min()) / float(d["varn"]) ** 2)
        w /= w.sum()
        for j in range(J):
            A += w[j] * np.conj(Zs[j]).T @ Zs[j]
            bvec += w[j] * np.conj(Zs[j]).T @ d["Y_d"][t][:, None]
    for t in range(len(d["Z_p"])):
        A += np.conj(d["Z_p"][t]).T @ d["Z_p"][t]
        bvec += np.conj(d["Z_p"][t]).T @ d["Y_p"][t][:, None]
    assert rel(np.kron(np.conj(R), np.eye(n_rx)), A) < 1e-12
    assert rel(np.conj(rhs).reshape(-1), bvec) < 1e-12
    assert rel(mstep_solve(R, rhs), np.linalg.solve(A, bvec)) < 1e-10


def test_reduced_lstsq_equals_kronecker_form_lstsq(sbce):
    """PM.py:108 runs np.linalg.lstsq on the K x K sums; on a rank-deficient system
    (L = 66 > T_p + T_d = 32, weight-1 hypotheses) the reduced-form restatement with
    rcond = eps * K returns the same minimum-norm theta and rank (n_rx copies)."""
    from oracle.em_reduced import mstep_lstsq
    n_tx, n_rx, N, T_p, T_d = 2, 2, 32, 12, 20
    b = sbce.signal_model.synthetic_batch(1, n_tx, n_rx, N, T_p, T_d, 4, 0.05, seed=21)
    Psi, x = b["psi_d"][0].T, b["x_d"][0]
    S = x[:, :, None] * np.conj(x[:, None, :])
    R, rhs = mstep_build(b["u_p"][0], b["y_p"][0], Psi, b["y_d"][0], x, S)
    K = R.shape[0] * n_rx
    A = np.zeros((K, K), complex)
    bvec = np.zeros((K, 1), complex)
    for t in range(T_d):
        Z = np.kron(np.kron(Psi[:, t][None], x[t][None]), np.eye(n_rx))
        A += np.conj(Z).T @ Z
        bvec += np.conj(Z).T @ b["y_d"][0][t][:, None]
    for t in range(T_p):
        Z = np.kron(b["u_p"][0][t][None], np.eye(n_rx))
        A += np.conj(Z).T @ Z
        bvec += np.conj(Z).T @ b["y_p"][0][t][:, None]
    th_ref, _, rank_ref, _ = np.linalg.lstsq(A, bvec)      # the reference call, default rcond
    th, rank = mstep_lstsq(R, rhs)
    assert rank_ref == n_rx * rank and rank <= T_p + T_d
    assert rel(th, th_ref) < 1e-10


def test_gemm_build_equals_einsum_build(sbce):
    from oracle.em_reduced import mstep_build_gemm
    b = sbce.signal_model.synthetic_batch(1, 3, 2, 7, 5, 30, 16, 0.1, seed=2)
    rng = np.random.default_rng(0)
    m = rng.standard_normal((30, 3)) + 1j * rng.standard_normal((30, 3))
    C = rng.standard_normal((30, 3, 3)) + 1j * rng.standard_normal((30, 3, 3))
    S = C @ np.conj(np.swapaxes(C, 1, 2))
    args = (b["u_p"][0], b["y_p"][0], b["psi_d"][0].T, b["y_d"][0], m, S)
    R0, r0 = mstep_build(*args)
    R1, r1 = mstep_build_gemm(*args)
    assert rel(R1, R0) < 1e-13 and rel(r1, r0) < 1e-13


def _fexp_neg_numpy(z):
    """Bit-level numpy mirror of csrc/sbce_internal.h fexp_neg (Cody-Waite + degree-12)."""
    z = np.maximum(z, -745.5)
    kd = np.rint(z * 1.4426950408889634074)
    # the device reduction is an FMA; kd*ln2_hi (11 x 53 bits) is exact in x87 long double
    ld = np.longdouble
    r = (ld(z) - kd.astype(ld) * ld(6.93147180559945286227e-01)).astype(np.float64)
    r = r - kd * 2.31904681384629955842e-17
    c = [1.0, 1.0, 0.5, 1.66666666666666666667e-01, 4.16666666666666666667e-02,
         8.33333333333333333333e-03, 1.38888888888888888889e-03, 1.98412698412698412698e-04,
         2.48015873015873015873e-05, 2.75573192239858906526e-06, 2.75573192239858906526e-07,
         2.50521083854417187751e-08, 2.08767569878680989792e-09]
    p = np.full_like(r, c[12])
    for k in range(11, -1, -1):
        p = p * r + c[k]
    return np.ldexp(p, kd.astype(np.int64))


def test_device_exp_polynomial_accuracy():
    """The E-step's exp() (sbce_internal.h fexp_neg) is accurate to a few ulp on [-745, 0]."""
    z = -np.concatenate([np.linspace(0, 1, 2001), np.linspace(1, 700, 20001)])
    got = _fexp_neg_numpy(z)
    want = np.exp(z)
    rel_err = np.abs(got - want) / want
    assert rel_err.max() < 1e-15
    assert _fexp_neg_numpy(np.array([-np.inf]))[0] == 0.0
    assert _fexp_neg_numpy(np.array([0.0]))[0] == 1.0


def test_sweep_snr_replay_reproduces_reference_data(sbce):
    """sweeps.gen_snr replays PMd/SNR/all_Detectors.py's draw order (KAT-2 data)."""
    k = golden("kat2_snr")
    pts, varns = sbce.sweeps.gen_snr(monte_iter=1, seed=0)
    assert np.allclose(varns, k["varn"], rtol=1e-15)
    for i in range(6):
        t = pts[i][0]
        assert np.array_equal(t["h"], k["h"])
        assert np.array_equal(t["Psi_d"], k["Ptd"])
        assert rel(t["Y_d"], k["Y_d"][i]) < 1e-14 and rel(t["Y_p"], k["Y_p"][i]) < 1e-14
        assert rel(t["h0"], k["h0"][i]) < 1e-12


PM_CASES = [("kat1_s7", "pm_r0_theta", False, 0, 3), ("kat1_s7", "pmbeta_r1_theta", True, 1, 3),
            ("pm_nt4", "pm_theta", False, None, None), ("pm_nt4", "pmbeta_theta", True, None, None),
            ("pm_nt3_m16", "pm_theta", False, None, None),
            ("pm_nt3_m16", "pmbeta_theta", True, None, None)]


@pytest.mark.parametrize("case,key,soft,r,itera", PM_CASES)
def test_pm_oracle_matches_reference(case, key, soft, r, itera):
    """PM.em_pm (uniform list) and PM_beta.em_pm (posterior list) incl. the off-by-one
    list channel, the concatenated stream order and the oracle early stop."""
    from oracle.pm import em_pm
    d = golden(case)
    n_tx, n_rx, M = int(d["n_tx"]), int(d["n_rx"]), int(d["M"])
    if r is None:
        r = int(d["r_soft"] if soft else d["r_uniform"])
        itera = int(d["itera"])
    th = em_pm(d["Y_d"], d["Y_p"], u_from_zp(d["Z_p"], n_rx), d["Ptd"], float(d["varn"]), itera,
               d["h0"], n_tx, n_rx, r, cons_from_aps(d["aps"], M), soft=soft, h=d["h"])
    assert rel(th, d[key]) < 1e-12


DET_CASES = [("kat1_s7", 3), ("det_nt3", None), ("det_nt2_m16", None)]


@pytest.mark.parametrize("case,itera", DET_CASES)
@pytest.mark.parametrize("kind", ["zf", "mmse"])
def test_detector_oracle_matches_reference(case, itera, kind):
    """all_detectorsvsTd.em_zf / em_mmse: off-by-one channel, flattened-argmin decision,
    oracle early stop."""
    from oracle.detectors import em_detector
    d = golden(case)
    n_tx, n_rx = int(d["n_tx"]), int(d["n_rx"])
    th = em_detector(d["Y_d"], d["Y_p"], u_from_zp(d["Z_p"], n_rx), d["Ptd"], d["aps"],
                     float(d["varn"]), itera or int(d["itera"]), d["h0"], n_tx, n_rx, kind,
                     h=d["h"])
    assert rel(th, d[kind + "_theta"]) < 1e-12


def test_flattened_argmin_closed_form():
    """nearest_symbol_ecul's flat argmin over (J, n_tx, n_tx) (all_detectorsvsTd.py:49-52)
    equals the closed form the device kernel uses, incl. the IndexError cases."""
    import itertools
    from oracle.detectors import ecul_literal, ecul_index
    q = golden("qam")
    rng = np.random.default_rng(0)
    for M, nt in ((4, 2), (4, 3), (16, 2), (64, 2)):
        cons = q[f"cons{M}"]
        aps = np.array(list(itertools.product(*([cons] * nt))))
        for _ in range(300):
            z = (rng.standard_normal(nt) + 1j * rng.standard_normal(nt)) * np.abs(cons).max()
            f = ecul_index(z, aps, M)
            if f >= len(aps):
                with pytest.raises(IndexError):
                    ecul_literal(z, aps)
            else:
                assert np.array_equal(ecul_literal(z, aps), aps[f])


def test_ser_oracle_matches_reference():
    """SER/log_max_SER.py em decisions + the script's SER expression (:162)."""
    from oracle.ser import em_hard_with_decisions, ser_reference, ser_elementwise
    d = golden("ser_logmax")
    n_rx = int(d["n_rx"])
    for k in range(2):
        th, dec = em_hard_with_decisions(d[f"Y_d{k}"], d[f"Y_p{k}"], u_from_zp(d[f"Z_p{k}"], n_rx),
                                         d["Ptd"], d["aps"], float(d[f"varn{k}"]), int(d["itera"]),
                                         d[f"h0{k}"])
        assert rel(th, d[f"theta{k}"]) < 1e-12
        assert np.array_equal(dec, d[f"X_dest{k}"])
        assert ser_reference(d["X_d"], d[f"X_dest{k}"]) == float(d[f"ser{k}"])
        assert 0.0 <= ser_elementwise(d["X_d"], dec) <= ser_reference(d["X_d"], dec)


def test_ser_sweep_replays_reference_data(sbce):
    """sweeps.gen_ser reproduces log_max_SER.py's draw order (data of the fixture)."""
    d = golden("ser_logmax")
    points, varns = sbce.sweeps.gen_ser(tuple(int(x) for x in d["snr"]), int(d["T_d"]),
                                        int(d["T_p"]), int(d["N"]), int(d["n_rx"]),
                                        int(d["n_tx"]), 1, int(d["M"]), 10.0, 5)
    for k in range(2):
        t = points[k][0]
        # Y = Z h is a dense matmul in the reference: equal to rounding, not bitwise
        assert rel(t["Y_d"], d[f"Y_d{k}"]) < 1e-13 and rel(t["Y_p"], d[f"Y_p{k}"]) < 1e-13
        assert rel(t["h0"], d[f"h0{k}"]) < 1e-12
        assert np.array_equal(t["X_d"], d["X_d"])
        assert abs(varns[k] - float(d[f"varn{k}"])) < 1e-15


def _sup_padded(d, k):
    T = d[f"Y{k}"].shape[0]
    Xs = np.zeros((T, int(d["n_tx"])), dtype=complex)
    Xp = d[f"X_p{k}"][:T]
    Xs[:Xp.shape[0]] = Xp
    return Xs


def test_superimposed_oracle_matches_reference():
    """Parallel/ParallelProtocol_Tp.py em: hypotheses x_j + x_p,t, T_p < T_d and T_p > T_d."""
    from oracle.superimposed import em_superimposed
    d = golden("superimposed")
    for k in range(2):
        th = em_superimposed(d[f"Y{k}"], d[f"Psi{k}"], d["aps"], float(d["varn"]),
                             int(d["itera"]), _sup_padded(d, k))
        assert rel(th, d[f"theta{k}"]) < 1e-12


def test_superimposed_sweep_replays_reference_data(sbce):
    d = golden("superimposed")
    pts = sbce.sweeps.gen_superimposed(tuple(int(x) for x in d["T_ps"]), int(d["T_d"]), int(d["N"]),
                                       int(d["n_rx"]), int(d["n_tx"]), 1, int(d["M"]),
                                       float(d["varn"]), 17)
    for k in range(2):
        t = pts[k][0]
        assert np.array_equal(t["h"], d["h"]) and np.array_equal(t["Psi"], d[f"Psi{k}"])
        assert np.array_equal(t["X_sup"], _sup_padded(d, k))
        assert rel(t["Y"], d[f"Y{k}"]) < 1e-13


# ---------------------------------------------------------------- Gaussian-prior EM
def _gauss_case(d, k):
    N, n_tx, n_rx, T_d, T_p, itera = (int(v) for v in d[f"dims{k}"])
    return N, n_tx, n_rx, T_d, T_p, itera, float(d[f"varn{k}"]), float(d[f"varx{k}"])


@pytest.mark.parametrize("k", range(5))
def test_gaussian_oracle_matches_reference(k):
    """MIMO_Gaussian_proposed.py EM_Gaussian_proposed: the literal Q x Q restatement and the
    reduced form (+ expansion) against the reference's own output (n_rx = 2, 1, 3; varx != 1)."""
    from oracle import gaussian as g
    d = golden("gaussian")
    N, n_tx, n_rx, T_d, T_p, itera, varn, varx = _gauss_case(d, k)
    ref = d[f"H_hat{k}"]
    # case 4 (N = 32, Q = 256): the reference's lstsq pseudo-inverse of the rank-65 256 x 256
    # A is itself only good to ~1e-5 (two lstsq orderings differ by 2e-5)
    tol = 1e-10 if k < 4 else 1e-4
    lit = g.em_gaussian_literal(d[f"Y_d{k}"], d[f"Y_p{k}"], d[f"Z_p{k}"], d[f"Ptd{k}"], varn,
                                itera, d[f"H0{k}"], varx, n_tx)
    assert rel(lit, ref) < tol
    U = np.stack([np.kron(d[f"Ptp{k}"][:, t], d[f"X_p{k}"][:, t]) for t in range(T_p)])
    Hr = g.em_gaussian_reduced(d[f"Y_d{k}"], d[f"Y_p{k}"], U, d[f"Ptd{k}"], varn, itera,
                               g.reduce_channel(d[f"H0{k}"], n_tx, n_rx), varx, n_tx)
    assert rel(g.expand(Hr, n_rx), ref) < tol


def test_gaussian_host_layout(sbce):
    """Host-side reduction of the reference's z_p / H_initial (em.gaussian_regressors,
    em.reduce_gaussian_channel) against the oracle."""
    from oracle import gaussian as g
    d = golden("gaussian")
    for k in range(4):
        N, n_tx, n_rx, T_d, T_p, itera, varn, varx = _gauss_case(d, k)
        U = sbce.gaussian_regressors(list(d[f"Z_p{k}"]), N, n_tx, n_rx)
        Uo = np.stack([np.kron(d[f"Ptp{k}"][:, t], d[f"X_p{k}"][:, t]) for t in range(T_p)])
        assert rel(U, Uo) < 1e-15
        th = sbce.reduce_gaussian_channel(d[f"H0{k}"], n_tx, n_rx)
        assert rel(th, g.reduce_channel(d[f"H0{k}"], n_tx, n_rx).T.reshape(-1)) < 1e-15
    bad = np.array(d["Z_p0"])
    bad[0, 1] = 1.0
    with pytest.raises(ValueError):
        sbce.gaussian_regressors(list(bad), 4, 2, 2)


def test_gaussian_sweep_replays_reference_data(sbce):
    """sweeps.gen_gaussian reproduces the reference script's draw order (fixture case 0/1)."""
    d = golden("gaussian")
    for k, seed in ((0, 31), (1, 32)):
        N, n_tx, n_rx, T_d, T_p, itera, varn, varx = _gauss_case(d, k)
        t = sbce.sweeps.gen_gaussian((T_p,), T_d, N, n_rx, n_tx, 1, varn, varx, seed)[0][0]
        H = sbce.signal_model.full_gaussian_channel(t["h"], n_rx)
        assert np.array_equal(H, d[f"H{k}"])
        assert np.array_equal(t["Psi_d"], d[f"Ptd{k}"])
        assert rel(t["Y_d"], d[f"Y_d{k}"]) < 1e-13 and rel(t["Y_p"], d[f"Y_p{k}"]) < 1e-13
        assert rel(t["h0"], sbce.reduce_gaussian_channel(d[f"H0{k}"], n_tx, n_rx)) < 1e-12


# ---------------------------------------------------------------- all_detectorsvsTd / LLF drivers
def test_detector_grid_replays_reference_data(sbce):
    """sweeps.gen_detectors reproduces PMd/all_detectorsvsTd.py's data (its own helpers, its
    driver's draw order :371-382) at the fixture's T_d point."""
    d = golden("alldet_td15")
    points, varns = sbce.sweeps.gen_detectors((int(d["T_d"]),), None, int(d["T_p"]), int(d["N"]),
                                              int(d["n_rx"]), int(d["n_tx"]), 1, int(d["M"]),
                                              float(d["varn"]), seed=int(d["seed"]))
    t = points[0][0][0]
    assert rel(t["h"], d["h"]) < 1e-15
    assert rel(t["Y_d"], d["Y_d"]) < 1e-13 and rel(t["Y_p"], d["Y_p"]) < 1e-13
    assert rel(t["h0"], d["h0"]) < 1e-10
    assert rel(t["Psi_d"], d["Ptd"]) < 1e-15


def test_detector_oracles_match_reference_five_ems():
    """The oracle restatements of all_detectorsvsTd.py's five EMs (oracle early stop on the
    true h in every one) against the reference's own outputs at one T_d point."""
    from oracle.pm import em_pm
    from oracle.detectors import em_detector
    d = golden("alldet_td15")
    n_rx, n_tx, itera = int(d["n_rx"]), int(d["n_tx"]), int(d["itera"])
    Up = u_from_zp(d["Z_p"], n_rx)
    varn, h = float(d["varn"]), d["h"]
    args = (d["Y_d"], d["Y_p"], Up, d["Ptd"])
    got = {
        "pm": em_pm(*args, varn, itera, d["h0"], n_tx, n_rx, int(d["partition_r"]), d["cons"],
                    soft=True, h=h),
        "ml": em_reduced(*args, d["aps"], varn, itera, d["h0"], mode="hard", h=h),
        "zf": em_detector(*args, d["aps"], varn, itera, d["h0"], n_tx, n_rx, "zf", h=h),
        "mmse": em_detector(*args, d["aps"], varn, itera, d["h0"], n_tx, n_rx, "mmse", h=h),
        "em": em_reduced(*args, d["aps"], varn, itera, d["h0"], h=h),
    }
    for k, th in got.items():
        assert rel(th, d[f"{k}_theta"]) < 1e-9, k
        assert abs(nmse(th, h) / float(d[f"{k}_nmse"]) - 1) < 1e-9, k


def test_llf_driver_replays_reference(sbce):
    """sweeps.gen_llf reproduces PMd/IterationsvsLLF.py's driver data, and the oracle's genie
    LLF (:76) on them equals the reference's per-trial LLF curves."""
    from oracle.em_loop import llf_genie
    d = golden("llf_driver")
    n_tx, n_rx, T_d, T_p, M = (int(d[k]) for k in ("n_tx", "n_rx", "T_d", "T_p", "M"))
    varn, itera = float(d["varn"]), int(d["itera"])
    trials = sbce.sweeps.gen_llf(T_d, T_p, int(d["N"]), n_rx, n_tx, int(d["monte_iter"]), M, varn,
                                 seed=int(d["seed"]))
    aps = sbce.qam.all_possible_symbols(sbce.qam.qam_constellation(M), n_tx)
    for i, t in enumerate(trials):
        assert rel(t["h"], d[f"h{i}"]) < 1e-15 and rel(t["Y_d"], d[f"Y_d{i}"]) < 1e-13
        th, trace = em_reduced(t["Y_d"], t["Y_p"], t["U_p"], t["Psi_d"], aps, varn, itera, t["h0"],
                               return_trace=True)
        assert rel(th, d[f"theta{i}"]) < 1e-10
        Z_p = [np.kron(u[None], np.eye(n_rx)) for u in t["U_p"]]
        Z_d = [np.kron(np.kron(t["Psi_d"][:, k][None], t["X_d"][k][None]), np.eye(n_rx))
               for k in range(T_d)]
        llf = [llf_genie(th_l, t["Y_p"][..., None], Z_p, t["Y_d"][..., None], Z_d, T_d, T_p, n_tx, M,
                         varn)
               for th_l in trace]
        assert np.allclose(llf, d[f"llf{i}"], rtol=1e-11, atol=0)


def test_oracle_matches_reference_at_cfg1_kernel_instantiation():
    """n_tx = n_rx = 4, 16-QAM (J = 65,536, the cfg-1 E-step) through the reference em()
    itself (tests/golden/make_golden.py case_cfg1_kernel): the reduced-form oracle agrees."""
    d = golden("cfg1_kernel")
    n_rx = int(d["n_rx"])
    Up = u_from_zp(d["Z_p"], n_rx)
    for it in (1, int(d["itera"])):
        th = em_reduced(d["Y_d"], d["Y_p"], Up, d["Ptd"], d["aps"], float(d["varn"]), it, d["h0"])
        assert rel(th, d[f"theta_it{it}"]) < 1e-11, it


# ------------------------------------------------- the five curves of PMd/SNR/all_Detectors.py
_SNR_KEYS = {"pm_soft": "pm", "hard": "ml", "zf": "zf", "mmse": "mmse", "soft": "em"}


def _oracle_snr_em(mode, y_d, y_p, psi, u_p, cons, varn, itera, theta0, h, partition_r):
    """The oracle twin of one SNR-script EM (CPU), one trial."""
    from oracle.pm import em_pm
    from oracle.detectors import em_detector
    n_rx = y_d.shape[1]
    n_tx = u_p.shape[1] // psi.shape[0]
    if mode == "pm_soft":
        return em_pm(y_d, y_p, u_p, psi, varn, itera, theta0, n_tx, n_rx, partition_r, cons,
                     soft=True, h=h)
    aps = aps_from_cons(cons, n_tx)
    if mode in ("zf", "mmse"):
        return em_detector(y_d, y_p, u_p, psi, aps, varn, itera, theta0, n_tx, n_rx, mode, h=h)
    return em_reduced(y_d, y_p, u_p, psi, aps, varn, itera, theta0, mode=mode)


def test_kat2_driver_five_detectors_oracle_vs_reference():
    """The oracle's five EMs (PM r=1 with the early stop, log-max, ZF, MMSE, exact; no early stop
    for the last four, as PMd/SNR/all_Detectors.py has them) against the reference's own run of
    the script's driver (tests/golden/kat2_driver.npz: 3 trials x 6 SNR points)."""
    k = golden("kat2_driver")
    n_rx, itera, r = int(k["n_rx"]), int(k["itera"]), int(k["partition_r"])
    dets = [str(x) for x in k["dets"]]
    for i in range(int(k["monte_iter"])):
        Up = u_from_zp(k[f"Z_p{i}"], n_rx)
        for j in range(len(k["snr"])):
            for mode, key in _SNR_KEYS.items():
                if f"{key}_theta{i}_{j}" not in k:
                    continue
                stop = mode == "pm_soft"
                th = _oracle_snr_em(mode, k[f"Y_d{i}_{j}"], k[f"Y_p{i}_{j}"], k[f"Ptd{i}"], Up,
                                    k["cons"], float(k["varn"][j]), itera, k[f"h0{i}_{j}"],
                                    k[f"h{i}"] if stop else None, r)
                assert rel(th, k[f"{key}_theta{i}_{j}"]) < 1e-11, (mode, i, j)
                nm = nmse(th, k[f"h{i}"])
                assert abs(nm / k["nmse"][dets.index(key), i, j] - 1) < 1e-9


def test_snr_sweep_replays_reference_driver_data(sbce):
    """sweeps.gen_snr (seed 0) reproduces the SNR script's draw order over several trials."""
    k = golden("kat2_driver")
    n = int(k["monte_iter"])
    points, varns = sbce.sweeps.gen_snr(monte_iter=n, seed=0)
    assert np.allclose(varns, k["varn"], rtol=1e-15, atol=0)
    for j in range(len(k["snr"])):
        for i in range(n):
            t = points[j][i]
            assert np.array_equal(t["h"], k[f"h{i}"])
            assert rel(t["Y_d"], k[f"Y_d{i}_{j}"]) < 1e-14      # y = Z h + n, summation order
            assert rel(t["Y_p"], k[f"Y_p{i}_{j}"]) < 1e-14
            assert np.array_equal(t["Psi_d"], k[f"Ptd{i}"])
            assert rel(t["h0"], k[f"h0{i}_{j}"]) < 1e-12


def test_snr_sweep_five_detectors_one_collective(sbce, monkeypatch):
    """Host logic of sweeps.nmse_vs_snr on the CPU: every detector with the script's early-stop
    flag (h passed to em_pm only), partition_r = 1 for the PM list, and ONE all-reduce for all
    (detector, SNR) accumulators.  em_batch is replaced by the oracle here (GPU: test_gpu_sweeps)."""
    k = golden("kat2_driver")
    seen = []

    def fake_em_batch(y_d, y_p, psi_d, u_p, cons, varn, itera, theta0, mode="soft",
                      partition_r=0, h_true=None, **kw):
        seen.append((mode, partition_r, h_true is not None))
        vt = np.broadcast_to(np.asarray(varn, dtype=float), (len(y_d),))   # per-trial (ABI 6)
        th = np.stack([_oracle_snr_em(mode, y_d[b], y_p[b], psi_d[b].T, u_p[b], cons, vt[b], itera,
                                      theta0[b], None if h_true is None else h_true[b],
                                      partition_r) for b in range(len(y_d))])
        return dict(theta=th, status=np.zeros(len(y_d), dtype=np.int32))

    class Gloo:
        class ReduceOp:
            SUM = "sum"

        def __init__(self):
            self.calls = 0

        def is_available(self):
            return True

        def is_initialized(self):
            return True

        def get_backend(self):
            return "gloo"

        def all_reduce(self, t, op=None):
            self.calls += 1

    stub = Gloo()
    monkeypatch.setattr(sbce.sweeps, "em_batch", fake_em_batch)
    monkeypatch.setattr(sbce.sweeps, "_dist", lambda: (stub, 1, 0))
    snr, curves, flagged = sbce.sweeps.nmse_vs_snr(monte_iter=int(k["monte_iter"]), seed=0,
                                                   return_status=True)
    assert stub.calls == 1
    assert {(m, r, s) for m, r, s in seen} == {("pm_soft", 1, True), ("hard", 0, False),
                                              ("zf", 0, False), ("mmse", 0, False),
                                              ("soft", 0, False)}
    dets = [str(x) for x in k["dets"]]
    for mode, key in _SNR_KEYS.items():
        ref = k["curve"][dets.index(key)]
        assert np.allclose(curves[mode], ref, rtol=1e-9, atol=0), mode
        assert not flagged[mode].any()


@pytest.mark.parametrize("shape", [(4, 4, 64, 16, 100), (4, 4, 149, 16, 200), (2, 2, 15, 4, 5)])
def test_chol_policy_on_rank_deficient_R(sbce, shape):
    """np.linalg.solve (Proposed_method_NMSEvsTp.py:80) on a rank-deficient R (hard moments,
    rank R <= T_p + T_d < L) has no reproducible answer: the reference's
    LU returns rounding noise.  The device's CHOL policy (oracle.mstep_chol_policy): pivots
    <= 1e-14 max diag R dropped -- finite theta that solves the normal equations and whose
    range-space part is lstsq's minimum-norm solution.  The round-5 clamp policy overflows
    (the cause of the all-NaN theta at L = 600)."""
    from oracle.em_reduced import mstep_chol_policy, mstep_lstsq, range_part
    n_tx, n_rx, N, T_p, T_d = shape
    varn = float(sbce.signal_model.snr_to_varn(20.0))
    b = sbce.signal_model.synthetic_batch(1, n_tx, n_rx, N, T_p, T_d, 16 if n_tx == 4 else 4, varn,
                                          seed=11)
    x = b["x_d"][0]
    S = x[:, :, None] * np.conj(x[:, None, :])
    R, rhs = mstep_build(b["u_p"][0], b["y_p"][0], b["psi_d"][0].T, b["y_d"][0], x, S)
    th_ls, rank = mstep_lstsq(R, rhs)
    assert rank <= T_p + T_d < R.shape[0]
    th_c, bad_c = mstep_chol_policy(R, rhs, clamp=True)
    if R.shape[0] > 64:
        assert not np.isfinite(th_c).all()               # the old clamp overflows
    th, bad = mstep_chol_policy(R, rhs)
    assert np.isfinite(th).all() and bad.any()           # (a noise pivot may sit above tol)
    X = np.conj(th).reshape(R.shape[0], n_rx)
    assert np.abs(R @ X - rhs).max() / np.abs(rhs).max() < 1e-10
    assert rel(range_part(R, th, n_rx), th_ls) < 1e-10


def test_root_td_variant_replay_and_oracle(sbce):
    """Root-level Proposed_method_NMSEvsTd.py (tests/golden/root_td.npz, the reference's own run):
    C-order h, pilots then per T_d point symbols / deterministic DFT data phases over T_d
    (:92-94, irs_matrix(data='dft_td'), no RNG draw) / noise; the zero-initialised EM (:44-77)
    restated by the oracle reproduces the reference theta at both T_d points."""
    sm = sbce.signal_model
    d = golden("root_td")
    N, n_tx, n_rx, T_p, M = (int(d[k]) for k in ("N", "n_tx", "n_rx", "T_p", "M"))
    np.random.seed(int(d["seed"]))
    h = sm.channel_matrix(n_tx, n_rx, N, 1.0, order="C")
    X_p = sm.pilot_symbols(n_tx, M, T_p)
    assert np.array_equal(h, d["h"])
    for k, T_d in enumerate(d["T_ds"]):
        X_d, aps = sm.symbols(n_tx, M, int(T_d))
        Ptp, Ptd = sm.irs_matrix(T_p, int(T_d), N, pilot="dft_tp", data="dft_td")
        Ptp, Ptd = sm.insert_direct(Ptp), sm.insert_direct(Ptd)
        assert np.array_equal(Ptd, d[f"Ptd{k}"]) and np.array_equal(Ptp, d["Ptp"])
        Y_p, Y_d, U_p, _, _ = sm.received_signals(T_p, int(T_d), Ptp, Ptd, n_rx, n_tx, X_d, X_p, h,
                                                  float(d["varn"]), with_initial=False)
        assert rel(Y_d, d[f"Y_d{k}"]) < 1e-14 and rel(Y_p, d[f"Y_p{k}"]) < 1e-14
        th = em_reduced(Y_d, Y_p, U_p, Ptd, aps, float(d["varn"]), int(d["itera"]),
                        np.zeros(len(h), dtype=complex))
        assert rel(th, d[f"theta{k}"]) < 1e-12
