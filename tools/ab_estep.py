"""Diagnostic: same-process A/B of the E-step under environment arms, at theta_0 (iteration 0)
and at the converged theta, plus the whole cfg1 EM (3 stream sub-batches); moments and theta
compared bitwise across arms.
  python tools/ab_estep.py SBCE_ESTEP_F32=0 SBCE_ESTEP_F32=1     (SNR=0 for the 0 dB point)"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402
import __graft_entry__ as ge  # noqa: E402

pkg = ge.package()
pkg._lib.use_ab()       # the A/B build: SBCE_* switches, counters, clocks
snr = float(os.environ.get("SNR", "20"))
varn = float(pkg.signal_model.snr_to_varn(snr))
batch = pkg.signal_model.synthetic_batch(1000, 4, 4, 64, 16, 256, 16, varn, seed=0)
eng = pkg.EMEngine(batch, varn)
eng3 = pkg.EMEngine(batch, varn, streams=3)


def timeit(fn, reps):
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps


arms = sys.argv[1:] or ["SBCE_ESTEP_F32=0", "SBCE_ESTEP_F32=1"]
out, ref = {}, {}
for rnd in range(2):
    for arm in arms:
        k, v = arm.split("=", 1)
        os.environ[k] = v
        pkg._lib.reload_debug_env()
        eng.theta.copy_(eng.theta0)
        t_e0 = timeit(eng.estep, 5)
        m0 = eng.mom.cpu().numpy()
        t_em = timeit(lambda: eng3.run(20), 2)
        th = eng3.theta.cpu().numpy()
        eng.run(20)
        t_e = timeit(eng.estep, 5)
        m1 = eng.mom.cpu().numpy()
        del os.environ[k]
        pkg._lib.reload_debug_env()
        if not ref:
            ref = {"m0": m0, "m1": m1, "th": th}
        r = {"estep_it0_ms": t_e0, "estep_conv_ms": t_e, "em3_ms": t_em,
             "em3_emits": 20000 / t_em * 1e3,
             "it0_mom_equal": bool(np.array_equal(m0, ref["m0"])),
             "conv_mom_equal": bool(np.array_equal(m1, ref["m1"])),
             "theta_equal": bool(np.array_equal(th, ref["th"]))}
        out.setdefault(arm, []).append(r)
        print(rnd, arm, json.dumps(r), flush=True)
print(json.dumps({"snr": snr, "arms": out}))
