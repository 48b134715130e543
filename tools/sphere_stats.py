"""Diagnostic: the prep pass's sphere enumeration on the cfg1 batch (1000 trials) after 0, 1, 5
and 20 EM iterations: symbols resolved / left to the sweep, sweep MFMAs per symbol, and the
E-step time, per arm of environment settings, e.g.
  python tools/sphere_stats.py SBCE_ESTEP_SPHERE=0 SBCE_SPHERE_BUDGET=48 SBCE_SPHERE_BUDGET=96"""
import ctypes
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402
import __graft_entry__ as ge  # noqa: E402

pkg = ge.package()
pkg._lib.use_ab()       # the A/B build: SBCE_* switches, counters, clocks
B = int(os.environ.get("B", "1000"))
varn = float(pkg.signal_model.snr_to_varn(float(os.environ.get("SNR", "20"))))
batch = pkg.signal_model.synthetic_batch(B, 4, 4, 64, 16, 256, 16, varn, seed=0)
eng = pkg.EMEngine(batch, varn)
lib = pkg._lib.load()
nsym = B * 256
for it in (0, 1, 5, 20):
    if it:                   # EMEngine.run restarts from theta_0
        eng.run(it)
    for arm in ["SBCE_X=0"] + sys.argv[1:]:
        k, v = arm.split("=", 1)
        os.environ[k] = v
        os.environ["SBCE_ESTEP_COUNT"] = "1"
        pkg._lib.reload_debug_env()   # the library reads SBCE_* switches once
        cnt = ctypes.c_ulonglong(0)
        sph = (ctypes.c_ulonglong * 3)()
        lib.sbce_debug_estep_mfma(None, 1)
        lib.sbce_debug_estep_sphere(None, 1)
        eng.estep()
        torch.cuda.synchronize()
        lib.sbce_debug_estep_mfma(ctypes.byref(cnt), 0)
        lib.sbce_debug_estep_sphere(sph, 0)
        del os.environ["SBCE_ESTEP_COUNT"]
        pkg._lib.reload_debug_env()   # the library reads SBCE_* switches once
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        eng.estep()
        e0.record()
        for _ in range(5):
            eng.estep()
        e1.record()
        torch.cuda.synchronize()
        ms = e0.elapsed_time(e1) / 5
        del os.environ[k]
        pkg._lib.reload_debug_env()   # the library reads SBCE_* switches once
        print(f"after {it:2d} EM its  {arm:24s} single {sph[2] / nsym:6.3f} enum {sph[0] / nsym:6.3f} "
              f"listed {sph[1] / nsym:6.3f} "
              f"{cnt.value / nsym:7.2f} MFMA/symbol  E-step {ms:7.3f} ms", flush=True)
