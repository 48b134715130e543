"""Diagnostic: FP64 MFMAs the E-step sweep issues per symbol on the cfg1 batch (after EM has
run a few iterations), under alternating environment settings, e.g.
  python tools/estep_count.py SBCE_X=0 SBCE_ESTEP_ROWB=0"""
import ctypes
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402
import __graft_entry__ as ge  # noqa: E402

pkg = ge.package()
pkg._lib.use_ab()       # the A/B build: SBCE_* switches, counters, clocks
varn = float(pkg.signal_model.snr_to_varn(float(os.environ.get("SNR", "20"))))
batch = pkg.signal_model.synthetic_batch(1000, 4, 4, 64, 16, 256, 16, varn, seed=0)
eng = pkg.EMEngine(batch, varn)
lib = pkg._lib.load()
for it in (1, 5, 20):
    eng.run(it)
    for arm in sys.argv[1:] or ["SBCE_X=0"]:
        k, v = arm.split("=", 1)
        os.environ[k] = v
        os.environ["SBCE_ESTEP_COUNT"] = "1"
        pkg._lib.reload_debug_env()   # the library reads SBCE_* switches once
        cnt = ctypes.c_ulonglong(0)
        lib.sbce_debug_estep_mfma(None, 1)
        eng.estep()
        torch.cuda.synchronize()
        lib.sbce_debug_estep_mfma(ctypes.byref(cnt), 0)
        del os.environ["SBCE_ESTEP_COUNT"], os.environ[k]
        pkg._lib.reload_debug_env()   # the library reads SBCE_* switches once
        print(f"after {it:2d} EM its  {arm:24s} {cnt.value / (1000 * 256):8.2f} MFMA/symbol", flush=True)
