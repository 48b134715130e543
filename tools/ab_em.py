"""Diagnostic A/B: whole-EM time (20 iterations, cfg1, 1000 trials) under alternating
environment settings in ONE process, e.g.  python tools/ab_em.py SBCE_EM_STREAMS=1 SBCE_EM_STREAMS=2"""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402
import __graft_entry__ as ge  # noqa: E402

pkg = ge.package()
pkg._lib.use_ab()       # the A/B build: SBCE_* switches, counters, clocks
varn = float(pkg.signal_model.snr_to_varn(20.0))
batch = pkg.signal_model.synthetic_batch(1000, 4, 4, 64, 16, 256, 16, varn, seed=0)
eng = pkg.EMEngine(batch, varn)
eng.run(20)
torch.cuda.synchronize()
for rnd in range(3):
    for arm in sys.argv[1:]:
        k, v = arm.split("=", 1)
        os.environ[k] = v
        pkg._lib.reload_debug_env()   # the library reads SBCE_* switches once
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(2):
            eng.run(20)
        torch.cuda.synchronize()
        dt = (time.perf_counter() - t0) / 2
        nm = float(eng.nmse().mean())
        print(f"round {rnd} {arm:24s} {dt * 1e3:8.2f} ms/run  {20000 / dt:9.0f} EM-it/s  nmse {nm:.12f}",
              flush=True)
        del os.environ[k]
        pkg._lib.reload_debug_env()   # the library reads SBCE_* switches once
