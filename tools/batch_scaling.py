"""Diagnostic: E-step and M-step time vs the number of trials per launch at the cfg1 shape
(flat time = latency-bound per trial, proportional = throughput-bound)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402
import __graft_entry__ as ge  # noqa: E402

pkg = ge.package()
varn = float(pkg.signal_model.snr_to_varn(20.0))


def timeit(fn, reps=10):
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps


for B in [int(x) for x in (sys.argv[1:] or ["250", "500", "1000", "2000"])]:
    batch = pkg.signal_model.synthetic_batch(B, 4, 4, 64, 16, 256, 16, varn, seed=0)
    eng = pkg.EMEngine(batch, varn)
    eng.run(2)
    eng.estep()
    torch.cuda.synchronize()
    print(f"B={B:5d}  estep {timeit(eng.estep):.3f} ms  mstep {timeit(eng.mstep):.3f} ms", flush=True)
    del eng, batch
    torch.cuda.empty_cache()
