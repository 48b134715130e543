"""Diagnostic: the cfg1 batch (1000 trials x 20 EM iterations) as K independent sub-batches,
each its own EMEngine on its own HIP stream (trials are independent), against one engine.
  python tools/stream_split.py 1 2 4 8"""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402
import __graft_entry__ as ge  # noqa: E402

pkg = ge.package()
B = int(os.environ.get("B", "1000"))
varn = float(pkg.signal_model.snr_to_varn(20.0))
batch = pkg.signal_model.synthetic_batch(B, 4, 4, 64, 16, 256, 16, varn, seed=0)
ref = None
for k in [int(x) for x in sys.argv[1:]] or [1, 2, 4]:
    bounds = np.linspace(0, B, k + 1).astype(int)
    engs = []
    for i in range(k):
        sub = {key: (v[bounds[i]:bounds[i + 1]] if isinstance(v, np.ndarray) and v.ndim > 1
                     and v.shape[0] == B else v) for key, v in batch.items()}
        engs.append(pkg.EMEngine(sub, varn))
    streams = [torch.cuda.Stream() for _ in range(k)]
    main = torch.cuda.current_stream()

    def step():
        ev = torch.cuda.Event()
        ev.record(main)
        for e, s in zip(engs, streams):
            s.wait_event(ev)
            with torch.cuda.stream(s):
                e.run(20)
        for s in streams:
            main.wait_stream(s)

    step()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(3):
        step()
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / 3
    th = torch.cat([e.theta for e in engs]).cpu().numpy()
    if ref is None:
        ref = th
    print(f"K={k}: {dt * 1e3:8.2f} ms per 20-iteration run  {B * 20 / dt:10.0f} EM-it/s  "
          f"max|dtheta| vs K=first {np.abs(th - ref).max():.1e}", flush=True)
