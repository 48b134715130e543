"""Diagnostic: trials of the bench's cfg5 grid whose EM result is not finite.  For each T_d of the
grid (64 trials per SNR point, the bench's seeds, all SNR points in one call per detector), every
detector: count of non-finite theta, and for the first such trial its (SNR, status, iterations) and
the per-iteration theta norms; its inputs are saved to gpurun_out/cfg5_nan_trial.npz."""
import json
import sys
import numpy as np

sys.path.insert(0, ".")
import __graft_entry__ as ge  # noqa: E402
import bench  # noqa: E402

pkg = ge.package()
g = bench.GRID["cfg5"]
varns = [float(v) for v in pkg.signal_model.snr_to_varn(g["SNR"], g["power"])]
saved = False
PINV = sys.argv[1] if len(sys.argv) > 1 else "scipy"
for k, td in enumerate(g["T_d"]):
    pts = [pkg.signal_model.synthetic_batch(64, 2, 2, 15, 20, td, 64, vn, pinv=PINV, seed=(0 * 1000003 + 0) * 1000 + k * 50 + j)
           for j, vn in enumerate(varns)]
    b = {key: np.concatenate([p[key] for p in pts]) for key in ("y_d", "y_p", "psi_d", "u_p", "theta0", "h")}
    vt = np.repeat(np.asarray(varns), 64)
    for det in g["detectors"]:
        r = pkg.em_batch(b["y_d"], b["y_p"], b["psi_d"], b["u_p"], pts[0]["cons"], vt, 5, b["theta0"],
                         mode=det, partition_r=1 if det == "pm_soft" else 0, h_true=b["h"])
        bad = np.where(~np.isfinite(r["theta"]).all(axis=1))[0]
        flagged = np.where(r["status"] != 0)[0]
        print(json.dumps({"T_d": td, "det": det, "nonfinite": len(bad), "flagged": len(flagged),
                          "flagged_status": sorted(set(int(s) for s in r["status"][flagged])),
                          "bad_snr": sorted(set(float(g["SNR"][i // 64]) for i in bad))}), flush=True)
        if len(bad) and not saved:
            i = int(bad[0])
            norms = []
            for it in range(1, 6):
                ri = pkg.em_batch(b["y_d"][i:i + 1], b["y_p"][i:i + 1], b["psi_d"][i:i + 1],
                                  b["u_p"][i:i + 1], pts[0]["cons"], vt[i], it, b["theta0"][i:i + 1],
                                  mode=det, h_true=b["h"][i:i + 1])
                norms.append([float(np.linalg.norm(ri["theta"][0])), int(ri["status"][0]),
                              int(ri["iters_done"][0])])
            print("first bad trial", i, "snr", g["SNR"][i // 64], "status", int(r["status"][i]),
                  "iters", int(r["iters_done"][i]), "per-iteration (norm, status, iters)", norms)
            np.savez("gpurun_out/cfg5_nan_trial.npz", **{kk: v[i] for kk, v in b.items()}, varn=vt[i],
                     T_d=td, det=det, cons=pts[0]["cons"])
            saved = True
