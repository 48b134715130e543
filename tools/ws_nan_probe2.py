"""Diagnostic: sbce_mstep (build + solve) at L = 600 from fixed moments in a workspace pre-filled
with 0x00 and with 0xFF: are R's lower triangle / B^H (copied before the solve) and theta equal
and finite?  Narrows a stale-workspace read to the build or the tiled factorisation."""
import sys
import numpy as np
import torch

sys.path.insert(0, ".")
import __graft_entry__ as ge  # noqa: E402

pkg = ge.package()
pkg._lib.use_ab()       # the A/B build: SBCE_* switches, counters, clocks
L_ = pkg._lib
n_tx, n_rx, N, T_p, T_d, M = 4, 4, 149, 16, 200, 16
solve = sys.argv[1] if len(sys.argv) > 1 else "chol"
varn = float(pkg.signal_model.snr_to_varn(20.0))
b = pkg.signal_model.synthetic_batch(2, n_tx, n_rx, N, T_p, T_d, M, varn, seed=11)
x = b["x_d"]
mom = np.concatenate([x, (x[..., :, None] * np.conj(x[..., None, :])).reshape(2, T_d, -1)], axis=2)
dev = lambda a: torch.from_numpy(np.ascontiguousarray(a, dtype=np.complex128)).cuda()
Yd, Yp, Ps, Up, Cs, Mo = (dev(b["y_d"]), dev(b["y_p"]), dev(b["psi_d"]), dev(b["u_p"]), dev(b["cons"]),
                          dev(mom))
P, L = N + 1, (N + 1) * n_tx
dims = L_.Dims(2, n_tx, n_rx, P, T_p, T_d, M, 0, varn, 1.0)
solve_id = {"chol": L_.SBCE_SOLVE_CHOL, "drop": L_.SBCE_SOLVE_CHOL_DROP, "lstsq": L_.SBCE_SOLVE_MINNORM}[solve]
nbytes = L_.workspace_bytes(dims, solve_id)
res = {}
for fill in (0x00, 0xFF):
    ws = torch.empty(nbytes, dtype=torch.uint8, device="cuda")
    ws.fill_(fill)
    th = torch.zeros((2, L * n_rx), dtype=torch.complex128, device="cuda")
    st = torch.zeros(2, dtype=torch.int32, device="cuda")
    Rout = torch.zeros((2, L, L), dtype=torch.complex128, device="cuda")
    rhs = torch.zeros((2, L, n_rx), dtype=torch.complex128, device="cuda")
    p = L_.Ptrs(Yd.data_ptr(), Yp.data_ptr(), Ps.data_ptr(), Up.data_ptr(), Cs.data_ptr(), th.data_ptr(),
                None, None, None, None, st.data_ptr(), ws.data_ptr(), ws.numel(), None, None, None)
    L_.check(L_.load().sbce_mstep(dims, p, Mo.data_ptr(), solve_id, Rout.data_ptr(), rhs.data_ptr(),
                                  torch.cuda.current_stream().cuda_stream), "sbce_mstep")
    torch.cuda.synchronize()
    R = Rout.cpu().numpy()
    lo = np.tril_indices(L)
    res[fill] = (R[:, lo[0], lo[1]], rhs.cpu().numpy(), th.cpu().numpy(), st.cpu().numpy())
    bad = ~np.isfinite(th.cpu().numpy())
    print(f"fill {fill:#x}: R lower finite {np.isfinite(res[fill][0]).all()} rhs finite "
          f"{np.isfinite(res[fill][1]).all()} theta finite {np.isfinite(res[fill][2]).all()} "
          f"(nonfinite entries {bad.sum()}, first {np.argwhere(bad)[:3].tolist()}) status {res[fill][3]}")
print("R lower equal", np.array_equal(res[0][0], res[0xFF][0]), "rhs equal",
      np.array_equal(res[0][1], res[0xFF][1]), "theta equal", np.array_equal(res[0][2], res[0xFF][2]))
