"""Diagnostic (CPU, NumPy): the breadth-first sphere enumeration's path counts per level at the
cfg1 iteration-0 E-step (theta_0 from the pilots alone, 20 dB), for the kernel's radius
(Babai point + 50 varn^2) and for the tightest valid radius (the ML distance + 50 varn^2),
on 128 symbols of two trials.  Shows why the iteration-0 symbols reach the MFMA sweep: even at
the tight radius two thirds of them hold > 128 paths at some level, although the posterior
keeps one hypothesis.  Not part of the product."""
import sys, itertools, numpy as np
sys.path.insert(0, __import__('os').path.dirname(__import__('os').path.dirname(__import__('os').path.abspath(__file__))))
import __graft_entry__ as ge
pkg = ge.package()
varn = float(pkg.signal_model.snr_to_varn(20.0))
b = pkg.signal_model.synthetic_batch(4, 4, 4, 64, 16, 256, 16, varn, seed=0)
cons = b['cons']; M = 16; NT = 4; P = b['P']
s2 = varn**2; thr = 50 * s2; reg = 0.1 * s2
cm2 = np.max(np.abs(cons)**2); slack = reg * cm2
allx = np.array(list(itertools.product(range(M), repeat=NT)))
stats = []
for tr in range(2):
    Hc = b['theta0'][tr].reshape(P, NT, 4)        # [p][a][r]
    for t in range(0, 256, 4):
        H = np.einsum('p,par->ra', b['psi_d'][tr, t], Hc)   # n_rx x n_tx
        y = b['y_d'][tr, t]
        d = np.sum(np.abs(y[None, :] - cons[allx] @ H.T)**2, axis=1)
        dstar = d.min()
        Ginv = np.linalg.inv(H.conj().T @ H + reg * np.eye(NT))
        g = np.real(np.diag(Ginv))
        lev = np.array([np.sum((g > g[q]) | ((g == g[q]) & (np.arange(NT) < q))) for q in range(NT)])
        perm = np.argsort(lev)      # perm[l] = stream at level l
        Hp = H[:, perm]
        Gp = Hp.conj().T @ Hp + reg * np.eye(NT)
        Lm = np.linalg.cholesky(Gp)
        zf = np.linalg.solve(Lm, Hp.conj().T @ y)
        c0 = np.sum(np.abs(y)**2) - np.sum(np.abs(zf)**2)
        # Babai
        xb = np.zeros(NT, complex); db = 0
        for l in range(NT - 1, -1, -1):
            e = zf[l] - sum(np.conj(Lm[j, l]) * xb[j] for j in range(l + 1, NT))
            T = np.abs(Lm[l, l] * cons - e)**2 - reg * np.abs(cons)**2
            k = np.argmin(T); xb[l] = cons[k]; db += T[k]
        R0 = db
        res = []
        for Rrel in (R0 + thr, dstar - c0 + thr):
            paths = [((), 0.0)]
            counts = []
            for l in range(NT - 1, -1, -1):
                newp = []
                for (xs, pb) in paths:
                    xfull = dict(zip(range(NT - 1, l, -1), xs))
                    e = zf[l] - sum(np.conj(Lm[j, l]) * xfull[j] for j in range(l + 1, NT))
                    T = np.abs(Lm[l, l] * cons - e)**2 - reg * np.abs(cons)**2
                    for k in np.nonzero(pb + T <= Rrel + l * slack)[0]:
                        newp.append((xs + (cons[k],), pb + T[k]))
                paths = newp
                counts.append(len(paths))
                if len(paths) > 5000: counts.append(-1); break
            res.append(counts)
        nin = np.sum(d <= dstar + thr)
        stats.append((res[0], res[1], nin, (db + c0 - dstar) / s2))
for s in stats[:40]:
    print(s)
mx = lambda c: max(c) if -1 not in c else 99999
print("loose radius: frac max-level > 128:", np.mean([mx(s[0]) > 128 for s in stats]))
print("tight radius: frac max-level > 128:", np.mean([mx(s[1]) > 128 for s in stats]))
print("median (R0 - d*)/varn^2", np.median([s[3] for s in stats]))
