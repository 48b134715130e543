"""QAM constellation tables in the order of the reference's vendored ``komm``
QAModulation ("Proposed method/QAM.py":306-322): square M = L^2, base amplitude 1,
in-phase index fastest:  s -> (2*(s % L) - L + 1) + 1j*(2*(s // L) - L + 1).

This order fixes the hypothesis enumeration (``itertools.product`` over this
table, "Proposed method/Proposed_method_NMSEvsTp.py":32-38) and the symbol draws
(``qamCons[np.random.choice(range(M), n_tx, 'True')]``, :31).
"""
import numpy as np


def qam_constellation(M):
    L = int(round(np.sqrt(M)))
    if L * L != M or L & (L - 1):
        raise ValueError("M must be a square power of two (4, 16, 64, 256)")
    ci = np.arange(-L + 1, L, 2, dtype=np.int64).astype(float)
    cq = np.arange(-L + 1, L, 2, dtype=np.int64).astype(float)
    return (ci + 1j * cq[:, None]).reshape(-1)


def energy_per_symbol(M):
    """E_s = mean |s|^2 ("Proposed method/QAM.py":81): 2, 10, 42 for 4/16/64-QAM."""
    c = qam_constellation(M)
    return float(np.mean(c.real ** 2 + c.imag ** 2))


def all_possible_symbols(cons, n_tx):
    """J = M^n_tx hypotheses in itertools.product order (first stream slowest)."""
    cons = np.asarray(cons)
    M = cons.size
    idx = np.indices((M,) * n_tx).reshape(n_tx, -1).T
    return cons[idx]
