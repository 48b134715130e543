"""CPU oracle for the EM semi-blind channel estimator — TEST INFRASTRUCTURE ONLY.

Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline``
leg may import anything under ``oracle/``, and only as the checker (or the timed
CPU baseline), never as a product code path.  The product package fails loudly
when its HIP library is missing; it never falls back to this module.

Parity pinning: both faces of the oracle are checked against golden fixtures
produced by running the reference's own ``em`` functions in the CPU container
(``tests/golden/make_golden.py``; SURVEY.md §8c known-answer values).

Two faces:
  * ``em_loop``    — reference-structured restatement: per symbol, per hypothesis,
                     dense Kronecker regressor Z, float64 log-sum-exp in place of
                     the reference's arbitrary-exponent mpmath/gmpy2 ``exp``.
  * ``em_reduced`` — the reduced form the GPU implements: per-symbol posterior
                     moments + one L x L Hermitian system per trial (commutation
                     identity, SURVEY.md §8 preamble).
"""
from .em_loop import em_loop, em_ml_loop, llf_genie  # noqa: F401
from .em_reduced import (  # noqa: F401
    heff, estep_moments, mstep_build, mstep_solve, em_reduced, nmse,
)
