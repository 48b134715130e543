#!/bin/bash
# product / A/B library split + back-substitution prefetch: full GPU suite, smoke, cfg1 + cfg5 bench,
# the small M-step A/B and solve clocks
O=gpurun_out/r06_r7; mkdir -p $O
timeout -k 10 480 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || exit $?
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 &&
timeout -k 10 300 python bench.py > $O/bench_cfg1.log 2>&1 &&
timeout -k 10 300 python bench.py --config cfg5 > $O/bench_cfg5.log 2>&1 &&
timeout -k 10 180 python tools/ab_small.py 120 > $O/ab120.log 2>&1 &&
timeout -k 10 120 python tools/small_clock.py 120 > $O/clock.log 2>&1
