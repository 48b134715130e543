#!/bin/bash
# 4-column-panel MFMA small solve: targeted GPU tests, A/B timing, solve clocks, cfg5 bench
O=gpurun_out/r06_r8; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_em.py tests/test_gpu_sweeps.py -m gpu -x -q --timeout 120 --timeout-method thread -k "small or rank_deficient or cfg5 or root_td or captured or detector" > $O/tests.log 2>&1 || exit $?
timeout -k 10 180 python tools/ab_small.py 120 > $O/ab120.log 2>&1 &&
timeout -k 10 180 python tools/ab_small.py 15 > $O/ab15.log 2>&1 &&
timeout -k 10 120 python tools/small_clock.py 120 > $O/clock.log 2>&1 &&
timeout -k 10 300 python bench.py --config cfg5 > $O/bench_cfg5.log 2>&1
