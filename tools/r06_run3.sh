#!/bin/bash
# small M-step: targeted tests, the A/B and the solve clocks
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "small or cfg5 or rank_deficient or detector_grid or workspace" > gpurun_out/r06_t3.log 2>&1
rc=$?
echo "tests_rc=$rc" >> gpurun_out/r06_t3.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 120 python tools/ab_small.py 120 20 > gpurun_out/r06_ab_small3.log 2>&1 &&
timeout -k 10 120 python tools/ab_small.py 15 20 >> gpurun_out/r06_ab_small3.log 2>&1 &&
timeout -k 10 120 python tools/small_clock.py 120 > gpurun_out/r06_clk.log 2>&1
