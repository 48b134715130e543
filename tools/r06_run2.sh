#!/bin/bash
# round-6 GPU pass 2: small M-step tests, the small M-step A/B and the cfg5 grid
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "small or cfg5 or rank_deficient or root_td or detector_grid or workspace or sweeps" > gpurun_out/r06_t2.log 2>&1
rc=$?
echo "tests_rc=$rc" >> gpurun_out/r06_t2.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 120 python tools/ab_small.py 120 20 > gpurun_out/r06_ab_small2.log 2>&1 &&
timeout -k 10 120 python tools/ab_small.py 15 20 >> gpurun_out/r06_ab_small2.log 2>&1 &&
timeout -k 10 300 python bench.py --config cfg5 > gpurun_out/r06_cfg5b.log 2>&1
