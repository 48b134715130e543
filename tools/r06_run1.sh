#!/bin/bash
# round-6 GPU pass: tests (assertion failures do not stop the pass; a fault / abort / timeout does),
# the small M-step A/B, cfg1 and cfg5 benches
timeout -k 10 420 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r06_t1.log 2>&1
rc=$?
echo "tests_rc=$rc" >> gpurun_out/r06_t1.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 120 python tools/ab_small.py 120 20 > gpurun_out/r06_ab_small.log 2>&1 &&
timeout -k 10 120 python tools/ab_small.py 15 20 >> gpurun_out/r06_ab_small.log 2>&1 &&
timeout -k 10 200 python bench.py > gpurun_out/r06_b1.log 2>&1 &&
timeout -k 10 300 python bench.py --config cfg5 > gpurun_out/r06_cfg5.log 2>&1
