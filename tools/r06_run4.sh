#!/bin/bash
# full GPU suite + smoke, then the cfg1 and cfg5 bench lines
timeout -k 10 420 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r06_t4.log 2>&1
rc=$?
echo "tests_rc=$rc" >> gpurun_out/r06_t4.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r06_smoke.log 2>&1 &&
timeout -k 10 200 python bench.py > gpurun_out/r06_b4.log 2>&1 &&
timeout -k 10 300 python bench.py --config cfg5 > gpurun_out/r06_cfg5_4.log 2>&1
