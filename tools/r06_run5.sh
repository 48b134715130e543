#!/bin/bash
timeout -k 10 420 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r06_t5.log 2>&1
rc=$?
echo "tests_rc=$rc" >> gpurun_out/r06_t5.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python bench.py --config cfg5 > gpurun_out/r06_cfg5_5.log 2>&1 &&
timeout -k 10 600 bash tools/sq_issued.sh r06_sq
