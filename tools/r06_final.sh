#!/bin/bash
# round-6 closing run: full GPU suite, smoke, cfg1 bench (the driver's default line), cfg5 kernel
# trace + timeline, cfg5 bench; every GPU step under its own limit, stop at the first failure
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r06_final; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || exit $?
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || exit $?
timeout -k 10 300 python bench.py > $O/bench_cfg1.log 2>&1 || exit $?
PMC=0 bash tools/profile_cfg5.sh r06_final_cfg5 > $O/profile_cfg5.log 2>&1 || exit $?
timeout -k 10 300 python bench.py --config cfg5 > $O/bench_cfg5.log 2>&1
