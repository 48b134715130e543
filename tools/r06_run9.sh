#!/bin/bash
# diag_inverse_rd with unconditional operand reads: Cholesky tests, cfg1 bench, kernel trace
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r06_r9; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_em.py -m gpu -x -q --timeout 120 --timeout-method thread -k "chol or cfg1 or rank_deficient or valu or workspace" > $O/tests.log 2>&1 || exit $?
timeout -k 10 300 python bench.py > $O/bench_cfg1.log 2>&1 || exit $?
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$O/trace" -o run -- python3 "$R/bench.py" \
    --steps 20 --warmup 3 --no-cpu-baseline > "$O/trace.log" 2>&1 || exit $?
python3 "$R/tools/trace_summary.py" "$O/trace" > "$O/kernel_stats_cfg1.csv"
rm -rf "$O/trace"
