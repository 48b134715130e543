#!/bin/bash
# cfg5 raw kernel trace (kept): per-launch durations and per-stream gaps of one grid step
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r06_c5t; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d "$O/trace" -o run -- python3 "$R/bench.py" \
    --config cfg5 --steps 1 --warmup 1 --no-cpu-baseline > "$O/trace.log" 2>&1 || exit $?
find "$O/trace" -name "*kernel_trace.csv" -exec cp {} "$O/kernel_trace.csv" \;
rm -rf "$O/trace"
