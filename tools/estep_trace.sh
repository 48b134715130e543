#!/bin/bash
# cfg1 kernel trace (--stats) of a short bench run: per-kernel E-step durations
#   bash tools/estep_trace.sh <tag>
set -e
TAG=${1:-etrace}
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$TAG
mkdir -p "$O"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$O/trace" -o run -- \
    python3 "$R/bench.py" --config cfg1 --steps 2 --warmup 1 --no-cpu-baseline --streams 1 > "$O/trace.log" 2>&1
python3 "$R/tools/trace_summary.py" "$O/trace" > "$O/kernel_stats_cfg1.csv"
rm -rf "$O/trace"
timeout -k 10 300 python3 "$R/bench.py" --config cfg1 --steps 3 --warmup 1 --no-cpu-baseline > "$O/bench_cfg1.log" 2>&1
echo done
