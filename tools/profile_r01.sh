#!/bin/bash
# Round profile: bench line, kernel-trace stats, and two separate PMC passes
# (FETCH_SIZE, WRITE_SIZE) of the same bench command.  Run from the repo root
# on the GPU box:  gpurun -- bash tools/profile_r01.sh <tag>
set -e
TAG=${1:-r01}
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$TAG
mkdir -p "$O"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 python3 "$R/bench.py" --steps 3 --warmup 1 > "$O/bench.log" 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$O/trace" -o run -- \
    python3 "$R/bench.py" --steps 2 --warmup 1 --no-cpu-baseline > "$O/trace.log" 2>&1
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -d "$O/pmc_fetch" -o run -- \
    python3 "$R/bench.py" --steps 1 --warmup 0 --iters 2 --kernel-reps 2 --no-cpu-baseline > "$O/pmc_fetch.log" 2>&1
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE -d "$O/pmc_write" -o run -- \
    python3 "$R/bench.py" --steps 1 --warmup 0 --iters 2 --kernel-reps 2 --no-cpu-baseline > "$O/pmc_write.log" 2>&1
echo done
