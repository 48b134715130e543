#!/bin/bash
# Round profile on the GPU box (run from the repo root):
#   bash tools/profile_round.sh <tag>
# cfg1: bench line, kernel-trace stats, separate FETCH_SIZE / WRITE_SIZE PMC passes;
# cfg2 (reduced trials): kernel-trace stats and PMC passes of the large-L M-step.
set -e
TAG=${1:-r01}
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$TAG
mkdir -p "$O"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 python3 "$R/bench.py" --steps 3 --warmup 1 > "$O/bench_cfg1.log" 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$O/trace_cfg1" -o run -- \
    python3 "$R/bench.py" --steps 2 --warmup 1 --no-cpu-baseline > "$O/trace_cfg1.log" 2>&1
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -d "$O/pmc_fetch_cfg1" -o run -- \
    python3 "$R/bench.py" --steps 1 --warmup 0 --iters 2 --kernel-reps 2 --no-cpu-baseline > "$O/pmc_fetch_cfg1.log" 2>&1
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE -d "$O/pmc_write_cfg1" -o run -- \
    python3 "$R/bench.py" --steps 1 --warmup 0 --iters 2 --kernel-reps 2 --no-cpu-baseline > "$O/pmc_write_cfg1.log" 2>&1
C2="--config cfg2 --trials 256 --iters 2 --steps 1 --warmup 1 --kernel-reps 1 --no-cpu-baseline"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$O/trace_cfg2" -o run -- \
    python3 "$R/bench.py" $C2 > "$O/trace_cfg2.log" 2>&1
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -d "$O/pmc_fetch_cfg2" -o run -- \
    python3 "$R/bench.py" --config cfg2 --trials 64 --iters 1 --steps 1 --warmup 0 --kernel-reps 1 --no-cpu-baseline > "$O/pmc_fetch_cfg2.log" 2>&1
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE -d "$O/pmc_write_cfg2" -o run -- \
    python3 "$R/bench.py" --config cfg2 --trials 64 --iters 1 --steps 1 --warmup 0 --kernel-reps 1 --no-cpu-baseline > "$O/pmc_write_cfg2.log" 2>&1
echo done
