#!/bin/bash
# BASELINE configs[2] (8x8, N_RIS = 256, PM_beta r = 1, min-norm solve): the bench line at
# BASELINE's 1250 trials x 5 iterations per GPU, PMC FETCH / WRITE passes and a kernel trace at
# 256 trials -> gpurun_out/<tag>/
set -e
TAG=${1:-r06_cfg2}
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$TAG
mkdir -p "$O"
cd /tmp && export TMPDIR=/tmp
PM="--config cfg2 --trials 256 --iters 1 --steps 1 --warmup 0 --kernel-reps 1 --no-cpu-baseline"
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE -d "$O/pmc_fetch" -o run -- python3 "$R/bench.py" $PM > "$O/pmc_fetch.log" 2>&1
timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE -d "$O/pmc_write" -o run -- python3 "$R/bench.py" $PM > "$O/pmc_write.log" 2>&1
python3 "$R/tools/pmc_summary.py" --fetch "$O/pmc_fetch" --write "$O/pmc_write" --config cfg2 --trials 256 \
    --out "$O/pmc_cfg2.json" > "$O/pmc_summary.txt"
rm -rf "$O/pmc_fetch" "$O/pmc_write"
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$O/trace" -o run -- python3 "$R/bench.py" \
    --config cfg2 --trials 256 --iters 2 --steps 1 --warmup 1 --kernel-reps 1 --no-cpu-baseline > "$O/trace.log" 2>&1
python3 "$R/tools/trace_summary.py" "$O/trace" > "$O/kernel_stats_cfg2.csv"
rm -rf "$O/trace"
timeout -k 10 600 python3 "$R/bench.py" --config cfg2 --steps 1 --warmup 1 --kernel-reps 1 \
    --pmc "$O/pmc_cfg2.json" > "$O/bench_cfg2_1250x5.log" 2>&1
echo done
