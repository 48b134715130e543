#!/bin/bash
# BASELINE cfg 5 (the SNR x T_d grid, five EMs) on the GPU box:
#   bash tools/profile_cfg5.sh <tag>
# the bench line, a kernel-trace --stats run of the same command (-> kernel_stats_cfg5.csv) and
# separate FETCH_SIZE / WRITE_SIZE PMC passes over the roofline launches alone
# (bench.py --roofline-only) -> pmc_cfg5.json.  Every GPU step has its own time limit.
set -e
TAG=${1:-r05_cfg5}
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$TAG
mkdir -p "$O"
cd /tmp && export TMPDIR=/tmp
C="--config cfg5"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$O/trace_cfg5" -o run -- \
    python3 "$R/bench.py" $C --steps 2 --warmup 1 --no-cpu-baseline > "$O/trace_cfg5.log" 2>&1
python3 "$R/tools/trace_summary.py" "$O/trace_cfg5" > "$O/kernel_stats_cfg5.csv"
python3 "$R/tools/trace_timeline.py" "$O/trace_cfg5" --last-frac 0.5 > "$O/timeline_cfg5.txt"
rm -rf "$O/trace_cfg5"
if [ "${PMC:-1}" = 1 ]; then
    timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE -d "$O/pmc_fetch_cfg5" -o run -- \
        python3 "$R/bench.py" $C --roofline-only --kernel-reps 2 > "$O/pmc_fetch_cfg5.log" 2>&1
    timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE -d "$O/pmc_write_cfg5" -o run -- \
        python3 "$R/bench.py" $C --roofline-only --kernel-reps 2 > "$O/pmc_write_cfg5.log" 2>&1
    python3 "$R/tools/pmc_summary.py" --fetch "$O/pmc_fetch_cfg5" --write "$O/pmc_write_cfg5" \
        --config cfg5 --trials 1280 --out "$O/pmc_cfg5.json" > /dev/null
    rm -rf "$O/pmc_fetch_cfg5" "$O/pmc_write_cfg5"
    timeout -k 10 300 python3 "$R/bench.py" $C --steps 3 --warmup 1 --pmc "$O/pmc_cfg5.json" \
        > "$O/bench_cfg5.log" 2>&1
fi
echo done
