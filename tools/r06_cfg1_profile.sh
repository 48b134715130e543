#!/bin/bash
# cfg1 round profile (bench.py default line): FETCH / WRITE PMC passes (one stream: whole-batch
# launches), the bench line with that PMC, and a kernel-trace --stats run of the same command
set -e
TAG=${1:-r06_cfg1}
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$TAG
mkdir -p "$O"
cd /tmp && export TMPDIR=/tmp
PM="--config cfg1 --steps 1 --warmup 0 --iters 2 --kernel-reps 2 --streams 1 --no-cpu-baseline"
timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE -d "$O/pmc_fetch" -o run -- python3 "$R/bench.py" $PM > "$O/pmc_fetch.log" 2>&1
timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE -d "$O/pmc_write" -o run -- python3 "$R/bench.py" $PM > "$O/pmc_write.log" 2>&1
python3 "$R/tools/pmc_summary.py" --fetch "$O/pmc_fetch" --write "$O/pmc_write" --config cfg1 --trials 1000 \
    --out "$O/pmc_cfg1.json" > /dev/null
rm -rf "$O/pmc_fetch" "$O/pmc_write"
timeout -k 10 400 python3 "$R/bench.py" --steps 20 --warmup 3 --pmc "$O/pmc_cfg1.json" > "$O/bench_cfg1.log" 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$O/trace" -o run -- python3 "$R/bench.py" \
    --steps 20 --warmup 3 --no-cpu-baseline > "$O/trace.log" 2>&1
python3 "$R/tools/trace_summary.py" "$O/trace" > "$O/kernel_stats_cfg1.csv"
rm -rf "$O/trace"
echo done
