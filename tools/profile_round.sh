#!/bin/bash
# Round profile on the GPU box (run from the repo root):
#   bash tools/profile_round.sh <tag>
# Per workload (cfg1: the default bench line; cfg2: BASELINE configs[2] at 256 trials):
#   separate FETCH_SIZE / WRITE_SIZE PMC passes -> gpurun_out/<tag>/pmc_<cfg>.json
#   (tools/pmc_summary.py; bench.py --pmc reads it for roofline.traffic),
#   the bench line itself, and a kernel-trace --stats run of the same command.
# Every GPU step has its own time limit; the script stops at the first failure.
# The PMC passes run cfg1 with --streams 1 (whole-batch launches only: per-launch bytes of the
# launches bench.py's roofline times); the bench line and the kernel trace use the default
# schedule (four stream sub-batches at cfg1; tools/trace_summary.py keeps one row per grid).
set -e
TAG=${1:-r01}
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$TAG
mkdir -p "$O"
cd /tmp && export TMPDIR=/tmp

C1="--config cfg1"
C2="--config cfg2 --trials 256 --iters 2"
for W in cfg1 cfg2; do
    if [ $W = cfg1 ]; then C=$C1; PM="$C1 --steps 1 --warmup 0 --iters 2 --kernel-reps 2 --streams 1";
    else C=$C2; PM="--config cfg2 --trials 256 --iters 1 --steps 1 --warmup 0 --kernel-reps 1"; fi
    timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE -d "$O/pmc_fetch_$W" -o run -- \
        python3 "$R/bench.py" $PM --no-cpu-baseline > "$O/pmc_fetch_$W.log" 2>&1
    timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE -d "$O/pmc_write_$W" -o run -- \
        python3 "$R/bench.py" $PM --no-cpu-baseline > "$O/pmc_write_$W.log" 2>&1
    TR=$([ $W = cfg1 ] && echo 1000 || echo 256)
    python3 "$R/tools/pmc_summary.py" --fetch "$O/pmc_fetch_$W" --write "$O/pmc_write_$W" \
        --config $W --trials $TR --out "$O/pmc_$W.json" > /dev/null
    rm -rf "$O/pmc_fetch_$W" "$O/pmc_write_$W"     # raw databases: gpurun_out/ must stay < 64 MiB
    if [ $W = cfg1 ]; then
        timeout -k 10 400 python3 "$R/bench.py" $C --steps 3 --warmup 1 --pmc "$O/pmc_$W.json" \
            > "$O/bench_$W.log" 2>&1
        timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$O/trace_$W" -o run -- \
            python3 "$R/bench.py" $C --steps 2 --warmup 1 --no-cpu-baseline > "$O/trace_$W.log" 2>&1
    else
        timeout -k 10 400 python3 "$R/bench.py" $C --steps 1 --warmup 1 --kernel-reps 1 \
            --pmc "$O/pmc_$W.json" > "$O/bench_$W.log" 2>&1
        timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$O/trace_$W" -o run -- \
            python3 "$R/bench.py" $C --steps 1 --warmup 1 --kernel-reps 1 --no-cpu-baseline \
            > "$O/trace_$W.log" 2>&1
    fi
    python3 "$R/tools/trace_summary.py" "$O/trace_$W" > "$O/kernel_stats_$W.csv"
    rm -rf "$O/trace_$W"
done
echo done
