#!/bin/bash
# Round-end verification on the GPU box (run from the repo root):
#   bash tools/final_round.sh <tag>
# the whole -m gpu suite, smoke(), then the cfg1 PMC passes + bench line + kernel trace
# (as tools/profile_round.sh does for cfg1) and the cfg5 profile (tools/profile_cfg5.sh).
# Every GPU step has its own time limit; the script stops at the first failure.
set -e
TAG=${1:-final}
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$TAG
mkdir -p "$O"
timeout -k 10 900 python3 -u -m pytest -x -q --timeout 200 --timeout-method thread "$R/tests" -m gpu \
    > "$O/gpu_tests.log" 2>&1
timeout -k 10 300 python3 -c "import sys; sys.path.insert(0, '$R'); import __graft_entry__ as g; g.smoke(); print('smoke ok')" \
    > "$O/smoke.log" 2>&1
cd /tmp && export TMPDIR=/tmp
PM="--config cfg1 --steps 1 --warmup 0 --iters 2 --kernel-reps 2 --streams 1"
timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE -d "$O/pmc_fetch_cfg1" -o run -- \
    python3 "$R/bench.py" $PM --no-cpu-baseline > "$O/pmc_fetch_cfg1.log" 2>&1
timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE -d "$O/pmc_write_cfg1" -o run -- \
    python3 "$R/bench.py" $PM --no-cpu-baseline > "$O/pmc_write_cfg1.log" 2>&1
python3 "$R/tools/pmc_summary.py" --fetch "$O/pmc_fetch_cfg1" --write "$O/pmc_write_cfg1" \
    --config cfg1 --trials 1000 --out "$O/pmc_cfg1.json" > /dev/null
rm -rf "$O/pmc_fetch_cfg1" "$O/pmc_write_cfg1"
timeout -k 10 400 python3 "$R/bench.py" --config cfg1 --steps 3 --warmup 1 --pmc "$O/pmc_cfg1.json" \
    > "$O/bench_cfg1.log" 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$O/trace_cfg1" -o run -- \
    python3 "$R/bench.py" --config cfg1 --steps 2 --warmup 1 --no-cpu-baseline > "$O/trace_cfg1.log" 2>&1
python3 "$R/tools/trace_summary.py" "$O/trace_cfg1" > "$O/kernel_stats_cfg1.csv"
rm -rf "$O/trace_cfg1"
cd "$R"
bash "$R/tools/profile_cfg5.sh" "$TAG"
echo done
