#!/bin/bash
# E-step record traffic check on the GPU box (run from the repo root):
#   bash tools/tree_traffic.sh <tag>
# the E-step GPU tests, then separate FETCH_SIZE / WRITE_SIZE PMC passes over a whole-batch
# (--streams 1) cfg1 run -> gpurun_out/<tag>/pmc_cfg1.json, and the cfg1 bench line.
set -e
TAG=${1:-tree}
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$TAG
mkdir -p "$O"
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 200 --timeout-method thread \
    "$R/tests/test_gpu_em.py" "$R/tests/test_gpu_estep_pair.py" -m gpu > "$O/tests.log" 2>&1
cd /tmp && export TMPDIR=/tmp
PM="--config cfg1 --steps 1 --warmup 0 --iters 2 --kernel-reps 2 --streams 1"
timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE -d "$O/pmc_fetch" -o run -- \
    python3 "$R/bench.py" $PM --no-cpu-baseline > "$O/pmc_fetch.log" 2>&1
timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE -d "$O/pmc_write" -o run -- \
    python3 "$R/bench.py" $PM --no-cpu-baseline > "$O/pmc_write.log" 2>&1
python3 "$R/tools/pmc_summary.py" --fetch "$O/pmc_fetch" --write "$O/pmc_write" \
    --config cfg1 --trials 1000 --out "$O/pmc_cfg1.json" > "$O/pmc_summary.txt"
rm -rf "$O/pmc_fetch" "$O/pmc_write"
timeout -k 10 400 python3 "$R/bench.py" --config cfg1 --steps 3 --warmup 1 --pmc "$O/pmc_cfg1.json" \
    --no-cpu-baseline > "$O/bench_cfg1.log" 2>&1
echo done
