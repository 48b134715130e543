#!/bin/bash
# Large-L workloads with the min-norm (lstsq) solve on the GPU box:
#   bash tools/profile_large.sh <tag>
# cfg2 (256 trials, 2 EM iterations) and cfg4 (32 trials, 1 iteration): the bench line and a
# kernel-trace --stats run -> gpurun_out/<tag>/.
set -e
TAG=${1:-r03_large}
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$TAG
mkdir -p "$O"
cd /tmp && export TMPDIR=/tmp
for W in cfg2 cfg4; do
    if [ $W = cfg2 ]; then C="--config cfg2 --trials 256 --iters 2"; else C="--config cfg4 --trials 32 --iters 1"; fi
    timeout -k 10 400 python3 "$R/bench.py" $C --steps 1 --warmup 1 --kernel-reps 1 \
        --no-cpu-baseline > "$O/bench_$W.log" 2>&1
    timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$O/trace_$W" -o run -- \
        python3 "$R/bench.py" $C --steps 1 --warmup 0 --kernel-reps 1 --no-cpu-baseline \
        > "$O/trace_$W.log" 2>&1
    python3 "$R/tools/trace_summary.py" "$O/trace_$W" > "$O/kernel_stats_$W.csv"
    rm -rf "$O/trace_$W"
done
echo done
