#!/bin/bash
# E-step cost across the NMSE-vs-SNR range, on the GPU box:
#   bash tools/profile_snr.sh <tag> [snr ...]
# Per SNR: the cfg1 bench line (E-step / M-step times, sphere-pass resolution) and a
# kernel-trace --stats run of the same command -> gpurun_out/<tag>/.
set -e
TAG=${1:-r03_snr}
shift || true
SNRS=${@:-"10 0 -5"}
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$TAG
mkdir -p "$O"
cd /tmp && export TMPDIR=/tmp
for S in $SNRS; do
    timeout -k 10 300 python3 "$R/bench.py" --config cfg1 --snr "$S" --steps 2 --warmup 1 \
        --no-cpu-baseline > "$O/bench_cfg1_snr$S.log" 2>&1
    timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$O/trace_snr$S" -o run -- \
        python3 "$R/bench.py" --config cfg1 --snr "$S" --steps 1 --warmup 1 --no-cpu-baseline \
        > "$O/trace_snr$S.log" 2>&1
    python3 "$R/tools/trace_summary.py" "$O/trace_snr$S" > "$O/kernel_stats_cfg1_snr$S.csv"
    rm -rf "$O/trace_snr$S"
done
echo done
