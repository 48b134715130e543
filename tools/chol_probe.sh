#!/bin/bash
# Cholesky diagnostics on the GPU box (run from the repo root):  bash tools/chol_probe.sh <tag>
# One SQ counter pass (wave-cycle split, MFMA busy, instruction counts) and one kernel trace of
# a single-stream cfg1 run; summaries to gpurun_out/<tag>/ (raw databases removed).
set -e
TAG=${1:-probe}
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$TAG
mkdir -p "$O"
cd /tmp && export TMPDIR=/tmp
B="$R/bench.py --steps 1 --warmup 0 --iters 3 --kernel-reps 1 --no-cpu-baseline --streams 1"
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY \
    SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_INSTS_VALU SQ_INSTS_LDS GRBM_GUI_ACTIVE \
    -d "$O/sq" -o run -- python3 $B > "$O/sq.log" 2>&1
python3 "$R/tools/pmc_sq.py" "$O/sq" > "$O/sq.txt"
rm -rf "$O/sq"
timeout -k 10 120 rocprofv3 --kernel-trace -d "$O/tr" -o run -- python3 $B > "$O/tr.log" 2>&1
python3 "$R/tools/trace_seq.py" "$O/tr" "" --last 120 > "$O/seq.txt"
rm -rf "$O/tr"
echo probe done
