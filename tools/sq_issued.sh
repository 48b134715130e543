#!/bin/bash
# Issued FP64 work of the E-step launches bench.py prices (cfg1 steady state; cfg5's soft E-step at
# T_d = 120): one SQ PMC pass each -> gpurun_out/<tag>/sq_<cfg>.json (tools/sq_issued.py)
set -e
TAG=${1:-r06_sq}
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$TAG
mkdir -p "$O"
cd /tmp && export TMPDIR=/tmp
CTR="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_TRANS_F64 SQ_INSTS_VALU_MFMA_MOPS_F64 SQ_INSTS_MFMA"
for W in cfg1 cfg5; do
    timeout -s KILL 240 rocprofv3 --pmc $CTR -d "$O/pmc_$W" -o run -- python3 "$R/tools/sq_drive.py" $W 3 > "$O/pmc_$W.log" 2>&1
    TR=$([ $W = cfg1 ] && echo 1000 || echo 1280)
    python3 "$R/tools/sq_issued.py" "$O/pmc_$W" --config $W --trials $TR --reps 3 --out "$O/sq_$W.json" > "$O/sq_$W.txt"
    rm -rf "$O/pmc_$W"
done
echo done
