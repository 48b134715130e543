#!/bin/bash
# SQ counters of the cfg5 phase launches (tools/ab_cfg5_phases.py at T_d = 120), two passes:
# instruction mix, then wave cycles / waits.  bash tools/sq_cfg5.sh <tag>
set -e
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${1:-sq_cfg5}
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_BRANCH SQ_INSTS_SMEM -d $O/p1 -o run -- python3 $R/tools/ab_cfg5_phases.py 120 > $O/p1.log 2>&1
python3 $R/tools/pmc_sq.py $O/p1 > $O/insts.txt
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE -d $O/p2 -o run -- python3 $R/tools/ab_cfg5_phases.py 120 > $O/p2.log 2>&1
python3 $R/tools/pmc_sq.py $O/p2 > $O/waits.txt
rm -rf $O/p1 $O/p2
