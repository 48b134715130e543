# SQ counters of the iteration-0 E-step (tools/estep_it0.py) for the given SBCE_ESTEP_F32 values:
#   bash tools/sq_it0.sh [0 1]   (GPU box, repo root)
set -e
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
for F in ${@:-0 1}; do
  SBCE_ESTEP_F32=$F timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_MFMA GRBM_GUI_ACTIVE -d $R/gpurun_out/sqit0a_$F -o run -- python3 $R/tools/estep_it0.py > $R/gpurun_out/sqit0a_$F.log 2>&1
  python3 $R/tools/pmc_sq.py $R/gpurun_out/sqit0a_$F
  SBCE_ESTEP_F32=$F timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_BRANCH SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INST_CYCLES_SALU SQ_ACTIVE_INST_MISC -d $R/gpurun_out/sqit0b_$F -o run -- python3 $R/tools/estep_it0.py > $R/gpurun_out/sqit0b_$F.log 2>&1
  python3 $R/tools/pmc_sq.py $R/gpurun_out/sqit0b_$F
done
