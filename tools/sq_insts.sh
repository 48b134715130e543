set -e
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_BRANCH SQ_INSTS_SMEM -d $R/gpurun_out/sqi1 -o run -- python3 $R/tools/estep_only.py > $R/gpurun_out/sqi1.log 2>&1
python3 $R/tools/pmc_sq.py $R/gpurun_out/sqi1
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_TRANS_F64 SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_CVT SQ_INSTS_VMEM_WR -d $R/gpurun_out/sqi2 -o run -- python3 $R/tools/estep_only.py > $R/gpurun_out/sqi2.log 2>&1
python3 $R/tools/pmc_sq.py $R/gpurun_out/sqi2
