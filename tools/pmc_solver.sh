#!/bin/bash
# rocprofv3 counter passes over one dev-library solve launch (tools/solve_probe.py).
set -o pipefail
export TMPDIR=/tmp
LIB=${1:-libkmpc_dev_v2.so}
OUT=gpurun_out/pmc_${LIB%.so}
mkdir -p $OUT
P="python3 tools/solve_probe.py 16384"
export KMPC_DEV_LIB=$LIB REPS=1
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_INSTS_VMEM SQ_INSTS_BRANCH SQ_WAVE_CYCLES -d $OUT/a -o run -- $P > $OUT/a.log 2>&1 &&
timeout -k 10 300 rocprofv3 --pmc SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_IFETCH SQ_LDS_BANK_CONFLICT -d $OUT/b -o run -- $P > $OUT/b.log 2>&1 &&
timeout -k 10 300 rocprofv3 --pmc SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_TRANS_F64 SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_MISC SQ_BUSY_CYCLES SQ_INSTS_VALU_INT32 -d $OUT/c -o run -- $P > $OUT/c.log 2>&1
echo "exit $?"
