#!/bin/bash
# PMC passes over the configs[1] rollout kernels (tools/gemm_probe.py), one pass per counter group.
#   bash tools/pmc_gemm.sh [lib]
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/pmc_gemm
mkdir -p $OUT
export KMPC_DEV_LIB=${1:-}
P="python3 tools/gemm_probe.py"
timeout -s KILL 90 rocprofv3 --kernel-trace --stats -d $OUT/trace -o run -- $P > $OUT/trace.log 2>&1 &&
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_LDS SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_ANY -d $OUT/a -o run -- $P > $OUT/a.log 2>&1 &&
timeout -s KILL 90 rocprofv3 --pmc SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_LDS_IDX_ACTIVE SQ_LDS_UNALIGNED_STALL SQ_WAVES -d $OUT/b -o run -- $P > $OUT/b.log 2>&1 &&
timeout -s KILL 90 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum TCP_TCC_READ_REQ_sum SQ_INST_CYCLES_VMEM -d $OUT/c -o run -- $P > $OUT/c.log 2>&1
echo "exit $?"
