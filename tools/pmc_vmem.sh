#!/bin/bash
# Phase split (dev build) + memory/issue counters of the product solve kernel.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/pmc_vm
mkdir -p $OUT
P="python3 tools/solve_probe.py 16384"
export REPS=1
timeout -k 10 120 python3 tools/phase_stats.py 16384 libkmpc_dev.so > $OUT/phase.log 2>&1 &&
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_FLAT SQ_INSTS_BRANCH SQ_INST_CYCLES_VMEM SQ_WAVES SQ_INSTS_SMEM SQ_INSTS_VALU_TRANS_F64 -d $OUT/a -o run -- $P > $OUT/a.log 2>&1 &&
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_INT64 SQ_INSTS_VALU_CVT SQ_INSTS_VALU_FMA_F32 SQ_INSTS_VALU_ADD_F32 -d $OUT/b -o run -- $P > $OUT/b.log 2>&1
echo "exit $?"
