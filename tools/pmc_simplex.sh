#!/bin/bash
# PMC passes over the configs[1] presolve (simplex_kernel) — tools/simplex_probe.py
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/pmc_simplex
mkdir -p $OUT
P="python3 tools/simplex_probe.py"
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_ACTIVE_INST_VALU -d $OUT/a -o run -- $P > $OUT/a.log 2>&1 &&
timeout -s KILL 90 rocprofv3 --pmc SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_BRANCH SQ_WAVES SQ_INSTS_VALU_TRANS_F64 SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_ADD_F64 -d $OUT/b -o run -- $P > $OUT/b.log 2>&1
echo "exit $?"
