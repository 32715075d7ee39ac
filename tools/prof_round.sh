#!/bin/bash
# Profiling passes only (tests/smoke/bench run separately): rocprofv3 kernel trace + HBM and f64
# issue PMC passes of the C3 bench, then the C5 large-window kernel passes (tools/pmc_big.sh).
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
B="python bench.py --cpu-seconds 0 --steps 3 --warmup 1"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run -- $B > gpurun_out/prof.log 2>&1 &&
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/pmc_fetch -o run -- $B > gpurun_out/pmc_fetch.log 2>&1 &&
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/pmc_write -o run -- $B > gpurun_out/pmc_write.log 2>&1 &&
timeout -k 10 300 rocprofv3 --pmc SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_TRANS_F64 SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU -d gpurun_out/pmc_f64 -o run -- $B > gpurun_out/pmc_f64.log 2>&1 &&
bash tools/pmc_big.sh
echo "exit $?"
