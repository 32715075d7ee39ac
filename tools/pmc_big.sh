#!/bin/bash
# rocprofv3 kernel trace + HBM / issue counter passes over one C5 solve launch (tools/c5_probe.py)
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/pmc_big
mkdir -p $OUT
P="python3 tools/c5_probe.py 1024"
export REPS=1
timeout -s KILL 120 rocprofv3 --kernel-trace --stats -d $OUT/trace -o run -- $P > $OUT/trace.log 2>&1 &&
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d $OUT/fetch -o run -- $P > $OUT/fetch.log 2>&1 &&
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d $OUT/write -o run -- $P > $OUT/write.log 2>&1 &&
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_WAIT_INST_ANY -d $OUT/sq -o run -- $P > $OUT/sq.log 2>&1
echo "exit $?"
