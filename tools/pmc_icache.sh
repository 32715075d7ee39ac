#!/bin/bash
# rocprofv3 counter passes over one product solve launch (tools/solve_probe.py): issue/stall split
# and instruction-cache behaviour of the solve kernel.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/pmc_ic
mkdir -p $OUT
P="python3 tools/solve_probe.py 16384"
export REPS=1
timeout -s KILL 60 rocprofv3 -L > $OUT/counters.txt 2>&1
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_IFETCH SQ_ACTIVE_INST_VALU SQ_INSTS_VALU -d $OUT/a -o run -- $P > $OUT/a.log 2>&1 &&
timeout -s KILL 120 rocprofv3 --pmc SQC_ICACHE_MISSES -d $OUT/b -o run -- $P > $OUT/b.log 2>&1 &&
timeout -s KILL 120 rocprofv3 --pmc SQC_ICACHE_HITS -d $OUT/c -o run -- $P > $OUT/c.log 2>&1 &&
timeout -s KILL 120 rocprofv3 --pmc SQ_IFETCH_LEVEL SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAIT_INST_LDS SQ_INSTS_SMEM SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_MISC -d $OUT/d -o run -- $P > $OUT/d.log 2>&1
echo "exit $?"
