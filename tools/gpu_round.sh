#!/bin/bash
# One GPU session: parity tests, smoke, bench, rocprofv3 kernel trace + HBM PMC passes of the bench.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
B="python bench.py --cpu-seconds 0 --steps 3 --warmup 1"
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/gputests.log 2>&1 &&
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 &&
timeout -k 10 400 python bench.py > gpurun_out/bench.log 2>gpurun_out/bench.err &&
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run -- $B > gpurun_out/prof.log 2>&1 &&
timeout -k 10 400 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/pmc_fetch -o run -- $B > gpurun_out/pmc_fetch.log 2>&1 &&
timeout -k 10 400 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/pmc_write -o run -- $B > gpurun_out/pmc_write.log 2>&1 &&
timeout -k 10 400 rocprofv3 --pmc SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_TRANS_F64 SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU -d gpurun_out/pmc_f64 -o run -- $B > gpurun_out/pmc_f64.log 2>&1
echo "exit $?"
