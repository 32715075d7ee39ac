#!/bin/bash
# f32-phase variant A/B and a kernel trace of the small-P lock-step backtest (P = 64)
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
bash tools/ab_mixed.sh "$@" > gpurun_out/ab_rc.log 2>&1 && grep -q "exit 0" gpurun_out/ab_rc.log &&
CASES=64x40 GRAPH=0 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_lock -o run -- python3 tools/lockstep_probe.py > gpurun_out/prof_lock.log 2>&1 &&
python3 tools/prof_summary.py gpurun_out/lock_kernels.md "$(find gpurun_out/prof_lock -name '*.db' | head -1)" > /dev/null 2>&1
find gpurun_out/prof_lock -name '*.db' -delete
echo "exit $?"
