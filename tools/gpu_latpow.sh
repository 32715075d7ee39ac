#!/bin/bash
# Dev: rollout-side GPU tests, then a kernel trace of the C3 rollout (tools/c3_rollout_probe.py)
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_rollout_gpu.py tests/test_window_gpu.py tests/test_integration_gpu.py tests/test_backtest_gpu.py -x -q --timeout 300 --timeout-method thread > gpurun_out/t_roll.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/c3r -o r -- python3 tools/c3_rollout_probe.py > /dev/null 2>&1 && python3 tools/trace_order.py gpurun_out/c3r/r_results.db 0 400 > gpurun_out/c3r_order.txt; rc=$?
find gpurun_out/c3r -name "*.db" -delete
exit $rc
