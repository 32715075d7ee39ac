#!/bin/bash
# mixed-precision variant A/B, the lock-step backtest probe (eager vs HIP graph), the bf16 decision
# gap (bench.secondary_c5), then the backtest / rollout / window parity tests
set -o pipefail
mkdir -p gpurun_out
bash tools/ab_mixed.sh "$@" > gpurun_out/ab_rc.log 2>&1 && grep -q "exit 0" gpurun_out/ab_rc.log &&
timeout -k 10 400 python3 -u tools/lockstep_probe.py > gpurun_out/lockstep.log 2>&1 &&
timeout -k 10 300 python3 -u tools/bf16_gap_probe.py > gpurun_out/bf16gap.log 2>&1 &&
timeout -k 10 900 python -u -m pytest tests/test_backtest_gpu.py tests/test_rollout_gpu.py tests/test_window_gpu.py -m gpu -x -v --timeout 200 --timeout-method thread > gpurun_out/tests3.log 2>&1
echo "exit $?"
