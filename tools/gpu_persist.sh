#!/bin/bash
# Dev: backtest GPU tests, then the lock-step probe (persistent default vs 3 path groups)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_backtest_gpu.py -x -q --timeout 300 --timeout-method thread > gpurun_out/t_bt.log 2>&1 || exit $?
CASES=${CASES:-64x130,256x130,1024x130} PRE=1 GRAPH=0 PATH_GROUPS=${PG:-d,3} timeout -k 10 300 python3 -u tools/lockstep_probe.py > gpurun_out/lsp.log 2>&1
