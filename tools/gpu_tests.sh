#!/bin/bash
# GPU parity tests only (optionally a subset: bash tools/gpu_tests.sh tests/test_mv_gpu.py)
set -o pipefail
mkdir -p gpurun_out
T=${1:-tests}
timeout -k 10 600 python -u -m pytest $T -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/gputests.log 2>&1
echo "exit $?"
