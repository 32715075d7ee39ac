#!/bin/bash
# dev loop on the GPU box: solver parity tests, then the N / shape sweeps
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest ${TESTS:-tests/test_solver_gpu.py} -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gputests.log 2>&1 &&
timeout -k 10 300 python3 -u tools/nsweep.py > gpurun_out/nsweep.log 2>&1 &&
timeout -k 10 300 python3 -u tools/shape_probe.py > gpurun_out/shape.log 2>&1
echo "exit $?"
