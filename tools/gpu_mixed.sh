#!/bin/bash
# mixed-precision dev loop on the GPU box: the A/B probe, then the solver + mixed parity tests
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u tools/mixed_probe.py ${B:-65536} > gpurun_out/mixed.log 2>&1 &&
timeout -k 10 700 python -u -m pytest ${TESTS:-tests/test_mixed_gpu.py tests/test_solver_gpu.py} -m gpu -x -v --timeout 200 --timeout-method thread > gpurun_out/solvetests.log 2>&1
echo "exit $?"
