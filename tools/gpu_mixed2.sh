#!/bin/bash
# the mixed-precision A/B (tools/ab_mixed.sh) and then the mixed / solver / rollout parity tests
set -o pipefail
bash tools/ab_mixed.sh "$@" > gpurun_out/ab_rc.log 2>&1 && grep -q "exit 0" gpurun_out/ab_rc.log &&
timeout -k 10 900 python -u -m pytest tests/test_mixed_gpu.py tests/test_solver_gpu.py tests/test_rollout_gpu.py -m gpu -x -v --timeout 200 --timeout-method thread > gpurun_out/solvetests.log 2>&1
echo "exit $?"
