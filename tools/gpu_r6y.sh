#!/bin/bash
# Round-6 GPU session Y: REFINE_RTOL 1e-4 / REFINE_MU 5e-7 in every kernel — the GPU suite, C5
# against the oracle (tools/c5_probe.py), then smoke + bench + profiles (tools/gpu_r6d.sh)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > gpurun_out/gputests.log 2>&1 || exit $?
REPS=3 NCHK=16 timeout -k 10 300 python3 -u tools/c5_probe.py 1024 > gpurun_out/c5_y.log 2>&1 || exit $?
bash tools/gpu_r6d.sh
