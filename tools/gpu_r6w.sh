#!/bin/bash
# Round-6 final session: the GPU suite, then smoke + the default bench line + the profiles
# (tools/gpu_r6d.sh)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > gpurun_out/gputests.log 2>&1 || exit $?
bash tools/gpu_r6d.sh
