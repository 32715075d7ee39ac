#!/bin/bash
# Round-6 GPU session Z: REFINE_RTOL 1e-4 alone (REFINE_MU stays 1e-6) — the GPU suite, then the
# default bench line
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > gpurun_out/gputests_z.log 2>&1 || exit $?
timeout -k 10 600 python -u bench.py --cpu-seconds 0 > gpurun_out/bench_z.log 2> gpurun_out/bench_z.err || exit $?
echo "exit 0"
