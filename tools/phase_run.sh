#!/bin/bash
# dev-library phase split (tools/phase_stats.py) on C3-shaped solves; args: dev library names
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python3 tools/phase_stats.py 16384 "$@" > gpurun_out/phase.log 2>&1
echo "exit $?"
