#!/bin/bash
# Round-6 GPU session L: the C5 large-window launch's tail (tools/c5_tail_probe.py)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python3 -u tools/c5_tail_probe.py > gpurun_out/c5_tail.log 2>&1 || exit $?
echo "exit 0"
