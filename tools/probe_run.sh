#!/bin/bash
# run one dev probe script on the GPU box: bash tools/probe_run.sh tools/shape_probe.py [args]
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 500 python3 -u "$@" > gpurun_out/probe.log 2>&1
echo "exit $?"
