#!/bin/bash
# GPU tests (all) + smoke + one bench line (no profiler passes): the quick round check.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/gputests.log 2>&1 &&
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 &&
timeout -k 10 400 python bench.py > gpurun_out/bench.log 2>gpurun_out/bench.err
echo "exit $?"
