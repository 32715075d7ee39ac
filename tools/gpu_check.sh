#!/bin/bash
# GPU parity tests + smoke + default bench (no profiler passes) [+ f64 peak probe].
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 700 python -u -m pytest ${1:-tests} -m gpu -x -v --timeout 180 --timeout-method thread > gpurun_out/gputests.log 2>&1 &&
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 &&
timeout -k 10 400 python bench.py > gpurun_out/bench.log 2>gpurun_out/bench.err &&
{ [ ! -x tools/dev/f64_peak ] || timeout -k 10 60 tools/dev/f64_peak > gpurun_out/f64_peak.log 2>&1; }
echo "exit $?"
