#!/bin/bash
# One GPU session: probe, parity tests, smoke, bench, rocprofv3 kernel trace of the bench.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python tools/probe_solver.py 65536 > gpurun_out/probe.log 2>&1 &&
timeout -k 10 600 python -m pytest tests -m gpu -x -q > gpurun_out/gputests.log 2>&1 &&
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 &&
timeout -k 10 400 python bench.py > gpurun_out/bench.log 2>gpurun_out/bench.err &&
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run -- python bench.py --cpu-seconds 0 > gpurun_out/prof.log 2>&1
echo "exit $?"
