#!/bin/bash
# GPU parity tests, smoke and the default bench line (no profiling passes)
set -o pipefail
mkdir -p gpurun_out
O=gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/gputests.log 2>&1 &&
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 &&
timeout -k 10 400 python bench.py > $O/bench.log 2>$O/bench.err
echo "exit $?"
