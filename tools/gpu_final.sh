#!/bin/bash
# Round-end check on one GPU box: every GPU test, smoke(), then the default bench line
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/gputests.log 2>&1 || exit $?
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/smoke.log 2>&1 || exit $?
timeout -k 10 600 python -u bench.py > gpurun_out/bench.log 2>&1 || exit $?
echo "exit 0"
