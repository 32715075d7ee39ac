#!/bin/bash
# Round-5 GPU session, part A: parity tests, smoke, the bench line (C3) and configs[3]'s per-rank
# workload (131,072 windows) as a bench line
set -o pipefail
mkdir -p gpurun_out
O=gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread > $O/gputests.log 2>&1 &&
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 &&
timeout -k 10 500 python bench.py > $O/bench.log 2>$O/bench.err &&
timeout -k 10 300 python bench.py --global-windows 131072 --cpu-seconds 0 --steps 3 --warmup 1 > $O/bench_c4rank.log 2>$O/bench_c4rank.err
echo "exit $?"
