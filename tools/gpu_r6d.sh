#!/bin/bash
# Round-6 evidence session: smoke, the default bench line, then tools/gpu_round6.sh (f64 peak,
# kernel trace, PMC passes of the headline, C5 passes).
set -o pipefail
mkdir -p gpurun_out
O=gpurun_out
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 &&
timeout -k 10 600 python -u bench.py > $O/bench.log 2>$O/bench.err &&
bash tools/gpu_round6.sh
