#!/bin/bash
# configs[1] (C2: 4,096 windows, N = 30, latent 128, H = 5) kernel trace: rocprofv3 --kernel-trace
# --stats of tools/c2_graph_probe.py (eager + graph-replayed steps), summarised on the box
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
O=gpurun_out
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/c2prof -o run -- python3 tools/c2_graph_probe.py > $O/c2prof.log 2>&1
rc=$?
python tools/prof_summary.py $O/c2_kernels.md "$(find $O/c2prof -name '*.db' | head -1)" > /dev/null
python tools/kern_table.py "$(find $O/c2prof -name '*.db' | head -1)" 12 > $O/c2_kern_table.txt
find $O/c2prof -name '*.db' -delete
echo "exit $rc"
