#!/bin/bash
# A/B of rollout variant libraries on the configs[1] step (tools/c2_graph_probe.py): step time and
# one step's kernel trace in launch order per library.   bash tools/ab_c2.sh lib...
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
: > gpurun_out/ab_c2.log
for L in "$@"; do
  echo "== $L" >> gpurun_out/ab_c2.log
  KMPC_DEV_LIB=$L timeout -k 10 120 python3 tools/c2_graph_probe.py >> gpurun_out/ab_c2.log 2>&1 || exit $?
  KMPC_DEV_LIB=$L timeout -k 10 200 rocprofv3 --kernel-trace -d gpurun_out/abc2_$L -o run -- python3 tools/c2_graph_probe.py > /dev/null 2>&1 || exit $?
  python3 tools/trace_order.py $(find gpurun_out/abc2_$L -name "*.db" | head -1) 60 9 >> gpurun_out/ab_c2.log 2>&1
  find gpurun_out/abc2_$L -name "*.db" -delete
done
echo "exit 0"
