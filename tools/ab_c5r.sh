#!/bin/bash
# configs[4] rollout per library: event time and one call's kernel trace in launch order.
#   bash tools/ab_c5r.sh lib...
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
: > gpurun_out/ab_c5r.log
for L in "$@"; do
  echo "== $L" >> gpurun_out/ab_c5r.log
  KMPC_DEV_LIB=$L timeout -k 10 120 python3 tools/c5_rollout_probe.py >> gpurun_out/ab_c5r.log 2>&1 || exit $?
  KMPC_DEV_LIB=$L timeout -k 10 200 rocprofv3 --kernel-trace -d gpurun_out/abc5r_$L -o run -- python3 tools/c5_rollout_probe.py > /dev/null 2>&1 || exit $?
  python3 tools/trace_order.py $(find gpurun_out/abc5r_$L -name "*.db" | head -1) 0 90 >> gpurun_out/ab_c5r.log 2>&1
  find gpurun_out/abc5r_$L -name "*.db" -delete
done
echo "exit 0"
