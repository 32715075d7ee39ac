#!/bin/bash
# A/B of solve-kernel variant libraries on the C3 solve (tools/solve_probe.py):
#   bash tools/ab_run.sh libkmpc_base.so libkmpc_x.so ...
set -o pipefail
mkdir -p gpurun_out
: > gpurun_out/ab.log
for L in "$@"; do
  echo "== $L" >> gpurun_out/ab.log
  KMPC_DEV_LIB=$L REPS=3 timeout -k 10 120 python3 -u tools/solve_probe.py 65536 >> gpurun_out/ab.log 2>&1 || exit $?
done
echo "exit 0"
