#!/bin/bash
# A/B of large-window variant libraries on the C5 solve (tools/c5_probe.py): bash tools/ab_c5.sh lib...
set -o pipefail
mkdir -p gpurun_out
: > gpurun_out/ab_c5.log
for L in "$@"; do
  echo "== $L" >> gpurun_out/ab_c5.log
  KMPC_DEV_LIB=$L REPS=3 NCHK=${NCHK:-0} timeout -k 10 300 python3 -u tools/c5_probe.py 1024 >> gpurun_out/ab_c5.log 2>&1 || exit $?
done
echo "exit 0"
