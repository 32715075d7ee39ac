#!/bin/bash
# A/B of variant libraries on large-window solve shapes (tools/c5_probe.py): bash tools/ab_big.sh libA.so libB.so ...
set -o pipefail
mkdir -p gpurun_out
: > gpurun_out/ab_big.log
for L in "$@"; do
  echo "== $L" >> gpurun_out/ab_big.log
  for S in "500 20 1024" "500 10 2048" "100 20 4096" "300 15 2048"; do
    set -- $S
    KMPC_DEV_LIB=$L REPS=3 PN=$1 PH=$2 timeout -k 10 120 python3 -u tools/c5_probe.py $3 2>/dev/null | grep " ms " | tail -1 >> gpurun_out/ab_big.log || exit $?
  done
done
echo "exit 0"
