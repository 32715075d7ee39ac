#!/bin/bash
# Dev A/B of path-persistent backtest variants (csrc/Makefile tvar libraries): bash tools/ab_persist.sh lib...
set -o pipefail
mkdir -p gpurun_out
: > gpurun_out/ab_persist.log
for L in "" "$@"; do
  echo "== ${L:-libkmpc.so}" >> gpurun_out/ab_persist.log
  KMPC_DEV_LIB=$L CASES=${CASES:-64x130,256x130} PRE=1 GRAPH=0 PATH_GROUPS=d timeout -k 10 300 python3 -u tools/lockstep_probe.py >> gpurun_out/ab_persist.log 2>&1 || exit $?
done
echo "exit 0"
