#!/bin/bash
# A/B of packed-kernel variant libraries (csrc/Makefile pvar) on small-window shapes:
#   bash tools/ab_pack.sh libkmpc.so libkmpc_x.so ... [-- shapes]
set -o pipefail
mkdir -p gpurun_out
: > gpurun_out/ab_pack.log
LIBS=(); while [ $# -gt 0 ] && [ "$1" != "--" ]; do LIBS+=("$1"); shift; done; shift
for L in "${LIBS[@]}"; do
  echo "== $L" >> gpurun_out/ab_pack.log
  KMPC_DEV_LIB=$L PACKED_ONLY=1 timeout -k 10 120 python3 -u tools/pack_probe.py "$@" >> gpurun_out/ab_pack.log 2>&1 || exit $?
done
echo "exit 0"
