#!/bin/bash
# Round-6 GPU session X: under the final rules, REFINE_RTOL 1e-4 (libkmpc_rt4) and REFINE_MU 5e-7
# (libkmpc_rm5) against the product's 1e-5 / 1e-6 (tools/mixed_probe.py at the 3e-5 handoff), twice
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
: > gpurun_out/ab_x.log
for L in "" libkmpc_rt4.so libkmpc_rm5.so "" libkmpc_rt4.so libkmpc_rm5.so; do
  echo "== ${L:-libkmpc.so}" >> gpurun_out/ab_x.log
  KMPC_DEV_LIB=$L REPS=4 NCHK=32 timeout -k 10 240 python3 -u tools/mixed_probe.py 65536 3e-5 >> gpurun_out/ab_x.log 2>&1 || exit $?
done
echo "exit 0"
