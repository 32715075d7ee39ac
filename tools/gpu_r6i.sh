#!/bin/bash
# Round-6 GPU session I: the float32 phase's two-lanes-per-row Schur LDL^T (product) against
# s32off: output digests and the C3 mixed solve.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
O=gpurun_out
: > $O/digest.log
for L in "" libkmpc_s32off.so; do
  echo "== ${L:-libkmpc.so}" >> $O/digest.log
  KMPC_DEV_LIB=$L timeout -k 10 200 python3 -u tools/digest_probe.py >> $O/digest.log 2>&1 || exit $?
done
: > $O/ab_mixed.log
for L in "" libkmpc_s32off.so "" libkmpc_s32off.so; do
  echo "== ${L:-libkmpc.so}" >> $O/ab_mixed.log
  KMPC_DEV_LIB=$L REPS=4 NCHK=16 timeout -k 10 240 python3 -u tools/mixed_probe.py 65536 5e-5 >> $O/ab_mixed.log 2>&1 || exit $?
done
echo "exit 0"
