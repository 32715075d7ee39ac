#!/bin/bash
# Round-6 GPU session F: the two-lanes-per-row Schur LDL^T (product) against sp0 (one lane per
# row): output digests (bit-identity), the C3 mixed / f64 solve, other register-kernel shapes.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
O=gpurun_out
: > $O/digest.log
for L in "" libkmpc_sp0.so; do
  echo "== ${L:-libkmpc.so}" >> $O/digest.log
  KMPC_DEV_LIB=$L timeout -k 10 200 python3 -u tools/digest_probe.py >> $O/digest.log 2>&1 || exit $?
done
: > $O/ab_mixed.log
for L in "" libkmpc_sp0.so "" libkmpc_sp0.so; do
  echo "== ${L:-libkmpc.so}" >> $O/ab_mixed.log
  KMPC_DEV_LIB=$L REPS=4 NCHK=16 timeout -k 10 240 python3 -u tools/mixed_probe.py 65536 5e-5 >> $O/ab_mixed.log 2>&1 || exit $?
done
LIBS="libkmpc.so libkmpc_sp0.so" SHAPES="N=64,H=10|N=120,H=10|N=90,H=7|N=200,H=10|N=250,H=10" \
  timeout -k 10 400 bash tools/ab_shapes.sh || exit $?
echo "exit 0"
