#!/bin/bash
# shape_probe.py over variant libraries: LIBS="libkmpc.so libkmpc_x.so" SHAPES="C2|C3" bash tools/ab_shapes.sh
set -o pipefail
mkdir -p gpurun_out
: > gpurun_out/ab_shapes.log
for L in ${LIBS:-libkmpc.so}; do
  echo "== $L" >> gpurun_out/ab_shapes.log
  KMPC_DEV_LIB=$L SHAPES="${SHAPES:-C2|N=64,H=10|N=30,H=5,cost|C1-shape|C3}" timeout -k 10 200 python3 -u tools/shape_probe.py >> gpurun_out/ab_shapes.log 2>&1 || exit $?
done
echo "exit 0"
