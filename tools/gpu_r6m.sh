#!/bin/bash
# Round-6 GPU session M: the one-GPU rate against the batch a rank solves at N = 1 / 8 / 4 / 2
# (65,536 / 131,072 / 262,144 / 524,288 windows of the bench stream; headline line only)
set -o pipefail
mkdir -p gpurun_out
: > gpurun_out/r6m.log
for G in 65536 131072 262144 524288; do
  echo "== $G" >> gpurun_out/r6m.log
  timeout -k 10 400 python -u bench.py --headline-only --steps 3 --warmup 1 --global-windows $G >> gpurun_out/r6m.log 2>>gpurun_out/r6m.err || exit $?
done
echo "exit 0"
