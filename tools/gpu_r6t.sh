#!/bin/bash
# Round-6 GPU session T: the secondary_c5 windows (bf16 and fp32 rollouts) with the initial
# multipliers 0.5 (product) and 1 (libkmpc_bim1.so, the large-window unit)
set -o pipefail
mkdir -p gpurun_out
: > gpurun_out/c5_init.log
for L in "" libkmpc_bim1.so "" libkmpc_bim1.so; do
  for DT in bf16 fp32; do
    echo "== ${L:-libkmpc.so} $DT" >> gpurun_out/c5_init.log
    KMPC_DEV_LIB=$L DT=$DT timeout -k 10 300 python3 -u tools/c5_tail_probe.py >> gpurun_out/c5_init.log 2>&1 || exit $?
  done
done
echo "exit 0"
