#!/bin/bash
# A/B of the mixed-precision pair: the product library and variant libraries (csrc/Makefile tvar),
# then a rocprofv3 kernel trace of the product library's probe (float32 / float64 kernel split)
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
: > gpurun_out/ab_mixed.log
for L in "" "$@"; do
  echo "== ${L:-libkmpc.so}" >> gpurun_out/ab_mixed.log
  KMPC_DEV_LIB=$L REPS=3 timeout -k 10 240 python3 -u tools/mixed_probe.py 65536 1e-4,5e-5 >> gpurun_out/ab_mixed.log 2>&1 || exit $?
done
REPS=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_mixed -o run -- python3 tools/mixed_probe.py 65536 1e-4 > gpurun_out/prof_mixed.log 2>&1 || exit $?
python3 tools/prof_summary.py gpurun_out/mixed_kernels.md "$(find gpurun_out/prof_mixed -name '*.db' | head -1)" > /dev/null 2>&1
find gpurun_out/prof_mixed -name '*.db' -delete
echo "exit 0"
