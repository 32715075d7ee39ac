#!/bin/bash
# Round-6 GPU session P: REFINE_RTOL 1e-5 in the product — the GPU suite, then C5 (large-window
# kernel) against the 1e-6 build (libkmpc_old6.so), alternating
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
O=gpurun_out
timeout -k 10 800 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gputests.log 2>&1 || exit $?
: > $O/ab_c5_rtol.log
for L in "" libkmpc_old6.so "" libkmpc_old6.so; do
  echo "== ${L:-libkmpc.so}" >> $O/ab_c5_rtol.log
  KMPC_DEV_LIB=$L REPS=3 NCHK=8 timeout -k 10 240 python3 -u tools/c5_probe.py 1024 >> $O/ab_c5_rtol.log 2>&1 || exit $?
done
echo "exit 0"
