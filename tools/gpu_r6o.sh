#!/bin/bash
# Round-6 GPU session O: REFINE_RTOL 1e-6 (product) against 1e-5 / 3e-5 / 1e-4 (tools/mixed_probe.py)
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
O=gpurun_out
: > $O/ab_refine2.log
run() {
  echo "== ${1:-libkmpc.so}" >> $O/ab_refine2.log
  KMPC_DEV_LIB=$1 REPS=4 NCHK=64 timeout -k 10 240 python3 -u tools/mixed_probe.py 65536 5e-5 >> $O/ab_refine2.log 2>&1
}
run "" && run libkmpc_rt5.so && run libkmpc_rt2.so && run libkmpc_rt4.so && run "" && run libkmpc_rt4.so || exit $?
echo "exit 0"
