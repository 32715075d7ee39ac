#!/bin/bash
# Round-6 GPU session R: the float32 phase's corrector refined from mu 1e-2 / 1e-3 (KMPC_F32_REFMU;
# libkmpc_rf2 / rf3) with deeper handoffs, against the product (no float32 refinement)
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
O=gpurun_out
: > $O/ab_r.log
run() {
  echo "== ${1:-libkmpc.so} $2" >> $O/ab_r.log
  KMPC_DEV_LIB=$1 REPS=3 NCHK=32 timeout -k 10 300 python3 -u tools/mixed_probe.py 65536 $2 >> $O/ab_r.log 2>&1
}
run "" 5e-5 && run libkmpc_rf2.so 5e-5,2e-5,1e-5,5e-6 && run libkmpc_rf3.so 5e-5,2e-5,1e-5 || exit $?
echo "exit 0"
