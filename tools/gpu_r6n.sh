#!/bin/bash
# Round-6 GPU session N: the refinement rule of the C3 solve — REFINE_RTOL 1e-6 (product) against
# 1e-5 / 3e-6, REFINE_MU 1e-6 against 3e-7, and n_refine 2 (runtime) — tools/mixed_probe.py
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
O=gpurun_out
: > $O/ab_refine.log
run() {   # $1 = library ("" = product), $2 = n_refine (0 = default)
  echo "== ${1:-libkmpc.so} NREF=$2" >> $O/ab_refine.log
  KMPC_DEV_LIB=$1 NREF=$2 REPS=4 NCHK=64 timeout -k 10 240 python3 -u tools/mixed_probe.py 65536 5e-5 >> $O/ab_refine.log 2>&1
}
run "" 0 && run libkmpc_rt5.so 0 && run libkmpc_rt3.so 0 && run libkmpc_rm3.so 0 && run "" 2 && run "" 0 && run libkmpc_rt5.so 0 || exit $?
echo "exit 0"
