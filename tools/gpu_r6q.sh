#!/bin/bash
# Round-6 GPU session Q: the C3 mixed solve against park0 (w, s kept in registers in the float64
# finish), the C3 unit at -Os / -O3 (product -O2), and the handoff threshold re-swept with the
# refinement tolerance 1e-5 (tools/mixed_probe.py, product library)
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
O=gpurun_out
: > $O/ab_q.log
run() {
  echo "== ${1:-libkmpc.so} $2" >> $O/ab_q.log
  KMPC_DEV_LIB=$1 REPS=4 NCHK=32 timeout -k 10 240 python3 -u tools/mixed_probe.py 65536 $2 >> $O/ab_q.log 2>&1
}
run "" 5e-5 && run libkmpc_park0.so 5e-5 && run libkmpc_c3os.so 5e-5 && run libkmpc_c3o3.so 5e-5 && run "" 1e-4,7e-5,5e-5,3e-5,2e-5 || exit $?
echo "exit 0"
