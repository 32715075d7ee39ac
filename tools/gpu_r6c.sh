#!/bin/bash
# Round-6 GPU session C: the large-window record fold (product, mode 3) against rf0, every GPU test,
# then the default bench line.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
O=gpurun_out
: > $O/ab_c5.log
for L in "" libkmpc_rf0.so "" libkmpc_rf0.so; do
  echo "== ${L:-libkmpc.so}" >> $O/ab_c5.log
  KMPC_DEV_LIB=$L REPS=3 NCHK=8 timeout -k 10 300 python3 -u tools/c5_probe.py 1024 >> $O/ab_c5.log 2>&1 || exit $?
done
timeout -k 10 600 python -u -m pytest tests -m gpu -q --timeout 200 --timeout-method thread -rf > $O/gputests.log 2>&1
rc=$?; echo "gputests rc $rc"; [ $rc -le 1 ] || exit $rc
timeout -k 10 600 python -u bench.py > $O/bench.log 2>&1 || exit $?
echo "exit 0"
