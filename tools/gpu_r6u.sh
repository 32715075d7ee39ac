#!/bin/bash
# Round-6 GPU session U: the no-short step 0.995 / capped sigma <= 0.2 rules (product) against
# 0.99 / no cap in every solve unit (libkmpc_oldrule.so) — whole bench lines with the box's copy of
# libkmpc.so swapped in place, then C5 (tools/c5_probe.py), then the GPU suite on the product
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
O=gpurun_out
P=koopman_mpc_portfolio_rebalancing_amd
cp $P/libkmpc.so $P/libkmpc_prod.so
: > $O/r6u_bench.log
for L in prod oldrule prod oldrule; do
  cp $P/libkmpc_$L.so $P/libkmpc.so
  echo "== $L" >> $O/r6u_bench.log
  timeout -k 10 400 python -u bench.py --cpu-seconds 0 >> $O/r6u_bench.log 2>>$O/r6u_bench.err || exit $?
done
cp $P/libkmpc_prod.so $P/libkmpc.so
: > $O/r6u_c5.log
for L in "" libkmpc_oldrule.so "" libkmpc_oldrule.so; do
  echo "== ${L:-libkmpc.so}" >> $O/r6u_c5.log
  KMPC_DEV_LIB=$L REPS=3 NCHK=8 timeout -k 10 240 python3 -u tools/c5_probe.py 1024 >> $O/r6u_c5.log 2>&1 || exit $?
done
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > $O/gputests.log 2>&1 || exit $?
echo "exit 0"
