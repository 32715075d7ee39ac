#!/bin/bash
# Round-6 GPU session S: the initial multipliers 1 (product) against 0.5 / 0.4 (KMPC_INIT_MULT;
# the register kernels of the C3, packed H <= 5 and H = 5 backtest units) — whole bench lines,
# the box's copy of libkmpc.so swapped in place; then C5 against 0.5 in the large-window kernel
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
O=gpurun_out
P=koopman_mpc_portfolio_rebalancing_amd
cp $P/libkmpc.so $P/libkmpc_prod.so
: > $O/r6s_bench.log
for L in prod im5 im4 prod im5 im4; do
  cp $P/libkmpc_$L.so $P/libkmpc.so
  echo "== $L" >> $O/r6s_bench.log
  timeout -k 10 400 python -u bench.py --cpu-seconds 0 >> $O/r6s_bench.log 2>>$O/r6s_bench.err || exit $?
done
cp $P/libkmpc_prod.so $P/libkmpc.so
: > $O/r6s_c5.log
for L in "" libkmpc_bim5.so "" libkmpc_bim5.so; do
  echo "== ${L:-libkmpc.so}" >> $O/r6s_c5.log
  KMPC_DEV_LIB=$L REPS=3 NCHK=8 timeout -k 10 240 python3 -u tools/c5_probe.py 1024 >> $O/r6s_c5.log 2>&1 || exit $?
done
echo "exit 0"
