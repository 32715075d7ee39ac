#!/bin/bash
# Round-6 GPU session K: the mixed solve's 64 B warm header (whole batch per launch) against the
# 20.2 KB record chunked by 131,072 windows (libkmpc_old.so): mixed tests, output digests, then
# alternating headline bench lines (the box's copy of libkmpc.so swapped in place).
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
O=gpurun_out
P=koopman_mpc_portfolio_rebalancing_amd
timeout -k 10 600 python -u -m pytest tests/test_mixed_gpu.py tests/test_window_gpu.py -x -q --timeout 300 --timeout-method thread > $O/r6k_tests.log 2>&1 || exit $?
: > $O/digest.log
for L in "" libkmpc_old.so; do
  echo "== ${L:-libkmpc.so}" >> $O/digest.log
  KMPC_DEV_LIB=$L timeout -k 10 200 python3 -u tools/digest_probe.py >> $O/digest.log 2>&1 || exit $?
done
cp $P/libkmpc.so $P/libkmpc_new.so
: > $O/r6k_bench.log
for L in new old new old; do
  cp $P/libkmpc_$L.so $P/libkmpc.so
  echo "== $L" >> $O/r6k_bench.log
  timeout -k 10 300 python -u bench.py --headline-only >> $O/r6k_bench.log 2>>$O/r6k_bench.err || exit $?
done
cp $P/libkmpc_new.so $P/libkmpc.so
echo "exit 0"
