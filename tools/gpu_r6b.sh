#!/bin/bash
# Round-6 GPU session B: A/B of the mixed solve's handoff (product = registers; h0 = HBM record,
# h2 = LDS) without the lsolve steering branch, PMC bytes of each; the large-window record fold
# (product) against rf0; then the solver / mixed / backtest GPU tests on the product library.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
O=gpurun_out
: > $O/ab_mixed.log
for L in "" libkmpc_h0.so libkmpc_h2.so "" libkmpc_h0.so libkmpc_h2.so; do
  echo "== ${L:-libkmpc.so}" >> $O/ab_mixed.log
  KMPC_DEV_LIB=$L REPS=4 NCHK=16 timeout -k 10 240 python3 -u tools/mixed_probe.py 65536 5e-5 >> $O/ab_mixed.log 2>&1 || exit $?
done
: > $O/ab_c5.log
for L in "" libkmpc_rf0.so "" libkmpc_rf0.so; do
  echo "== ${L:-libkmpc.so}" >> $O/ab_c5.log
  KMPC_DEV_LIB=$L REPS=3 NCHK=8 timeout -k 10 300 python3 -u tools/c5_probe.py 1024 >> $O/ab_c5.log 2>&1 || exit $?
done
: > $O/pmc_mixed.log
for L in "" libkmpc_h0.so libkmpc_h2.so; do
  n=${L:-prod}
  KMPC_DEV_LIB=$L REPS=1 NCHK=4 timeout -s KILL 200 rocprofv3 --pmc FETCH_SIZE -d $O/pf_$n -o run -- python3 tools/mixed_probe.py 65536 5e-5 > /dev/null 2>&1 || exit $?
  KMPC_DEV_LIB=$L REPS=1 NCHK=4 timeout -s KILL 200 rocprofv3 --pmc WRITE_SIZE -d $O/pw_$n -o run -- python3 tools/mixed_probe.py 65536 5e-5 > /dev/null 2>&1 || exit $?
  echo "== $n $(python3 tools/pmc_mixed.py 65536 $(find $O/pf_$n -name '*.db' | head -1) $(find $O/pw_$n -name '*.db' | head -1))" >> $O/pmc_mixed.log
done
find $O -name '*.db' -delete
timeout -k 10 500 python -u -m pytest tests/test_mixed_gpu.py tests/test_solver_gpu.py tests/test_backtest_gpu.py -m gpu -q --timeout 200 --timeout-method thread -rf > $O/gputests_b.log 2>&1
echo "exit $?"
