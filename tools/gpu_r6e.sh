#!/bin/bash
# Round-6 GPU session E: C3 mixed-solve variants (park, optimisation level, handoff form) and the
# handoff threshold on the product; the new sharded-bench GPU test.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
O=gpurun_out
: > $O/ab_mixed.log
for L in "" libkmpc_p0.so libkmpc_os.so libkmpc_o3.so libkmpc_h2p0.so ""; do
  echo "== ${L:-libkmpc.so}" >> $O/ab_mixed.log
  KMPC_DEV_LIB=$L REPS=4 NCHK=16 timeout -k 10 240 python3 -u tools/mixed_probe.py 65536 5e-5 >> $O/ab_mixed.log 2>&1 || exit $?
done
echo "== libkmpc.so handoff sweep" >> $O/ab_mixed.log
REPS=4 NCHK=16 timeout -k 10 300 python3 -u tools/mixed_probe.py 65536 7e-5,5e-5,3e-5 >> $O/ab_mixed.log 2>&1 || exit $?
timeout -k 10 600 python -u -m pytest tests/test_bench_gpu.py -m gpu -v --timeout 500 --timeout-method thread -rf > $O/gputests_e.log 2>&1
echo "exit $?"
