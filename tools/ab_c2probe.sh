#!/bin/bash
# tools/c2_graph_probe.py over variant libraries: LIBS="libkmpc.so libkmpc_x.so" [B=.. N=..] bash tools/ab_c2probe.sh
set -o pipefail
mkdir -p gpurun_out; : > gpurun_out/ab_c2probe.log
for L in ${LIBS:-libkmpc.so}; do
  echo "== $L" >> gpurun_out/ab_c2probe.log
  KMPC_DEV_LIB=$L timeout -k 10 120 python3 -u tools/c2_graph_probe.py >> gpurun_out/ab_c2probe.log 2>&1 || exit $?
done
echo "exit 0"
