#!/bin/bash
# A/B of rollout GEMM variant libraries (tools/x3_probe.py, encoder input 1024 wide so both 1024-wide
# layers have K = 1024): probe output + per-kernel rocprofv3 table per library.   bash tools/ab_x3.sh lib...
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
: > gpurun_out/ab_x3.log
for L in "$@"; do
  echo "== $L" >> gpurun_out/ab_x3.log
  KMPC_DEV_LIB=$L OBS=1024 timeout -k 10 200 rocprofv3 --kernel-trace -d gpurun_out/abx3_$L -o run -- python3 tools/x3_probe.py 2>&1 | grep -v "rocprofv3\]\|SQLite3\|amdgpu.ids\|HSA version\|generateRocpd" >> gpurun_out/ab_x3.log || exit $?
  python3 tools/kern_table.py $(find gpurun_out/abx3_$L -name "*.db" | head -1) 12 >> gpurun_out/ab_x3.log 2>&1
  find gpurun_out/abx3_$L -name "*.db" -delete
done
echo "exit 0"
