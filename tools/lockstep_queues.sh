#!/bin/bash
# Dev A/B: lock-step path groups against the number of HIP hardware queues per process
set -o pipefail
mkdir -p gpurun_out
: > gpurun_out/lsq.log
echo "== default queues" >> gpurun_out/lsq.log
CASES=64x130 PRE=1 GRAPH=0 PATH_GROUPS=1,3,4 timeout -k 10 200 python3 -u tools/lockstep_probe.py >> gpurun_out/lsq.log 2>&1 || exit $?
echo "== GPU_MAX_HW_QUEUES=8" >> gpurun_out/lsq.log
GPU_MAX_HW_QUEUES=8 CASES=64x130 PRE=1 GRAPH=0 PATH_GROUPS=3,4,6,7,8 timeout -k 10 200 python3 -u tools/lockstep_probe.py >> gpurun_out/lsq.log 2>&1 || exit $?
echo "== GPU_MAX_HW_QUEUES=16" >> gpurun_out/lsq.log
GPU_MAX_HW_QUEUES=16 CASES=64x130,256x130 PRE=1 GRAPH=0 PATH_GROUPS=3,8,12,15 timeout -k 10 200 python3 -u tools/lockstep_probe.py >> gpurun_out/lsq.log 2>&1 || exit $?
