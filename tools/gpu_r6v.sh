#!/bin/bash
# Round-6 GPU session V: the float32 handoff threshold re-swept under the round's new step / sigma
# rules and initial multipliers (tools/mixed_probe.py, product library), twice
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
: > gpurun_out/ab_v.log
for r in 1 2; do
  REPS=4 NCHK=32 timeout -k 10 300 python3 -u tools/mixed_probe.py 65536 1e-4,7e-5,5e-5,3e-5,2e-5 >> gpurun_out/ab_v.log 2>&1 || exit $?
done
echo "exit 0"
