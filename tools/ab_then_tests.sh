#!/bin/bash
# A/B of variant libraries on the C3 solve (tools/ab_run.sh), then the GPU parity tests on the
# product library: bash tools/ab_then_tests.sh libkmpc_a.so libkmpc_b.so ...
set -o pipefail
bash tools/ab_run.sh "$@" && bash tools/gpu_tests.sh
