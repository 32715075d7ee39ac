#!/bin/bash
# A/B of variant libraries on the C3 solve, then the dev library's phase split
set -o pipefail
bash tools/ab_run.sh "$@" && bash tools/phase_run.sh libkmpc_dev.so
