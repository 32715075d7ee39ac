#!/bin/bash
# The C3 solve's PMC passes only (HBM bytes, f64 issue counters) + their JSON summary.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
B="python bench.py --cpu-seconds 0 --steps 3 --warmup 1"
O=gpurun_out
timeout -k 10 60 tools/dev/f64_peak > $O/f64_peak.log 2>&1 &&
timeout -k 10 400 rocprofv3 --pmc FETCH_SIZE -d $O/pmc_fetch -o run -- $B > $O/pmc_fetch.log 2>&1 &&
timeout -k 10 400 rocprofv3 --pmc WRITE_SIZE -d $O/pmc_write -o run -- $B > $O/pmc_write.log 2>&1 &&
timeout -k 10 400 rocprofv3 --pmc SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_TRANS_F64 SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU -d $O/pmc_f64 -o run -- $B > $O/pmc_f64.log 2>&1
rc=$?
db() { find $O/$1 -name '*.db' | head -1; }
python tools/pmc_json.py $O/solve_pmc.json 65536 100 128 "$(db pmc_fetch)" "$(db pmc_write)" "$(db pmc_f64)" $O/f64_peak.log > /dev/null
python tools/prof_summary.py $O/pmc_c3.md "$(db pmc_fetch)" "$(db pmc_fetch)" "$(db pmc_write)" "$(db pmc_f64)" > /dev/null
find $O -name '*.db' -delete
echo "exit $rc"
