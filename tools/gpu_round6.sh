#!/bin/bash
# Round-6 profiling session: f64 peak probe, rocprofv3 kernel trace + HBM / f64 / f32 issue PMC passes of the bench, then the
# C5 large-window passes (tools/pmc_big.sh). Databases are summarised on the box and deleted.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
B="python bench.py --cpu-seconds 0 --steps 3 --warmup 1"
BH="$B --headline-only"   # (the PMC passes: the headline step only)
O=gpurun_out
timeout -k 10 60 tools/dev/f64_peak > $O/f64_peak.log 2>&1 &&
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/prof -o run -- $B > $O/prof.log 2>&1 &&
timeout -k 10 400 rocprofv3 --pmc FETCH_SIZE -d $O/pmc_fetch -o run -- $BH > $O/pmc_fetch.log 2>&1 &&
timeout -k 10 400 rocprofv3 --pmc WRITE_SIZE -d $O/pmc_write -o run -- $BH > $O/pmc_write.log 2>&1 &&
timeout -k 10 400 rocprofv3 --pmc SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_TRANS_F64 SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU -d $O/pmc_f64 -o run -- $BH > $O/pmc_f64.log 2>&1 &&
bash tools/pmc_big.sh &&
timeout -k 10 400 rocprofv3 --pmc SQ_INSTS_VALU_ADD_F32 SQ_INSTS_VALU_MUL_F32 SQ_INSTS_VALU_FMA_F32 SQ_INSTS_VALU_TRANS_F32 -d $O/pmc_f32 -o run -- $BH > $O/pmc_f32.log 2>&1
rc=$?
db() { find $O/$1 -name '*.db' | head -1; }
python tools/prof_summary.py $O/bench_c3.md "$(db prof)" "$(db pmc_fetch)" "$(db pmc_write)" "$(db pmc_f64)" > /dev/null
F32_DB="$(db pmc_f32)" python tools/pmc_json.py $O/solve_pmc.json 65536 100 128 "$(db pmc_fetch)" "$(db pmc_write)" "$(db pmc_f64)" $O/f64_peak.log > /dev/null
python tools/prof_summary.py $O/big_c5.md "$(db pmc_big/trace)" "$(db pmc_big/fetch)" "$(db pmc_big/write)" "$(db pmc_big/sq)" > /dev/null
find $O -name '*.db' -delete
echo "exit $rc"
