#!/bin/bash
# One GPU session: parity tests, smoke, bench, f64 peak probe, rocprofv3 kernel trace + HBM / f64
# issue PMC passes of the bench, then the C5 large-window passes (tools/pmc_big.sh). The rocpd
# databases are summarised on the box (profiles-ready .md / .json under gpurun_out/) and deleted.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
B="python bench.py --cpu-seconds 0 --steps 3 --warmup 1"
O=gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $O/gputests.log 2>&1 &&
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 &&
timeout -k 10 400 python bench.py > $O/bench.log 2>$O/bench.err &&
timeout -k 10 60 tools/dev/f64_peak > $O/f64_peak.log 2>&1 &&
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/prof -o run -- $B > $O/prof.log 2>&1 &&
timeout -k 10 400 rocprofv3 --pmc FETCH_SIZE -d $O/pmc_fetch -o run -- $B > $O/pmc_fetch.log 2>&1 &&
timeout -k 10 400 rocprofv3 --pmc WRITE_SIZE -d $O/pmc_write -o run -- $B > $O/pmc_write.log 2>&1 &&
timeout -k 10 400 rocprofv3 --pmc SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_TRANS_F64 SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU -d $O/pmc_f64 -o run -- $B > $O/pmc_f64.log 2>&1 &&
bash tools/pmc_big.sh
rc=$?
db() { find $O/$1 -name '*.db' | head -1; }
python tools/prof_summary.py $O/bench_c3.md "$(db prof)" "$(db pmc_fetch)" "$(db pmc_write)" "$(db pmc_f64)" > /dev/null
python tools/pmc_json.py $O/solve_pmc.json 65536 100 128 "$(db pmc_fetch)" "$(db pmc_write)" "$(db pmc_f64)" $O/f64_peak.log > /dev/null
python tools/prof_summary.py $O/big_c5.md "$(db pmc_big/trace)" "$(db pmc_big/fetch)" "$(db pmc_big/write)" "$(db pmc_big/sq)" > /dev/null
find $O -name '*.db' -delete
echo "exit $rc"
