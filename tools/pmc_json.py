"""Per-window PMC figures of the solve kernel for bench.py's roofline ``traffic`` and the f64 VALU
utilisation: python tools/pmc_json.py OUT.json WINDOWS_PER_LAUNCH ASSETS BLOCK FETCH_DB WRITE_DB F64_DB [F64_PEAK_LOG]

FETCH_SIZE is doubled (gfx950 correction, MI355X_MICROARCH.md §HBM); sizes are in KB per dispatch.
Executed f64 FLOPs = 64 lanes x (ADD + MUL + TRANS + 2 FMA) wave-instructions per dispatch; the
active-lane fraction is ASSETS / BLOCK (the window's lanes that hold an asset). F64_PEAK_LOG is the
output of tools/dev/f64_peak (the f64 FMA rate measured on the same part).
"""
import json
import os
import re
import sqlite3
import sys


# the C3 solve call's launches: ipm_mixed_kernel (float32 phase + float64 finish) and the retry
# ipm_kernel<..., 3> (the bench also runs other instances: the float64-only PH = 0 of the lock-step loop)
KERNEL = "%ipm_%kernel<10, 128, true, 7%"
EXCLUDE = "%, 64, 0>%"


def mean(db, counter):
    """Per solve call: the mean per dispatch of each kernel instance matching KERNEL, summed over
    the instances (the mixed-precision call dispatches the fused float32 phase + float64 finish
    and the retry pass once each)."""
    con = sqlite3.connect(db)
    try:
        rows = con.execute("select kernel_name, avg(value) from counters_collection where kernel_name like ? "
                           "and kernel_name not like ? and counter_name = ? group by kernel_name",
                           (KERNEL, EXCLUDE, counter)).fetchall()
    finally:
        con.close()
    vals = [float(v) for _, v in rows if v is not None]
    return sum(vals) if vals else None


def kernel_name(db):
    con = sqlite3.connect(db)
    try:
        r = con.execute("select distinct kernel_name from counters_collection where kernel_name like ? "
                        "and kernel_name not like ?", (KERNEL, EXCLUDE)).fetchall()
    finally:
        con.close()
    return " + ".join(x[0] for x in r) if r else None


out, B, N, blk = sys.argv[1], int(sys.argv[2]), int(sys.argv[3]), int(sys.argv[4])
fetch_db, write_db, f64_db = sys.argv[5], sys.argv[6], sys.argv[7]
f32_db = os.environ.get("F32_DB")   # optional pass with the float32 VALU counters (mixed precision)
d = {"kernel": kernel_name(fetch_db), "windows_per_launch": B,
     "fetch_bytes_per_window": 2 * 1024 * mean(fetch_db, "FETCH_SIZE") / B,
     "write_bytes_per_window": 1024 * mean(write_db, "WRITE_SIZE") / B,
     "source": "rocprofv3 --pmc passes of `python bench.py --cpu-seconds 0 --steps 3 --warmup 1 --headline-only` (tools/gpu_round6.sh)"}
ins = {c: mean(f64_db, c) for c in ("SQ_INSTS_VALU_ADD_F64", "SQ_INSTS_VALU_MUL_F64", "SQ_INSTS_VALU_FMA_F64",
                                    "SQ_INSTS_VALU_TRANS_F64", "SQ_WAVE_CYCLES", "SQ_WAIT_ANY",
                                    "SQ_ACTIVE_INST_VALU", "SQ_INSTS_VALU")}
if all(ins[c] is not None for c in list(ins)[:4]):
    d["f64_flops_per_window"] = 64 * (ins["SQ_INSTS_VALU_ADD_F64"] + ins["SQ_INSTS_VALU_MUL_F64"] +
                                      ins["SQ_INSTS_VALU_TRANS_F64"] + 2 * ins["SQ_INSTS_VALU_FMA_F64"]) / B
    d["active_lane_fraction"] = N / blk
if ins["SQ_WAVE_CYCLES"]:
    d["wait_any_fraction"] = ins["SQ_WAIT_ANY"] / ins["SQ_WAVE_CYCLES"]
    d["valu_active_fraction"] = ins["SQ_ACTIVE_INST_VALU"] / ins["SQ_WAVE_CYCLES"]
if ins["SQ_INSTS_VALU"]:
    d["f64_share_of_valu_insts"] = sum(ins[c] for c in list(ins)[:4]) / ins["SQ_INSTS_VALU"]
d["raw_counters_per_dispatch"] = ins
if f32_db:
    f32 = {c: mean(f32_db, c) for c in ("SQ_INSTS_VALU_ADD_F32", "SQ_INSTS_VALU_MUL_F32", "SQ_INSTS_VALU_FMA_F32",
                                        "SQ_INSTS_VALU_TRANS_F32")}
    if all(v is not None for v in f32.values()):
        d["f32_flops_per_window"] = 64 * (f32["SQ_INSTS_VALU_ADD_F32"] + f32["SQ_INSTS_VALU_MUL_F32"] +
                                          f32["SQ_INSTS_VALU_TRANS_F32"] + 2 * f32["SQ_INSTS_VALU_FMA_F32"]) / B
    d["raw_f32_counters_per_dispatch"] = f32
if len(sys.argv) > 8:
    v = [float(x) for x in re.findall(r"f64 fma: .*?([\d.]+) TFLOP/s", open(sys.argv[8]).read())]
    if v:   # best of the probe's runs (the first one includes clock ramp-up)
        d["f64_peak_flops"] = max(v) * 1e12
        d["f64_peak_source"] = "measured: tools/dev/f64_peak, best of its runs (independent v_fma_f64 chains over every CU)"
json.dump(d, open(out, "w"), indent=1)
print(json.dumps(d))
