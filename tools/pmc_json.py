"""Per-window PMC figures of the solve kernel for bench.py's roofline ``traffic`` and the f64 VALU
roofline: python tools/pmc_json.py OUT.json WINDOWS_PER_LAUNCH FETCH_DB WRITE_DB [F64_DB]

FETCH_SIZE is doubled (gfx950 correction, MI355X_MICROARCH.md §HBM); sizes are in KB per dispatch.
Executed f64 FLOPs = 64 lanes x (ADD + MUL + TRANS + 2 FMA) wave-instructions per dispatch.
"""
import json
import sqlite3
import sys


def mean(db, counter):
    con = sqlite3.connect(db)
    try:
        r = con.execute("select avg(value) from counters_collection where kernel_name like '%ipm_kernel%' "
                        "and counter_name = ?", (counter,)).fetchone()
    finally:
        con.close()
    return float(r[0]) if r and r[0] is not None else None


out, B, fetch_db, write_db = sys.argv[1], int(sys.argv[2]), sys.argv[3], sys.argv[4]
d = {"kernel": "ipm_kernel<10,128,true,7> (kmpc_solve, constant-case)", "windows_per_launch": B,
     "fetch_bytes_per_window": 2 * 1024 * mean(fetch_db, "FETCH_SIZE") / B,
     "write_bytes_per_window": 1024 * mean(write_db, "WRITE_SIZE") / B,
     "source": "rocprofv3 --pmc passes of `python bench.py --cpu-seconds 0 --steps 3 --warmup 1` (tools/gpu_round.sh)"}
if len(sys.argv) > 5:
    f = sys.argv[5]
    ins = {c: mean(f, c) for c in ("SQ_INSTS_VALU_ADD_F64", "SQ_INSTS_VALU_MUL_F64", "SQ_INSTS_VALU_FMA_F64",
                                   "SQ_INSTS_VALU_TRANS_F64")}
    if all(v is not None for v in ins.values()):
        d["f64_flops_per_window"] = 64 * (ins["SQ_INSTS_VALU_ADD_F64"] + ins["SQ_INSTS_VALU_MUL_F64"] +
                                          ins["SQ_INSTS_VALU_TRANS_F64"] + 2 * ins["SQ_INSTS_VALU_FMA_F64"]) / B
json.dump(d, open(out, "w"), indent=1)
print(json.dumps(d))
