"""Print the first dispatches of a rocprofv3 rocpd database in launch order with their durations:
python tools/trace_order.py DB [skip] [count]"""
import sqlite3
import sys

db, skip, n = sys.argv[1], int(sys.argv[2]) if len(sys.argv) > 2 else 0, int(sys.argv[3]) if len(sys.argv) > 3 else 40
con = sqlite3.connect(db)
cols = [r[1] for r in con.execute("pragma table_info(kernels)")]
s, e = ("start", "end") if "start" in cols else (cols[cols.index("start_timestamp")] if "start_timestamp" in cols else None, None)
q = f"select name, grid_x, grid_y, workgroup_x, {s}, \"{e}\" from kernels order by {s} limit {n} offset {skip}"
for name, gx, gy, wx, st, en in con.execute(q):
    print(f"{(en - st) / 1e3:9.1f} us  grid {gx}x{gy} wg {wx}  {name[:80]}")
