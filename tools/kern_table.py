"""Per-kernel table of a rocprofv3 --kernel-trace database: count, mean / min duration (us), grid.
python tools/kern_table.py RESULTS.db [TOP]"""
import sqlite3
import sys

con = sqlite3.connect(sys.argv[1])
top = int(sys.argv[2]) if len(sys.argv) > 2 else 20
rows = con.execute("select name, count(*), avg(duration) / 1000.0, min(duration) / 1000.0, grid_x, grid_y, grid_z, "
                   "workgroup_x from kernels group by name, grid_x, grid_y, grid_z "
                   "order by sum(duration) desc limit ?", (top,)).fetchall()
for name, n, avg, mn, gx, gy, gz, wg in rows:
    print(f"{n:5d} {avg:9.1f} {mn:9.1f} us  grid {gx}x{gy}x{gz} wg {wg}  {name[:90]}")
