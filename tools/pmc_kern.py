"""Per-kernel (and grid) counter means from rocprofv3 pass databases:
python tools/pmc_kern.py PATTERN DIR..."""
import glob, sqlite3, sys
pat = sys.argv[1]
for d in sys.argv[2:]:
    for db in sorted(glob.glob(f"{d}/**/*.db", recursive=True)):
        con = sqlite3.connect(db)
        cols = [c[1] for c in con.execute("pragma table_info(counters_collection)")]
        g = ", ".join(c for c in ("grid_x", "grid_y", "grid_z") if c in cols)
        key = "kernel_name" + (", " + g if g else "")
        q = (f"select {key}, counter_name, count(*), avg(value) from counters_collection "
             f"where kernel_name like ? group by {key}, counter_name")
        for r in con.execute(q, (f"%{pat}%",)):
            k = r[0]
            grid = "x".join(str(v) for v in r[1:-3])
            print(f"{k[:40]:40s} {grid:>12s} {r[-3]:28s} n={r[-2]} mean={r[-1]:.4g}")
