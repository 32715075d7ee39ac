"""Print per-kernel counter sums/means from rocprofv3 pass databases: python tools/pmc_table.py DIR..."""
import glob, sqlite3, sys
for d in sys.argv[1:]:
    for db in sorted(glob.glob(f"{d}/**/*.db", recursive=True)):
        con = sqlite3.connect(db)
        q = ("select kernel_name, counter_name, count(*), sum(value) from counters_collection "
             "where kernel_name like '%ipm_%' group by kernel_name, counter_name")
        for k, c, n, v in con.execute(q):
            print(f"{db.split('/')[-3]:>6} {k[:40]:40s} {c:28s} n={n} sum={v:.4g}")
