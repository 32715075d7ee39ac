"""Per-dispatch FETCH_SIZE (x2, gfx950) / WRITE_SIZE of ipm_mixed_kernel from rocprofv3 --pmc
databases, per window: python tools/pmc_mixed.py WINDOWS FETCH_DB WRITE_DB"""
import sqlite3
import sys


def avg(db, counter):
    con = sqlite3.connect(db)
    try:
        r = con.execute("select avg(value) from counters_collection where kernel_name like '%ipm_mixed_kernel%' "
                        "and counter_name = ?", (counter,)).fetchone()
    finally:
        con.close()
    return r[0]


B = int(sys.argv[1])
f, w = avg(sys.argv[2], "FETCH_SIZE"), avg(sys.argv[3], "WRITE_SIZE")
print(f"ipm_mixed_kernel per window: fetched {2 * 1024 * f / B:.0f} B, written {1024 * w / B:.0f} B")
