"""Summarise rocprofv3 rocpd databases (kernel trace --stats, --pmc passes) into profiles/.

usage: python tools/prof_summary.py OUT.md TRACE_DB [PMC_DB ...]
Writes the per-kernel duration table (the --stats view `top_kernels`), the launch resources of
each kernel, and per-kernel mean PMC values (FETCH_SIZE / WRITE_SIZE in KB per dispatch, with
the gfx950 FETCH_SIZE x2 correction of MI355X_MICROARCH.md §HBM applied in a separate column).
"""
import sqlite3
import sys


def rows(db, q):
    con = sqlite3.connect(db)
    try:
        return list(con.execute(q))
    finally:
        con.close()


def main():
    out, trace, pmcs = sys.argv[1], sys.argv[2], sys.argv[3:]
    lines = [f"# rocprofv3 summary ({trace})", "", "## Kernel durations (rocprofv3 --kernel-trace --stats)", "",
             "| kernel | calls | total µs | average µs | % |", "|---|---|---|---|---|"]
    for name, calls, tot, avg, pct in rows(trace, "select name,total_calls,total_duration,average,percentage from top_kernels"):
        lines.append(f"| `{name[:90]}` | {calls} | {tot:.0f} | {avg:.0f} | {pct:.2f} |")
    lines += ["", "## Launch resources", "", "| kernel | grid | workgroup | LDS B | scratch B | arch VGPR | accum VGPR | SGPR |",
              "|---|---|---|---|---|---|---|---|"]
    seen = set()
    for r in rows(trace, "select name,grid_x,workgroup_x,lds_size,scratch_size,vgpr_count,"
                         "accum_vgpr_count,sgpr_count from kernels"):
        if r[0] in seen or r[0].startswith("void at::"):
            continue
        seen.add(r[0])
        lines.append("| `" + r[0][:60] + "` | " + " | ".join(str(x) for x in r[1:]) + " |")
    for db in pmcs:
        lines += ["", f"## PMC ({db})", "", "| kernel | counter | dispatches | mean value per dispatch | corrected bytes / dispatch |",
                  "|---|---|---|---|---|"]
        q = ("select kernel_name, counter_name, count(*), avg(value) from counters_collection "
             "group by kernel_name, counter_name")
        for name, ctr, n, v in rows(db, q):
            if name.startswith("void at::") or name.startswith("__amd"):
                continue
            if ctr in ("FETCH_SIZE", "WRITE_SIZE"):   # KB; FETCH_SIZE x2 on gfx950
                corr = f"{v * 1024 * (2 if ctr == 'FETCH_SIZE' else 1):.4g}"
                val = f"{v:.1f} KB"
            else:
                corr, val = "", f"{v:.4g}"
            lines.append(f"| `{name[:60]}` | {ctr} | {n} | {val} | {corr} |")
    open(out, "w").write("\n".join(lines) + "\n")
    print("\n".join(lines))


if __name__ == "__main__":
    main()
