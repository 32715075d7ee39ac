#!/bin/bash
# Per-kernel register / spill / LDS summary of one solve translation unit (compile remarks).
# usage: tools/res_usage.sh koopman_mpc_portfolio_rebalancing_amd/csrc/kmpc_solve_p5.hip [extra hipcc flags]
SRC=$1; shift
/opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -Os -c "$SRC" -o /tmp/res_usage.o \
    -Rpass-analysis=kernel-resource-usage "$@" 2>&1 | python3 -c '
import re, sys
cur = None
rows = []
for line in sys.stdin:
    m = re.search(r"remark: +(.*?): (.*?) \[-Rpass", line)
    if not m: continue
    k, v = m.group(1).strip(), m.group(2).strip()
    if k == "Function Name":
        cur = {"name": v}; rows.append(cur)
    elif cur is not None:
        cur[k] = v
for r in rows:
    print(r["name"][:70], "VGPR", r.get("VGPRs"), "AGPR", r.get("AGPRs"), "spillV", r.get("VGPRs Spill"),
          "spillS", r.get("SGPRs Spill"), "LDS", r.get("LDS Size [bytes/block]"), "occ", r.get("Occupancy [waves/SIMD]"))
'
