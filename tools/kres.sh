#!/bin/bash
# per-kernel register / occupancy summary of csa_legacy.hip (hipcc remarks)
hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -shared -Rpass-analysis=kernel-resource-usage \
    -o /tmp/kres.so citizensassemblies-replication_amd/csrc/csa_legacy.hip 2>&1 | \
python3 -c '
import sys,re
cur=None; rows={}
for line in sys.stdin:
    m=re.search(r"remark:\s+(.*?)\s*\[-Rpass",line)
    if not m: continue
    t=m.group(1)
    if t.startswith("Function Name:"):
        cur=t.split(":",1)[1].strip(); rows[cur]={}
    elif cur and ":" in t:
        k,v=t.split(":",1); rows[cur][k.strip()]=v.strip()
for f,r in rows.items():
    if len(sys.argv)>1 and sys.argv[1] not in f: continue
    print("%-60s VGPR %-4s AGPR %-4s SGPR %-4s sSpill %-4s vSpill %-4s occ %-2s LDS %s"%(f[:60],r.get("VGPRs"),r.get("AGPRs"),r.get("TotalSGPRs"),r.get("SGPRs Spill"),r.get("VGPRs Spill"),r.get("Occupancy [waves/SIMD]"),r.get("LDS Size [bytes/block]")))
' "$@"
