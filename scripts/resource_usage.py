#!/usr/bin/env python3
"""Per-kernel register / scratch / occupancy table from hipcc's
-Rpass-analysis=kernel-resource-usage remarks (read on stdin).

    hipcc --offload-arch=gfx950 -O3 ... -c msa_capi.hip -Rpass-analysis=kernel-resource-usage 2>&1 |
        python3 scripts/resource_usage.py [substring-filter]
"""
import re
import subprocess
import sys

flt = sys.argv[1] if len(sys.argv) > 1 else ""
rows, cur = [], None
for line in sys.stdin:
    m = re.search(r"remark: (.*?) \[-Rpass", line)
    if not m:
        continue
    body = m.group(1).strip()
    if body.startswith("Function Name:"):
        cur = {"name": body.split(":", 1)[1].strip()}
        rows.append(cur)
    elif cur is not None and ":" in body:
        k, v = body.rsplit(":", 1)
        cur[k.strip()] = v.strip()
names = [r["name"] for r in rows]
try:
    dem = subprocess.run(["c++filt"], input="\n".join(names), capture_output=True, text=True).stdout.split("\n")
except OSError:
    dem = names
for r, d in zip(rows, dem):
    if flt and flt not in d:
        continue
    print(f"{r.get('VGPRs', '?'):>4} vgpr {r.get('AGPRs', '0'):>3} agpr {r.get('SGPRs', '?'):>4} sgpr "
          f"scratch {r.get('ScratchSize [bytes/lane]', '?'):>5} sspill {r.get('SGPRs Spill', '?'):>4} "
          f"vspill {r.get('VGPRs Spill', '?'):>4} occ {r.get('Occupancy [waves/SIMD]', '?'):>2}  {d[:110]}")
