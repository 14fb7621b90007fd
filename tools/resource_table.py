#!/usr/bin/env python3
"""Per-kernel VGPR / AGPR / SGPR / scratch / occupancy table of a HIP source for gfx950
(-Rpass-analysis=kernel-resource-usage), one line per kernel, demangled.
  python tools/resource_table.py file.hip [filter-substring]"""
import re
import subprocess
import sys

src = sys.argv[1]
filt = sys.argv[2] if len(sys.argv) > 2 else ""
r = subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-c", src, "-o",
                    "/dev/null", "-Rpass-analysis=kernel-resource-usage"], capture_output=True, text=True)
cur, rows = None, []
for line in r.stderr.splitlines():
    m = re.search(r"remark: Function Name: (\S+)", line)
    if m:
        cur = {"name": m.group(1)}
        rows.append(cur)
        continue
    m = re.search(r"remark: +([^:]+?)(?: \[[^]]*\])?: (\d+)", line)
    if m and cur is not None:
        cur[m.group(1).strip()] = m.group(2)
names = subprocess.run(["c++filt"], input="\n".join(r["name"] for r in rows), capture_output=True, text=True).stdout.split("\n")
for r, n in zip(rows, names):
    n = re.sub(r"\(.*", "", n.replace("(anonymous namespace)::", ""))
    if filt in n:
        print(f"{n:60s} VGPR {r.get('VGPRs','?'):>4} AGPR {r.get('AGPRs','?'):>4} SGPR {r.get('TotalSGPRs','?'):>4} "
              f"scratch {r.get('ScratchSize','?'):>4} occ {r.get('Occupancy','?')} lds {r.get('LDS Size','?')}")
