#!/usr/bin/env python3
"""Per-kernel register/LDS/occupancy summary from hipcc -Rpass-analysis=kernel-resource-usage output (stdin)."""
import re
import sys

rows, cur = [], None
for line in sys.stdin:
    m = re.search(r"remark: Function Name: (\S+)", line)
    if m:
        cur = {"name": m.group(1)}
        rows.append(cur)
        continue
    m = re.search(r"remark:\s+(VGPRs|AGPRs|TotalSGPRs|VGPRs Spill|SGPRs Spill|Occupancy \[waves/SIMD\]|"
                  r"LDS Size \[bytes/block\]|ScratchSize \[bytes/lane\]): (\d+)", line)
    if m and cur is not None:
        cur[m.group(1).split(" [")[0]] = int(m.group(2))
for r in rows:
    if "kernel" not in r["name"]:
        continue
    print(f"{r.get('VGPRs', '?'):>4} v {r.get('VGPRs Spill', 0):>3} vs {r.get('TotalSGPRs', '?'):>4} s "
          f"{r.get('SGPRs Spill', 0):>3} ss {r.get('ScratchSize', 0):>4} scr {r.get('Occupancy', '?'):>2} occ "
          f"{r.get('LDS Size', 0):>6} lds  {r['name'][:90]}")
