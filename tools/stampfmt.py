#!/usr/bin/env python3
"""Summarise gpurun_out/stamps.log (tools/stamps.py output): median per phase."""
import json
import sys

for line in open(sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/stamps.log"):
    if not line.startswith("{"):
        continue
    d = json.loads(line)
    if "lib" in d:
        print(d["lib"])
        continue
    if "grid_per_cu" in d:
        print(" grid", d["grid_per_cu"])
        continue
    print("  exit %.2f/%.2f setup %.2f flush %.2f" % (d["exit"][2], d["exit"][4], d["setup"][2], d["flush"][2]))
    for k in ("c0", "c1", "c2"):
        if k in d:
            c = d[k]
            print("   %s L%.2f F%.2f C%.2f %s" % (k, c["load"][2], c["finish"][2], c["count"][2],
                                             " ".join("%s=%.2f" % kv for kv in c.get("sub", {}).items())))
