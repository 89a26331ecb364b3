#!/usr/bin/env python3
"""Per-variant SQ instruction counts per wave from gpurun_out/valu_*/ (tools/gpu_valu.sh)."""
import csv
import glob
import os
from collections import defaultdict

for d in sorted(glob.glob("gpurun_out/valu_*")):
    f = glob.glob(os.path.join(d, "p1", "*counter_collection.csv"))
    if not f:
        continue
    acc = defaultdict(float)
    names = {}
    for r in csv.DictReader(open(f[0])):
        acc[(r["Dispatch_Id"], r["Counter_Name"])] += float(r["Counter_Value"])
        names[r["Dispatch_Id"]] = r["Kernel_Name"]
    per = defaultdict(lambda: defaultdict(list))
    for (disp, cn), v in acc.items():
        per[names[disp].split("(")[0].split("::")[-1]][cn].append(v)
    for k, cs in per.items():
        m = {c: sum(v) / len(v) for c, v in cs.items()}
        w = m.get("SQ_WAVES", 1)
        print("%-12s %-28s waves %6d " % (os.path.basename(d)[5:], k[:28], w) +
              " ".join("%s %.0f" % (c[8:], m[c] / w) for c in sorted(m) if c != "SQ_WAVES"))
