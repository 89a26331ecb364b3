#!/usr/bin/env python3
"""Print abtest logs (gpurun_out/ab_*.log) as a table."""
import glob, json, sys
for f in sorted(glob.glob(sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/ab_*.log")):
    print(f)
    for l in open(f):
        if l.startswith("{"):
            d = json.loads(l)
            print(f"  {d['variant']:<34} g={d['grid_per_cu']} s={d['sched']}  {d['ms']*1000:8.1f} us  {d['algo_GBps']:8.1f} GB/s  spread {d['spread']}")
