#!/usr/bin/env python3
"""Append the JSON lines of GPU session step logs (gpurun_out/<tag>/<step>.log) to a committed profiles/ file, each
tagged with its session and step: python tools/collect_ab.py profiles/r04_ab.jsonl r04h r04i ..."""
import glob
import json
import os
import sys

out, tags = sys.argv[1], sys.argv[2:]
root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
n = 0
with open(out, "a") as f:
    for t in tags:
        for lg in sorted(glob.glob(os.path.join(root, "gpurun_out", t, "*.log"))):
            step = os.path.basename(lg)[:-4]
            for line in open(lg, errors="replace"):
                if line.startswith("{"):
                    try:
                        d = json.loads(line)
                    except ValueError:
                        continue
                    f.write(json.dumps({"session": t, "step": step, **d}) + "\n")
                    n += 1
print(f"{out}: +{n} lines")
