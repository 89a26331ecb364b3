#!/usr/bin/env python3
"""Static instruction mix of the loop (depth-1 header) that contains a marker instruction, in one kernel of a hipcc -S
file: python tools/loopstat.py build/isa/cur.s <kernel-substring> <marker-regex>"""
import re
import sys

path, kname, marker = sys.argv[1], sys.argv[2], sys.argv[3]
L = open(path).read().split("\n")
start = next(i for i, l in enumerate(L) if re.match(r"^_Z\S*" + re.escape(kname) + r"\S*:", l))
end = next(i for i in range(start, len(L)) if L[i].strip().startswith("s_endpgm"))
K = L[start:end + 1]
mk = next(i for i, l in enumerate(K) if re.search(marker, l))
# the depth-1 loop header whose block list contains the marker's block
hdrs = [(i, re.match(r"(\.LBB\d+_\d+):", l).group(1)) for i, l in enumerate(K) if "Loop Header: Depth=1" in l]
best = None
for hi, lab in hdrs:
    tag = "Header=" + lab[1:].replace("LBB", "BB") + " "
    last = max([i for i, l in enumerate(K) if tag in l + " "] + [hi])
    j = last + 1
    while j < len(K) and not K[j].startswith(".LBB"):
        j += 1
    if hi <= mk < j:
        best = (hi, j, lab)
hi, j, lab = best
cnt = {}
for l in K[hi:j]:
    t = l.strip().split()
    if not t or t[0].startswith((";", ".")):
        continue
    op = t[0]
    key = ("readlane" if "readlane" in op else "writelane" if "writelane" in op else "valu" if op.startswith("v_")
           else "salu" if op.startswith("s_") else op.split("_")[0])
    cnt[key] = cnt.get(key, 0) + 1
print(lab, "lines", j - hi, cnt)
