#!/usr/bin/env python3
"""Basic blocks of one kernel's main loop in a hipcc -S file, with VALU / SALU / memory instruction counts per block
and the section markers (asm comments "; MARK_<name>") they fall in — the raw material of the per-section
instruction budget in DESIGN.md §6 (which blocks a clean chunk executes is read off the branches).
usage: tools/isa_blocks.py <file.s> <kernel-substring> <loop-header-label> [--path lbl,lbl,...]"""
import re
import sys


def classify(op):
    if op.startswith("v_readlane") or op.startswith("v_readfirstlane") or op.startswith("v_writelane"):
        return "valu"
    if op.startswith("v_"):
        return "valu"
    if op.startswith("s_waitcnt") or op.startswith("s_nop") or op.startswith("s_setprio"):
        return "wait"
    if op.startswith("s_cbranch") or op.startswith("s_branch"):
        return "branch"
    if op.startswith("s_load") or op.startswith("s_buffer_load"):
        return "smem"
    if op.startswith("s_"):
        return "salu"
    if op.startswith(("global_", "buffer_", "scratch_", "flat_")):
        return "vmem"
    if op.startswith("ds_"):
        return "lds"
    return "other"


def main():
    path, kname, hdr = sys.argv[1], sys.argv[2], sys.argv[3]
    want = None
    if "--path" in sys.argv:
        want = sys.argv[sys.argv.index("--path") + 1].split(",")
    L = open(path).read().split("\n")
    s = next(i for i, l in enumerate(L) if re.match(r"^_Z\S*" + re.escape(kname) + r"\S*:", l))
    e = next(i for i in range(s, len(L)) if L[i].strip().startswith("s_endpgm"))
    K = L[s:e + 1]
    h = next(i for i, l in enumerate(K) if l.startswith(hdr + ":"))
    tag = "Header=" + hdr[1:].replace("LBB", "BB") + " "
    last = max(i for i, l in enumerate(K) if tag in l + " ")
    j = last + 1
    while j < len(K) and not re.match(r"^(\.LBB\d+_\d+:|; %bb\.\d+:)", K[j]):
        j += 1
    blocks, cur, mark = [], None, "-"
    for l in K[h:j]:
        m = re.match(r"^(\.LBB\d+_\d+):|^; (%bb\.\d+):", l)
        if m:
            cur = {"label": m.group(1) or m.group(2), "n": {}, "mark": mark, "ops": []}
            blocks.append(cur)
            continue
        t = l.strip()
        if t.startswith("; MARK_"):
            mark = t[7:]
            continue
        if not t or t.startswith((";", ".")):
            continue
        op = t.split()[0]
        c = classify(op)
        cur["n"][c] = cur["n"].get(c, 0) + 1
        cur["ops"].append(t)
    for b in blocks:
        if want is not None and b["label"] not in want:
            continue
        br = [o for o in b["ops"] if o.startswith("s_cbranch") or o.startswith("s_branch")]
        print(f'{b["label"]:12s} [{b["mark"]:18s}] {b["n"]}  {" | ".join(br)}')
    if want is not None:
        tot = {}
        for b in blocks:
            if b["label"] in want:
                for k, v in b["n"].items():
                    tot.setdefault(b["mark"], {}).setdefault(k, 0)
                    tot[b["mark"]][k] += v
        for m, d in tot.items():
            print(m, d)


if __name__ == "__main__":
    main()
