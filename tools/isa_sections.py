#!/usr/bin/env python3
"""Static instruction budget of one kernel by source section: the kernel's instructions in a
`hipcc -S -DDK_ISA_MARKS` listing, each attributed to the last "; MARK_<name>" comment before it in layout order
(rx_diag.h DK_MARK), counted by class (VALU, SALU, branch, VMEM, LDS, SMEM, wait).

    python tools/isa_sections.py build/isa/rx_marked.s dk_rx_kernelILb0ELb1E [--json]
Cold sections (parse_slow, tcp_options) are listed separately; loop sections (med_step, large_step) are per
iteration. The section before the first mark is "prologue", after the loop "epilogue" (from the first mark that is
not in the loop)."""
import json
import re
import sys

sys.path.insert(0, __import__("os").path.dirname(__file__))
from isa_blocks import classify  # noqa: E402


def sections(path, kname):
    L = open(path).read().split("\n")
    s = next(i for i, l in enumerate(L) if re.match(r"^_Z\S*" + re.escape(kname) + r"\S*:", l))
    e = next(i for i in range(s, len(L)) if L[i].strip().startswith(".Lfunc_end"))
    out, mark, order = {}, "prologue", ["prologue"]
    for l in L[s:e]:
        t = l.strip()
        if t.startswith("; MARK_"):
            mark = t[7:].split()[0]
            if mark not in order:
                order.append(mark)
            continue
        if not t or t.startswith((";", ".")) or t.endswith(":"):
            continue
        c = classify(t.split()[0])
        d = out.setdefault(mark, {})
        d[c] = d.get(c, 0) + 1
    return order, out


def main():
    path, kname = sys.argv[1], sys.argv[2]
    order, out = sections(path, kname)
    if "--json" in sys.argv:
        print(json.dumps({m: out.get(m, {}) for m in order}))
        return
    keys = ["valu", "salu", "branch", "vmem", "lds", "smem", "wait", "other"]
    print(f"{'section':16s} " + " ".join(f"{k:>6s}" for k in keys))
    tot = {k: 0 for k in keys}
    for m in order:
        d = out.get(m, {})
        print(f"{m:16s} " + " ".join(f"{d.get(k, 0):6d}" for k in keys))
        for k in keys:
            tot[k] += d.get(k, 0)
    print(f"{'total':16s} " + " ".join(f"{tot[k]:6d}" for k in keys))


if __name__ == "__main__":
    main()
