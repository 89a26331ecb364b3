#!/usr/bin/env python3
"""Summarise tools/pmc_kernel.sh passes: per kernel, the mean over launches of every counter, plus derived figures
(instructions per wave, VALU busy %, occupancy %, wait share).
usage: tools/pmc_summary.py gpurun_out/pmc_<tag> [out.json] [kernel_us]
kernel_us: the kernel's average duration from a --kernel-trace run of the same build (the busy / occupancy shares are
taken against it at 2.4 GHz, i.e. lower bounds; GRBM_GUI_ACTIVE read inconsistently across passes on this pool)."""
import csv
import glob
import json
import os
import sys
from collections import defaultdict

CU = 256


def main():
    d = sys.argv[1]
    per = defaultdict(lambda: defaultdict(list))
    for f in sorted(glob.glob(os.path.join(d, "p*", "run_counter_collection.csv"))):
        # one value per (dispatch, counter): sum over dimensions (SE/CU/...) within a dispatch
        acc = defaultdict(float)
        names = {}
        for r in csv.DictReader(open(f)):
            key = (r["Dispatch_Id"], r["Counter_Name"])
            v = float(r["Counter_Value"])
            # GRBM_GUI_ACTIVE is a per-XCD clock count: the kernel's span is the max, not the sum
            acc[key] = max(acc[key], v) if r["Counter_Name"].startswith("GRBM") else acc[key] + v
            names[r["Dispatch_Id"]] = r["Kernel_Name"]
        for (disp, cn), v in acc.items():
            per[names[disp]][cn].append(v)
    out = {}
    for k, cs in per.items():
        m = {cn: sum(v) / len(v) for cn, v in cs.items()}
        short = k.split("(")[0].replace("void dk::(anonymous namespace)::", "")
        w = m.get("SQ_WAVES", 0)
        g = m.get("GRBM_GUI_ACTIVE", 0)
        der = {}
        if w:
            for cn in ("SQ_INSTS_VALU", "SQ_INSTS_SALU", "SQ_INSTS_LDS", "SQ_INSTS_VMEM_RD", "SQ_INSTS_VMEM_WR",
                       "SQ_INSTS_SMEM", "SQ_INSTS_BRANCH"):
                if cn in m:
                    der[cn + "_per_wave"] = round(m[cn] / w, 1)
        us = float(sys.argv[3]) if len(sys.argv) > 3 else 0.0
        if us:
            cyc = us * 2400.0  # shader cycles at the 2.4 GHz ceiling
            der["kernel_us_traced"] = us
            if "SQ_ACTIVE_INST_VALU" in m:  # quad-cycles summed over the 4 SIMDs of every CU
                der["VALUBusy_pct"] = round(100 * 4 * m["SQ_ACTIVE_INST_VALU"] / (4 * CU) / cyc, 1)
            if "SQ_WAVE_CYCLES" in m:  # resident waves per CU / 32
                der["OccupancyPercent"] = round(100 * 4 * m["SQ_WAVE_CYCLES"] / CU / cyc / 32, 1)
            if "SQ_WAVE_CYCLES" in m and "SQ_WAIT_ANY" in m:
                der["wait_any_share_of_wave_cycles"] = round(m["SQ_WAIT_ANY"] / m["SQ_WAVE_CYCLES"], 3)
        elif g:
            # gfx950: SQ_WAVE_CYCLES / SQ_ACTIVE_* count quad-cycles (MI355X_MICROARCH.md constants table)
            if "SQ_ACTIVE_INST_VALU" in m:
                der["VALUBusy_pct"] = round(100 * m["SQ_ACTIVE_INST_VALU"] / CU / g, 1)
            if "SQ_WAVE_CYCLES" in m:
                der["OccupancyPercent"] = round(400 * m["SQ_WAVE_CYCLES"] / g / CU / 32, 1)
            der["GRBM_GUI_ACTIVE_us_at_2.4GHz"] = round(g / 2400, 2)
        if "SQ_WAVE_CYCLES" in m and "SQ_WAIT_INST_ANY" in m:
            der["wait_inst_any_share_of_wave_cycles"] = round(m["SQ_WAIT_INST_ANY"] / m["SQ_WAVE_CYCLES"], 3)
        if "SQ_WAVE_CYCLES" in m and "SQ_ACTIVE_INST_ANY" in m:
            der["active_inst_any_share_of_wave_cycles"] = round(m["SQ_ACTIVE_INST_ANY"] / m["SQ_WAVE_CYCLES"], 3)
        out[short] = {"launches": len(next(iter(cs.values()))), "counters": {c: round(v, 1) for c, v in m.items()},
                      "derived": der}
    js = json.dumps(out, indent=1)
    print(js)
    if len(sys.argv) > 2:
        open(sys.argv[2], "w").write(js + "\n")


if __name__ == "__main__":
    main()
