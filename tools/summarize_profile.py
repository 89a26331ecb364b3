#!/usr/bin/env python3
"""Summarise the rocprofv3 outputs of tools/profile_bench.sh into profiles/ (committed evidence).

    python tools/summarize_profile.py <tag>
Writes profiles/<tag>_bench_kernel_stats.csv (verbatim kernel stats of the bench command), profiles/<tag>_pmc.csv
(per-kernel FETCH_SIZE / WRITE_SIZE averages) and profiles/pmc_traffic.json (per-launch HBM bytes bench.py reports as
roofline.traffic).

FETCH_SIZE unit on gfx950: the guide's rule (MI355X_MICROARCH.md §HBM) is that FETCH_SIZE reads 1/2 of the bytes of a
wide coalesced streaming read; we calibrate instead of assuming, with the read probe that runs in the same --pmc pass
over the same blob: factor = probe bytes / (probe FETCH_SIZE * 1024), applied to dk_rx_kernel's FETCH_SIZE.
WRITE_SIZE is reported as counted (exact for 16-B streaming stores per the guide; our 4-B-per-lane SoA stores are
uncalibrated).
"""
import csv
import json
import os
import shutil
import sys
from collections import defaultdict

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def counters(path):
    agg = defaultdict(list)
    for r in csv.DictReader(open(path)):
        agg[(r["Kernel_Name"], r["Counter_Name"])].append(float(r["Counter_Value"]))
    return {k: sum(v) / len(v) for k, v in agg.items()}


def kbench_info(path):
    rx, probe, tx = None, None, None
    for line in open(path):
        line = line.strip()
        if not line.startswith("{"):
            continue
        d = json.loads(line)
        if d.get("kernel") == "dk_rx":
            rx = d
        elif d.get("kernel") == "read_probe":
            probe = d
        elif d.get("kernel") in ("dk_tx", "dk_tx_fields"):
            tx = d
    return rx, probe, tx


def trace_summary(src):
    """Per kernel of each stats run: calls, mean, median and the mean without the first call (a run's first launch
    carries one-time costs: rocprofv3's stats average it in), from the kernel trace."""
    out = {}
    for sub in ("bench", "c3", "c1", "tx", "txf", "tcp"):
        f = os.path.join(src, sub, "run_kernel_trace.csv")
        if not os.path.exists(f):
            continue
        d = defaultdict(list)
        for r in csv.DictReader(open(f)):
            if r["Kernel_Name"].startswith("dk_"):
                d[r["Kernel_Name"]].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1000.0)
        out[sub] = {k: {"calls": len(v), "mean_us": round(sum(v) / len(v), 2),
                        "median_us": round(sorted(v)[len(v) // 2], 2),
                        "mean_after_first_us": round(sum(v[1:]) / max(len(v) - 1, 1), 2)} for k, v in d.items()}
    return out


def main():
    tag = sys.argv[1] if len(sys.argv) > 1 else "r01"
    src = os.path.join(ROOT, "gpurun_out", f"prof_{tag}")
    dst = os.path.join(ROOT, "profiles")
    os.makedirs(dst, exist_ok=True)
    stats = os.path.join(src, "bench", "run_kernel_stats.csv")
    if os.path.exists(stats):
        shutil.copy(stats, os.path.join(dst, f"{tag}_bench_kernel_stats.csv"))
    for sub in ("c3", "tx", "txf", "c1"):
        st = os.path.join(src, sub, "run_kernel_stats.csv")
        if os.path.exists(st):
            shutil.copy(st, os.path.join(dst, f"{tag}_{sub}_kernel_stats.csv"))
    tstats = os.path.join(src, "tcp", "run_kernel_stats.csv")
    if os.path.exists(tstats):
        shutil.copy(tstats, os.path.join(dst, f"{tag}_tcp_kernel_stats.csv"))
        shutil.copy(os.path.join(src, "tcp.json"), os.path.join(dst, f"{tag}_tcp_under_rocprof.json"))
    if os.path.exists(os.path.join(src, "bench.json")):
        shutil.copy(os.path.join(src, "bench.json"), os.path.join(dst, f"{tag}_bench_under_rocprof.json"))
    ts = trace_summary(src)
    if ts:
        json.dump(ts, open(os.path.join(dst, f"{tag}_kernel_trace_summary.json"), "w"), indent=1)
    traffic = {}
    rows = [["workload", "kernel", "FETCH_SIZE_KB", "WRITE_SIZE_KB", "calib_factor", "hbm_read_bytes",
             "hbm_write_bytes", "algo_bytes", "traffic_over_algo"]]
    for wl in ("c2_tcp1500", "c3_udp64", "c4_imix", "c5_tcp1500_10k", "c1_tcp1078", "c3_udp64_random_ports",
               "c2_tcp1500_libos", "c2_tcp1500_txf"):
        fdir, wdir = os.path.join(src, f"fetch_{wl}"), os.path.join(src, f"write_{wl}")
        if not os.path.exists(os.path.join(fdir, "run_counter_collection.csv")):
            continue
        fc = counters(os.path.join(fdir, "run_counter_collection.csv"))
        wc = counters(os.path.join(wdir, "run_counter_collection.csv"))
        rx, probe, tx = kbench_info(os.path.join(src, f"fetch_{wl}.log"))
        fk = {k[0]: v for k, v in fc.items() if k[1] == "FETCH_SIZE"}
        wk = {k[0]: v for k, v in wc.items() if k[1] == "WRITE_SIZE"}
        rxk = next(k for k in fk if "dk_rx_kernel" in k or "dk_rx_split_kernel" in k or "dk_rx_small_kernel" in k)
        rxname = next(nm for nm in ("dk_rx_split_kernel", "dk_rx_small_kernel", "dk_rx_kernel") if nm in rxk)
        pk = next(k for k in fk if "read_probe" in k)
        factor = probe["bytes"] / (fk[pk] * 1024.0)
        rd = fk[rxk] * 1024.0 * factor
        wr = wk.get(rxk, 0.0) * 1024.0
        algo = rx["algo_bytes"]
        if not wl.endswith("_txf"):  # the fields-form pass repeats c2_tcp1500's receive: only its TX kernel is new
            traffic[wl] = {"hbm_bytes_per_launch": int(rd + wr), "hbm_read_bytes": int(rd),
                           "hbm_write_bytes": int(wr), "kernel": rxname, "fetch_size_kb_raw": fk[rxk],
                           "write_size_kb_raw": wk.get(rxk, 0.0), "fetch_calibration_factor": round(factor, 4),
                           "algorithmic_bytes_per_launch": algo,
                           "source": f"profiles/{tag}_pmc.csv (rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE, "
                                     "separate passes)"}
        rows.append([wl, rxname, f"{fk[rxk]:.0f}", f"{wk.get(rxk, 0.0):.0f}", f"{factor:.4f}", f"{rd:.0f}",
                     f"{wr:.0f}", algo, f"{(rd + wr) / algo:.3f}"])
        rows.append([wl, "read_probe", f"{fk[pk]:.0f}", f"{wk.get(pk, 0.0):.0f}", "", probe["bytes"], "", "", ""])
        txk = next((k for k in fk if "dk_tx_kernel" in k or "dk_tx_split_kernel" in k), None)
        txname = "dk_tx_split_kernel" if txk and "split" in txk else "dk_tx_kernel"
        if tx and tx["kernel"] == "dk_tx_fields":
            txname += "<fields>"
        if tx and txk:
            trd, twr = fk[txk] * 1024.0 * factor, wk.get(txk, 0.0) * 1024.0
            traffic[wl + "_tx"] = {"hbm_bytes_per_launch": int(trd + twr), "hbm_read_bytes": int(trd),
                                   "hbm_write_bytes": int(twr), "fetch_calibration_factor": round(factor, 4),
                                   "algorithmic_bytes_per_launch": tx["algo_bytes"],
                                   "kernel": txname, "source": f"profiles/{tag}_pmc.csv ({txname})"}
            rows.append([wl, txname, f"{fk[txk]:.0f}", f"{wk.get(txk, 0.0):.0f}", f"{factor:.4f}",
                         f"{trd:.0f}", f"{twr:.0f}", tx["algo_bytes"], f"{(trd + twr) / tx['algo_bytes']:.3f}"])
    with open(os.path.join(dst, f"{tag}_pmc.csv"), "w", newline="") as f:
        csv.writer(f).writerows(rows)
    json.dump(traffic, open(os.path.join(dst, "pmc_traffic.json"), "w"), indent=1)
    print(json.dumps(traffic, indent=1))


if __name__ == "__main__":
    main()
