#!/usr/bin/env python3
"""Fixed vs per-frame cost of a receive kernel: the same workload at several batch sizes, each
size with `--rotate` distinct batches cycled (past the 256 MB MALL), launched back to back as bench.py's steps are
(deferred counter rows completed by the next launch), µs per launch from HIP events around `--iters` launches,
sizes interleaved over `--reps` repetitions (median). A least-squares line through (frames, µs) gives the launch's
fixed µs (intercept) and ns per frame (slope); the slope is also shown as TB/s of algorithmic bytes.

    python tools/sweep.py --workload c3_udp64 --frames 1M,2M,4M,8M --rotate 8
    python tools/sweep.py --workload c4_imix --frames 512K,1M,2M,4M --rotate 2
One JSON line per size, then one with the fit. --lib times another build (tools/variants.sh); --tuning passes
dk_diag_rx_set_tuning knobs (name=value,...).
"""
from __future__ import annotations

import argparse
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def parse_n(s: str) -> int:
    s = s.strip().upper()
    mul = {"K": 1 << 10, "M": 1 << 20}.get(s[-1], 1)
    return int(float(s[:-1] if s[-1] in "KM" else s) * mul)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--workload", default="c3_udp64")
    ap.add_argument("--frames", default="1M,2M,4M,8M")
    ap.add_argument("--rotate", type=int, default=8)
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--lib", default=None)
    ap.add_argument("--tuning", default="", help="dk_diag_rx_set_tuning knobs, e.g. grid_per_cu=2,tail=0")
    ap.add_argument("--tag", default="")
    ap.add_argument("--no-counts", action="store_true", help="no flow / verdict counters (cost attribution)")
    args = ap.parse_args()
    import torch

    import bench
    from demikernel_amd import Config, RxEngine, synth

    knobs = {k: int(v) for k, v in (kv.split("=") for kv in args.tuning.split(",") if kv)}
    sizes = [parse_n(s) for s in args.frames.split(",")]
    stream = torch.cuda.current_stream()
    runs = []
    for n in sizes:
        eng = RxEngine(Config(synth.BOB_IPV4), device=0, lib_path=os.path.abspath(args.lib) if args.lib else None,
                       tuning=knobs or None)
        made = [bench.make_batch(eng, args.workload, 0, synth.SEED + 1000 * k, 1, frames=n) for k in range(args.rotate)]
        batches = [m[0] for m in made]
        tr = made[0][2]
        fb = int(tr.frame_len.astype(np.int64).sum())
        algo = fb + n * (bench.DESC_BYTES + bench.RESULT_BYTES)
        res = eng.results(n, counts=not args.no_counts)
        runs.append({"n": n, "eng": eng, "batches": batches, "res": res, "algo": algo, "fb": fb, "t": []})
    bench.preheat(runs[0]["eng"], runs[0]["batches"][0], stream, 0.3)
    for rep in range(args.reps):
        for R in runs:
            eng, bs, res = R["eng"], R["batches"], R["res"]
            for k in range(3):
                eng.receive_batch(bs[k % len(bs)], res, stream=stream, defer_counts=True)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(stream)
            for k in range(args.iters):
                eng.receive_batch(bs[k % len(bs)], res, stream=stream, defer_counts=True)
            e1.record(stream)
            eng.flush_counts(stream)
            torch.cuda.synchronize()
            R["t"].append(e0.elapsed_time(e1) * 1e3 / args.iters)
    xs, ys = [], []
    for R in runs:
        us = float(np.median(R["t"]))
        xs.append(R["n"])
        ys.append(us)
        print(json.dumps({"tag": args.tag, "workload": args.workload, "frames": R["n"], "rotate": args.rotate,
                          "us_per_launch": round(us, 3), "us_spread": [round(min(R["t"]), 3), round(max(R["t"]), 3)],
                          "algo_bytes": R["algo"], "algo_TBps": round(R["algo"] / us / 1e6, 3),
                          "frac": round(R["algo"] / us / 1e6 / 8.0, 4), "tuning": knobs,
                          "counts": not args.no_counts}), flush=True)
    A = np.vstack([np.ones(len(xs)), np.asarray(xs, float)]).T
    (a, b), *_ = np.linalg.lstsq(A, np.asarray(ys), rcond=None)
    per_frame_bytes = runs[-1]["algo"] / runs[-1]["n"]
    resid = np.asarray(ys) - A @ np.array([a, b])
    print(json.dumps({"tag": args.tag, "workload": args.workload, "fit": "us = a + b * frames",
                      "fixed_us": round(float(a), 3), "ns_per_frame": round(float(b) * 1e3, 5),
                      "slope_TBps": round(per_frame_bytes / (float(b) * 1e6), 3),
                      "max_resid_us": round(float(np.abs(resid).max()), 3), "tuning": knobs}), flush=True)


if __name__ == "__main__":
    main()
