#!/usr/bin/env python3
"""Interleaved A/B timing of several libdk_rx.so builds in ONE process on the same batch (tuning tool).

    python tools/abtest.py --workload c2_tcp1500 --grids 2,3,4 build/variants/*.so
Each (variant, grid) is timed `--iters` launches per repetition, repetitions interleaved; prints the median ms.
"""
import argparse
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("variants", nargs="+")
    ap.add_argument("--workload", default="c2_tcp1500")
    ap.add_argument("--grids", default="2,3,4")
    ap.add_argument("--iters", type=int, default=10)
    ap.add_argument("--reps", type=int, default=7)
    ap.add_argument("--scheds", default="", help="comma list of sched knob values to interleave (default: host rule)")
    ap.add_argument("--knob", default="", help="NAME=v1,v2,...: interleave values of one more dk_diag_rx_set_tuning knob (e.g. DK_RX_SPLIT=0,1)")
    ap.add_argument("--tx", action="store_true", help="time dk_tx_checksum instead of the receive kernel")
    ap.add_argument("--rotate", type=int, default=1, help="distinct batches cycled per launch (C3: 8, past the MALL)")
    ap.add_argument("--frames", type=int, default=0, help="frames per batch (0: the workload's own)")
    ap.add_argument("--defer", action="store_true", help="deferred counters (DK_RX_BATCH_DEFER_COUNTS), as bench.py runs")
    ap.add_argument("--check", action="store_true", help="also compare every variant's results and counters with the "
                                                          "first variant's on one fresh launch")
    args = ap.parse_args()
    import torch

    import bench
    from demikernel_amd import Config, RxEngine, synth
    from demikernel_amd import _native as N

    base = RxEngine(Config(synth.BOB_IPV4))
    batch, flows, tr = bench.make_batch(base, args.workload, 0, synth.SEED, 1, frames=args.frames)
    rot = [batch] + [bench.make_batch(base, args.workload, 0, synth.SEED + 1000 * k, 1, frames=args.frames)[0]
                     for k in range(1, args.rotate)]
    engines = {}
    for v in args.variants:
        e = RxEngine(Config(synth.BOB_IPV4), lib_path=os.path.abspath(v))
        e.set_sockets(flows)
        engines[os.path.basename(v)[:-3]] = (e, e.results(batch.n))
    fb = int(tr.frame_len.astype(np.int64).sum())
    algo = fb + batch.n * (bench.DESC_BYTES + bench.RESULT_BYTES)
    grids = [int(g) for g in args.grids.split(",")]
    scheds = args.scheds.split(",") if args.scheds else [None]
    kname, kvals = (args.knob.split("=")[0], args.knob.split("=")[1].split(",")) if args.knob else ("", [None])
    configs = [(sc, kv) for sc in scheds for kv in kvals]
    times = {(k, g, cf): [] for k in engines for g in grids for cf in configs}
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    if not args.tx:  # untimed clock ramp (bench.preheat): the first ~10 ms of a fresh process run slow
        e0, r0 = next(iter(engines.values()))
        bench.preheat(e0, batch, torch.cuda.current_stream(), 0.25)
    for rep in range(args.reps):
        for g, cf in [(g, cf) for g in grids for cf in configs]:
            sc, kv = cf
            knobs = {"grid_per_cu": g if g > 0 else -1}
            if sc is not None:
                knobs["sched"] = int(sc)
            if kv is not None and kname.startswith("DK_RX_") and kname[6:].lower() in N.DK_DIAG_RX_KNOBS:
                knobs[kname[6:].lower()] = int(kv)
            for k, (e, r) in engines.items():
                e.set_tuning(**knobs)
                run = ((lambda b: e.tx_checksum(b)) if args.tx else  # noqa: E731
                       (lambda b: e.receive_batch(b, r, defer_counts=args.defer)))
                run(batch)
                ev0.record()
                for it in range(args.iters):
                    run(rot[it % len(rot)])
                ev1.record()
                torch.cuda.synchronize()
                times[(k, g, cf)].append(ev0.elapsed_time(ev1) / args.iters)
    if args.check and not args.tx:
        ref = None
        for k, (e, _) in engines.items():
            e.set_tuning()
            r = e.results(batch.n)
            e.receive_batch(batch, r)
            torch.cuda.synchronize()
            got = r.to_numpy()
            if ref is None:
                ref = (k, got)
                continue
            bad = [f for f in got if not np.array_equal(np.asarray(got[f]), np.asarray(ref[1][f]))]
            print(json.dumps({"check": k, "vs": ref[0], "mismatched": bad}), flush=True)
            if bad:
                sys.exit(5)
    for (k, g, cf), ts in sorted(times.items(), key=lambda x: (x[0][1], str(x[0][2]), x[0][0])):
        ms = float(np.median(ts))
        name = k if cf[1] is None else f"{k}[{kname}={cf[1]}]"
        print(json.dumps({"variant": name, "grid_per_cu": g, "sched": cf[0], "workload": args.workload, "tx": args.tx, "ms": round(ms, 4),
                          "algo_GBps": round(algo / ms / 1e6, 1), "spread": round((max(ts) - min(ts)) / ms, 3)}))


if __name__ == "__main__":
    main()
