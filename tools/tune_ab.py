#!/usr/bin/env python3
"""Interleaved A/B of tuning configurations (dk_diag_rx_set_tuning knobs) on one workload, in ONE process.

    python tools/tune_ab.py --workload c1_tcp1078 --rotate 3 "split=1" "split=0,stage=1" "split=0,stage=0,grid_per_cu=4"
Each configuration ("" = the host rule; pseudo-knob defer=1: deferred counters, one flush per timed block) is timed `--iters` launches per repetition, repetitions interleaved; one JSON
line per configuration with the median ms per launch and the roofline fraction of the algorithmic bytes.
--lib times a variant libdk_rx.so (tools/variants.sh); several --lib values interleave builds too.
"""
import argparse
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def parse_cfg(s):
    out = {}
    for kv in filter(None, s.split(",")):
        k, v = kv.split("=")
        out[k.strip()] = int(v)
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("configs", nargs="*", default=[""])
    ap.add_argument("--workload", default="c2_tcp1500")
    ap.add_argument("--rotate", type=int, default=1)
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--reps", type=int, default=7)
    ap.add_argument("--frames", type=int, default=0)
    ap.add_argument("--lib", action="append", default=[])
    ap.add_argument("--tcp-fields", action="store_true", help="results with tcp_seq/ack/win and tcp_opts")
    ap.add_argument("--no-counts", action="store_true")
    args = ap.parse_args()
    import torch

    import bench
    from demikernel_amd import Config, RxEngine, synth

    base = RxEngine(Config(synth.BOB_IPV4))
    made = [bench.make_batch(base, args.workload, 0, synth.SEED + 1000 * k, 1, frames=args.frames)
            for k in range(args.rotate)]
    batches = [m[0] for m in made]
    _, flows, tr = made[0]
    n = batches[0].n
    libs = args.lib or [None]
    engines = []
    for lp in libs:
        e = RxEngine(Config(synth.BOB_IPV4), lib_path=os.path.abspath(lp) if lp else None)
        e.set_sockets(flows)
        r = e.results(n, tcp_fields=args.tcp_fields, tcp_opts=args.tcp_fields, counts=not args.no_counts)
        engines.append((os.path.basename(lp)[:-3] if lp else "head", e, r))
    fb = int(tr.frame_len.astype(np.int64).sum())
    rb = bench.RESULT_BYTES + (12 if args.tcp_fields else 0)
    algo = fb + n * (bench.DESC_BYTES + rb)
    cfgs = [(c, parse_cfg(c)) for c in args.configs]
    times = {(en, c): [] for en, _, _ in engines for c, _ in cfgs}
    s = torch.cuda.current_stream()
    bench.preheat(engines[0][1], batches[0], s, 0.25)
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    for _ in range(args.reps):
        for c, kn in cfgs:
            kn = dict(kn)
            defer = bool(kn.pop("defer", 0))  # pseudo-knob: DK_RX_BATCH_DEFER_COUNTS + one flush per timed block
            for en, e, r in engines:
                e.set_tuning(**kn)
                e.receive_batch(batches[0], r)
                ev0.record()
                for it in range(args.iters):
                    e.receive_batch(batches[it % len(batches)], r, defer_counts=defer)
                if defer:
                    e.flush_counts()
                ev1.record()
                torch.cuda.synchronize()
                times[(en, c)].append(ev0.elapsed_time(ev1) / args.iters)
    for (en, c), ts in times.items():
        ms = float(np.median(ts))
        print(json.dumps({"lib": en, "tuning": c or "host rule", "workload": args.workload, "ms": round(ms, 4),
                          "frac": round(algo / ms / 1e6 / bench.HBM_PEAK_GBS, 4),
                          "spread": round((max(ts) - min(ts)) / ms, 3)}), flush=True)


if __name__ == "__main__":
    main()
