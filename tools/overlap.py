#!/usr/bin/env python3
"""Feasibility probe for a size-binned IMIX schedule (tuning tool): do the minimum-size-frame kernel and a large-frame
kernel overlap when they run side by side on two streams with grids that let both be resident?

    python tools/overlap.py [--small-per-cu 1] [--big-per-cu 2] [--big-kernel staged|split]
Times (HIP events, median of reps) the C3-like part (IMIX's small frames: 1.22M x 64 B) and the C2-like part
(IMIX's big-frame bytes: 0.49M x 1500 B) alone at those grids and together on two streams.
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
    ap.add_argument("--small-per-cu", type=int, default=1)
    ap.add_argument("--big-per-cu", type=int, default=2)
    ap.add_argument("--big-kernel", default="staged")
    ap.add_argument("--reps", type=int, default=9)
    ap.add_argument("--iters", type=int, default=8)
    args = ap.parse_args()
    import torch

    from demikernel_amd import Config, RxEngine, synth

    def batch(eng, n, ip_len, kind, nflows, seed):
        flows = synth.make_flows(nflows, kind=kind)
        tr = synth.traffic(n, np.full(n, ip_len, np.uint16), flows, seed=seed)
        eng.set_sockets(flows)
        return synth.build_device(tr, eng, seed=seed)

    es = RxEngine(Config(synth.BOB_IPV4))
    eb = RxEngine(Config(synth.BOB_IPV4))
    bs = batch(es, 1_220_000, 50, "udp", 1024, 3)
    bb = batch(eb, 490_000, 1486, "tcp", 1024, 4)
    rs, rb = es.results(bs.n), eb.results(bb.n)
    es.set_tuning(small=1, grid_per_cu=args.small_per_cu)
    eb.set_tuning(small=0, stage=1, split=1 if args.big_kernel == "split" else 0, grid_per_cu=args.big_per_cu)
    s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(4)]

    def timed(fn):
        ts = []
        for _ in range(args.reps):
            torch.cuda.synchronize()
            ev[0].record(s1)
            s2.wait_event(ev[0])
            for _ in range(args.iters):
                fn()
            ev[1].record(s1)
            ev[2].record(s2)
            s1.wait_event(ev[2])
            ev[3].record(s1)
            torch.cuda.synchronize()
            ts.append(ev[0].elapsed_time(ev[3]) / args.iters * 1e3)
        return round(float(np.median(ts)), 1)

    small = timed(lambda: es.receive_batch(bs, rs, stream=s1))
    big = timed(lambda: eb.receive_batch(bb, rb, stream=s2))

    def both():
        es.receive_batch(bs, rs, stream=s1)
        eb.receive_batch(bb, rb, stream=s2)
    together = timed(both)
    print(json.dumps({"small_per_cu": args.small_per_cu, "big_per_cu": args.big_per_cu, "big_kernel": args.big_kernel,
                      "small_us": small, "big_us": big, "together_us": together,
                      "sum_us": round(small + big, 1), "max_us": max(small, big)}))


if __name__ == "__main__":
    main()
