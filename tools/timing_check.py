#!/usr/bin/env python3
"""Tuning tool: the same receive launches timed two ways in one process, alternately — bench.time_kernel (the bench's
ShardedReceiver path, events around the timed region) and a bare loop of receive_batch calls (tools/abtest.py's way)
— to tell a methodology difference from a kernel difference."""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--workload", default="c4_imix")
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--preheat-ms", type=float, default=0.0, help="device-to-device copies on OTHER buffers first")
    args = ap.parse_args()
    import torch

    import bench
    from demikernel_amd import Config, RxEngine, synth

    eng = RxEngine(Config(synth.BOB_IPV4))
    batch, flows, tr = bench.make_batch(eng, args.workload, 0, synth.SEED, 1)
    stream = torch.cuda.current_stream()
    res = eng.results(batch.n)
    if args.preheat_ms > 0:  # GPU busy on unrelated memory: clocks ramp, this batch's pages stay untouched
        a = torch.empty(1 << 28, dtype=torch.uint8, device="cuda")
        b = torch.empty_like(a)
        torch.cuda.synchronize()
        import time
        t = time.perf_counter()
        while (time.perf_counter() - t) * 1e3 < args.preheat_ms:
            for _ in range(8):
                b.copy_(a)
            torch.cuda.synchronize()
    for rep in range(args.reps):
        _, kern, _, _ = bench.time_kernel(eng, [batch], res, args.steps, 5, stream)
        eng.receive_batch(batch, res)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(args.steps):
            eng.receive_batch(batch, res)
        e1.record()
        torch.cuda.synchronize()
        loop = e0.elapsed_time(e1) / 1e3 / args.steps
        torch.cuda.synchronize()
        t0 = torch.cuda.Event(enable_timing=True)
        t1 = torch.cuda.Event(enable_timing=True)
        t0.record()
        for _ in range(args.steps):
            eng.receive_batch(batch, res)
        t1.record()
        torch.cuda.synchronize()
        cold = t0.elapsed_time(t1) / 1e3 / args.steps
        print(json.dumps({"rep": rep, "time_kernel_us": round(kern * 1e6, 1), "loop_warm_us": round(loop * 1e6, 1),
                          "loop_after_sync_us": round(cold * 1e6, 1)}), flush=True)


if __name__ == "__main__":
    main()
