#!/usr/bin/env python3
"""Does the counters' collective overlap the receive kernel?

    python tools/overlap_collective.py [--out profiles/r04_overlap.json]
On one GPU, with a 1-rank RCCL communicator (dk_comm_init_all over device 0), ShardedReceiver steps at C2 and the C4
IMIX shard are timed in one process, interleaved: no collective (comm=None, what N = 1 runs), the all-reduce after
every step (deferred counter rows, and without deferral), after every 8 steps, and after every step with 8 CUs left
free of the receive kernel. If the persistent kernels keep RCCL's kernel from running beside them, a step grows by
the collective's own time (measured alone too).
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=32)
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--out", default="")
    args = ap.parse_args()
    import torch

    import bench
    from demikernel_amd import Comm, Config, RxEngine, synth
    from demikernel_amd.shard import ShardedReceiver

    comm = Comm.init_all([0])[0]
    stream = torch.cuda.current_stream()
    out = {"what": __doc__.strip().splitlines()[0], "gpu": torch.cuda.get_device_name(0), "steps": args.steps,
           "reps": args.reps, "workloads": {}}
    for wl in ("c2_tcp1500", "c4_imix"):
        eng = RxEngine(Config(synth.BOB_IPV4))
        batch, flows, tr = bench.make_batch(eng, wl, 0, synth.SEED)
        res = eng.results(batch.n)
        cus = torch.cuda.get_device_properties(0).multi_processor_count
        per_cu = 1 if wl == "c2_tcp1500" else 3  # split kernel / staged kernel (rx_host.cpp launch_batch)
        # mode: (communicator, deferred counters, gather every K steps, CUs left free for RCCL's kernel)
        # mode: (communicator, deferred counters, gather every K steps, CUs left free, collective on a side stream)
        modes = {"no_collective": (None, True, 1, 0, True), "rccl_every_step": (comm, True, 1, 0, True),
                 "rccl_every_step_no_defer": (comm, False, 1, 0, True), "rccl_every_8": (comm, True, 8, 0, True),
                 "rccl_every_8_same_stream": (comm, True, 8, 0, False),
                 "rccl_every_16": (comm, True, 16, 0, True),
                 "rccl_every_16_same_stream": (comm, True, 16, 0, False),
                 "rccl_every_step_same_stream": (comm, True, 1, 0, False),
                 "rccl_every_step_8_cus_free": (comm, True, 1, 8, True)}
        t = {m: [] for m in modes}
        bench.preheat(eng, batch, stream, 0.25)
        for _ in range(args.reps):
            for m, (cm, defer, every, free, side) in modes.items():
                eng.set_tuning(grid=(cus - free) * per_cu if free else -1)
                sr = ShardedReceiver(eng, res, cm, stream, defer=defer, gather_every=every, side_stream=side)
                for _ in range(3):
                    sr.step(batch)
                sr.drain()
                torch.cuda.synchronize()
                t0 = time.perf_counter()
                for _ in range(args.steps):
                    sr.step(batch)
                sr.drain()
                torch.cuda.synchronize()
                t[m].append((time.perf_counter() - t0) / args.steps * 1e3)
                if cm is not None:
                    fo, vo = sr.counts()
                    assert int(vo.sum()) == (args.steps + 3) * batch.n, (m, int(vo.sum()))
        eng.set_tuning()
        sr = ShardedReceiver(eng, res, comm, stream)
        coll = []
        for _ in range(10):
            c0, c1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            c0.record(sr.side)
            sr.reduce(0, sr.side)
            c1.record(sr.side)
            torch.cuda.synchronize()
            coll.append(c0.elapsed_time(c1))
        out["workloads"][wl] = {"frames": batch.n, "flows": len(flows),
                                "step_ms_median": {m: round(float(np.median(v)), 4) for m, v in t.items()},
                                "step_ms_all": {m: [round(x, 4) for x in v] for m, v in t.items()},
                                "collective_alone_ms_median": round(float(np.median(coll)), 4)}
        print(json.dumps({wl: out["workloads"][wl]["step_ms_median"],
                          "collective_alone_ms": out["workloads"][wl]["collective_alone_ms_median"]}), flush=True)
        del eng, batch, res
    comm.destroy()
    if args.out:
        json.dump(out, open(args.out, "w"), indent=1)


if __name__ == "__main__":
    main()
