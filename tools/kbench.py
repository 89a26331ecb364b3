#!/usr/bin/env python3
"""Kernel-level timing for tuning: dk_rx kernel on a workload vs the on-box streaming-read probe over the same blob.

    python tools/kbench.py [--workload c2_tcp1500] [--iters 50] [--probe]
Prints one JSON line per measurement. Also the command profiled by rocprofv3 (profiles/README.md).
"""
from __future__ import annotations

import argparse
import ctypes
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def time_events(fn, iters, warm=3):
    import torch

    for _ in range(warm):
        fn()
    torch.cuda.synchronize()
    a = torch.cuda.Event(enable_timing=True)
    b = torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(iters):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / 1e3 / iters


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--workload", default="c2_tcp1500")
    ap.add_argument("--iters", type=int, default=50)
    ap.add_argument("--probe", action="store_true")
    ap.add_argument("--probe-one", action="store_true", help="one probe config (mode 1, grid 1024): PMC calibration")
    ap.add_argument("--no-rx", action="store_true")
    ap.add_argument("--tx", action="store_true", help="also time dk_tx_checksum (rewrites the batch's checksums)")
    ap.add_argument("--tx-fields", action="store_true",
                    help="also time dk_tx_checksum_fields (the checksum pair returned, frames untouched)")
    ap.add_argument("--no-counts", action="store_true", help="pass NULL flow/verdict counters (cost attribution)")
    ap.add_argument("--modes", default="3,4,6,7,8")
    ap.add_argument("--grids", default="256,512,768,1024")
    ap.add_argument("--rotate", type=int, default=1, help="distinct batches cycled per launch (C3: 8, past the MALL)")
    ap.add_argument("--lib", default=None, help="a variant libdk_rx.so (tools/variants.sh) instead of the in-tree one")
    ap.add_argument("--tcp-fields", action="store_true", help="the LibOS record: + tcp_seq/ack/win and tcp_opts")
    ap.add_argument("--defer", action="store_true", help="deferred counters (DK_RX_BATCH_DEFER_COUNTS), as bench.py runs")
    args = ap.parse_args()

    import torch

    import bench
    from demikernel_amd import Config, RxEngine, synth
    from demikernel_amd import _native as N
    eng = RxEngine(Config(synth.BOB_IPV4), lib_path=os.path.abspath(args.lib) if args.lib else None)
    batch, flows, tr = bench.make_batch(eng, args.workload, 0, synth.SEED, 1)
    rot = [batch] + [bench.make_batch(eng, args.workload, 0, synth.SEED + 1000 * k, 1)[0] for k in range(1, args.rotate)]
    res = eng.results(batch.n, counts=not args.no_counts, tcp_fields=args.tcp_fields, tcp_opts=args.tcp_fields)
    it = [0]

    def next_batch():
        it[0] += 1
        return rot[it[0] % len(rot)]
    fb = int(tr.frame_len.astype(np.int64).sum())
    if not args.no_rx:
        t = time_events(lambda: eng.receive_batch(next_batch(), res, defer_counts=args.defer), args.iters)
        eng.flush_counts()
        algo = fb + batch.n * (bench.DESC_BYTES + bench.RESULT_BYTES + (12 if args.tcp_fields else 0))
        print(json.dumps({"kernel": "dk_rx", "workload": args.workload, "counts": not args.no_counts,
                          "frames": batch.n, "frame_bytes": fb, "algo_bytes": algo, "blob_bytes": batch.blob.numel(),
                          "ms": round(t * 1e3, 4),
                          "frame_GBps": round(fb / t / 1e9, 1), "algo_GBps": round(algo / t / 1e9, 1),
                          "mpkt_s": round(batch.n / t / 1e6, 1)}), flush=True)
    if args.tx:
        t = time_events(lambda: eng.tx_checksum(batch), args.iters)
        algo = fb + batch.n * (bench.DESC_BYTES + 4)
        print(json.dumps({"kernel": "dk_tx", "workload": args.workload, "frames": batch.n, "frame_bytes": fb,
                          "algo_bytes": algo, "ms": round(t * 1e3, 4), "frame_GBps": round(fb / t / 1e9, 1),
                          "algo_GBps": round(algo / t / 1e9, 1)}), flush=True)
    if args.tx_fields:
        fields = torch.empty(batch.n, dtype=torch.int32, device=batch.off.device)
        t = time_events(lambda: eng.tx_checksum_fields(batch, fields), args.iters)
        algo = fb + batch.n * (bench.DESC_BYTES + 4)
        print(json.dumps({"kernel": "dk_tx_fields", "workload": args.workload, "frames": batch.n, "frame_bytes": fb,
                          "algo_bytes": algo, "ms": round(t * 1e3, 4), "frame_GBps": round(fb / t / 1e9, 1),
                          "algo_GBps": round(algo / t / 1e9, 1)}), flush=True)
    if args.probe or args.probe_one:
        lib = N.load_library()
        nbytes = batch.blob.numel() // 16 * 16
        for mode in ((1,) if args.probe_one else tuple(int(m) for m in args.modes.split(','))):
            for grid in ((1024,) if args.probe_one else tuple(int(g) for g in args.grids.split(','))):
                scratch = torch.zeros(grid, dtype=torch.int32, device="cuda")
                s = torch.cuda.current_stream().cuda_stream

                def run():
                    lib.dk_diag_read_probe(ctypes.c_void_p(batch.blob.data_ptr()), nbytes,
                                           ctypes.c_void_p(scratch.data_ptr()), grid, mode, ctypes.c_void_p(s))

                t = time_events(run, args.iters)
                print(json.dumps({"kernel": "read_probe", "mode": mode, "grid": grid, "bytes": nbytes,
                                  "ms": round(t * 1e3, 4), "GBps": round(nbytes / t / 1e9, 1)}), flush=True)


if __name__ == "__main__":
    main()
