#!/usr/bin/env python3
"""Per-wave timeline of the small-frame kernel from a -DDK_DIAG_STAMPS build (tuning tool).

    python tools/stamps.py build/variants/stamps.so [--workload c3_udp64]
Stamps per wave (s_memtime): 0 entry, 11 after the workgroup barrier, 1 after setup, per chunk k < 3: 2+3k frames in registers, 3+3k parsed +
probed + results stored, 4+3k counted; 14 before the counter flush, 15 exit; 12/13 s_memrealtime at entry/exit;
16+5k..19+5k: rx_finish sub-phases of chunk k (32 slots per wave). Prints quantiles of each
phase (µs) and the wave start/end spread over the launch.
"""
import argparse
import ctypes
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("lib")
    ap.add_argument("--workload", default="c3_udp64")
    ap.add_argument("--rotate", type=int, default=8)
    ap.add_argument("--grids", default="0", help="comma list of grid_per_cu values (0 = the engine's rule)")
    ap.add_argument("--mhz", type=float, default=0.0, help="s_memtime rate (0: calibrated against s_memrealtime)")
    args = ap.parse_args()
    import torch

    import bench
    from demikernel_amd import Config, RxEngine, synth

    e = RxEngine(Config(synth.BOB_IPV4), lib_path=os.path.abspath(args.lib))
    batch, flows, tr = bench.make_batch(e, args.workload, 0, synth.SEED, 1)
    rot = [batch] + [bench.make_batch(e, args.workload, 0, synth.SEED + 1000 * k, 1)[0] for k in range(1, args.rotate)]
    e.set_sockets(flows)
    r = e.results(batch.n)
    lib = e.lib
    lib.dk_diag_stamps_read.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint64]
    for it in range(20):
        e.receive_batch(rot[it % len(rot)], r)
    torch.cuda.synchronize()
    nw = 1 << 16  # waves covered by the stamp buffer (32 u64 each)
    for g in [int(x) for x in args.grids.split(",")]:
        e.set_tuning(grid_per_cu=g if g > 0 else -1)
        print(json.dumps({"grid_per_cu": g}))
        timeline(args, e, lib, rot, r, nw)
    lib.dk_diag_path_stats_enable(e._ctx, 0)


def timeline(args, e, lib, rot, r, nw):
    import torch

    for rep in range(2):
        assert lib.dk_diag_path_stats_enable(e._ctx, 1) == 0
        e.receive_batch(rot[(rep + 3) % len(rot)], r)
        torch.cuda.synchronize()
        st = np.zeros(nw * 32, dtype=np.uint64)
        assert lib.dk_diag_stamps_read(e._ctx, st.ctypes.data, st.size) == 0
        st = st.reshape(nw, 32).astype(np.int64)
        used = st[:, 0] != 0
        st = st[used]
        t0 = st[:, 12].min()
        rt = lambda x: x * 0.01  # noqa: E731  (s_memrealtime: 100 MHz ticks -> µs)
        mhz = args.mhz or float(np.median((st[:, 15] - st[:, 0]) / np.maximum(st[:, 13] - st[:, 12], 1) * 100.0))
        us = lambda x: x / mhz  # noqa: E731  (s_memtime: shader clock ticks -> µs)
        q = lambda a: [round(float(v), 2) for v in np.percentile(a, [0, 10, 50, 90, 100])]  # noqa: E731
        row = {"mhz": round(mhz, 1), "waves": int(used.sum()), "start": q(rt(st[:, 12] - t0)), "exit": q(rt(st[:, 13] - t0)),
               "setup": q(us(st[:, 1] - st[:, 0])), "to_barrier": q(us(st[:, 11] - st[:, 0])), "flush": q(us(st[:, 15] - st[:, 14]))}
        for k in range(3):
            have = st[:, 2 + 3 * k] != 0
            if not have.any():
                break
            s = st[have]
            prev = s[:, 1] if k == 0 else s[:, 4 + 3 * (k - 1)]
            row[f"c{k}"] = {"waves": int(have.sum()), "load": q(us(s[:, 2 + 3 * k] - prev)),
                            "finish": q(us(s[:, 3 + 3 * k] - s[:, 2 + 3 * k])),
                            "count": q(us(s[:, 4 + 3 * k] - s[:, 3 + 3 * k])),
                            "end_since_entry": q(us(s[:, 4 + 3 * k] - s[:, 0]))}
            b = 16 + 5 * k  # rx_finish sub-phases: parse, probe issue + segment sum, verdict + demux, results
            sub = [s[:, 2 + 3 * k], s[:, b], s[:, b + 1], s[:, b + 2], s[:, b + 3]]
            row[f"c{k}"]["sub"] = {nm: q(us(sub[j + 1] - sub[j]))[2] for j, nm in
                                   enumerate(("bigframes+parse", "probe_issue+segsum", "verdict+demux", "results"))}
        from stamps_staged import phase_totals

        row["totals"] = phase_totals(st, us, ("window", "parse+table+stores", "count", "general_pass", "combine",
                                              "barrier+rows"))
        print(json.dumps(row))


if __name__ == "__main__":
    main()
