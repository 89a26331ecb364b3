#!/usr/bin/env python3
"""Per-wave timeline of the staged receive kernel (dk_rx_kernel) from a -DDK_DIAG_STAMPS build (tuning tool).

    python tools/stamps_staged.py build/variants/stamps.so [--workload c1_tcp1078] [--rotate 3]
--tuning tail=0 etc. sets dk_diag_rx_set_tuning knobs. Stamps per wave (s_memtime unless noted): 0 entry, 1 after the LDS init / table copy / barrier, per chunk k < 3:
2+3k before phase A+B, 3+3k after it, 4+3k after phase C; 11 after the loop, 14 after the staged flush and the pending
combine, 15 after the barrier and the counter rows; 12/13 s_memrealtime at entry/exit. Prints quantiles (µs)."""
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
    ap.add_argument("--workload", default="c1_tcp1078")
    ap.add_argument("--rotate", type=int, default=3)
    ap.add_argument("--tuning", default="", help="dk_diag_rx_set_tuning knobs, e.g. tail=0")
    args = ap.parse_args()
    import torch

    import bench
    from demikernel_amd import Config, RxEngine, synth

    e = RxEngine(Config(synth.BOB_IPV4), lib_path=os.path.abspath(args.lib))
    made = [bench.make_batch(e, args.workload, 0, synth.SEED + 1000 * k, 1) for k in range(args.rotate)]
    rot = [m[0] for m in made]
    e.set_sockets(made[0][1])
    if args.tuning:
        e.set_tuning(**{k: int(v) for k, v in (kv.split("=") for kv in args.tuning.split(","))})
    r = e.results(rot[0].n)
    lib = e.lib
    lib.dk_diag_stamps_read.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint64]
    for it in range(30):
        e.receive_batch(rot[it % len(rot)], r, defer_counts=True)
    e.flush_counts()
    torch.cuda.synchronize()
    nw = 1 << 16
    q = lambda a: [round(float(v), 2) for v in np.percentile(a, [0, 10, 50, 90, 100])]  # noqa: E731
    for rep in range(3):
        assert lib.dk_diag_path_stats_enable(e._ctx, 1) == 0
        e.receive_batch(rot[rep % len(rot)], r, defer_counts=True)
        torch.cuda.synchronize()
        st = np.zeros(nw * 32, dtype=np.uint64)
        assert lib.dk_diag_stamps_read(e._ctx, st.ctypes.data, st.size) == 0
        st = st.reshape(nw, 32).astype(np.int64)
        st = st[st[:, 0] != 0]
        t0 = st[:, 12].min()
        mhz = float(np.median((st[:, 15] - st[:, 0]) / np.maximum(st[:, 13] - st[:, 12], 1) * 100.0))
        us = lambda x: x / mhz  # noqa: E731
        row = {"waves": len(st), "mhz": round(mhz, 1), "start": q((st[:, 12] - t0) * 0.01),
               "exit": q((st[:, 13] - t0) * 0.01), "setup": q(us(st[:, 1] - st[:, 0])),
               "exit_spread_us": round(float(st[:, 13].max() - st[:, 13].min()) * 0.01, 2),
               "exit_p10_to_max_us": round(float(st[:, 13].max() - np.percentile(st[:, 13], 10)) * 0.01, 2),
               "tuning": args.tuning}
        for k in range(3):
            have = st[:, 2 + 3 * k] != 0
            if not have.any():
                break
            s = st[have]
            prev = s[:, 1] if k == 0 else s[:, 4 + 3 * (k - 1)]
            row[f"c{k}"] = {"waves": int(have.sum()), "desc+gap": q(us(s[:, 2 + 3 * k] - prev)),
                            "stream": q(us(s[:, 3 + 3 * k] - s[:, 2 + 3 * k])),
                            "phaseC": q(us(s[:, 4 + 3 * k] - s[:, 3 + 3 * k])),
                            "end_since_entry": q(us(s[:, 4 + 3 * k] - s[:, 0]))}
        row["totals"] = phase_totals(st, us, ("to_stream_end", "phaseC", "stage+flush", "count", "last_flush",
                                              "combine"))
        row["loop_end_to_flush"] = q(us(st[:, 14] - st[:, 11]))
        row["barrier+rows"] = q(us(st[:, 15] - st[:, 14]))
        row["entry_to_exit"] = q(us(st[:, 15] - st[:, 0]))
        print(json.dumps(row), flush=True)
    lib.dk_diag_path_stats_enable(e._ctx, 0)


def phase_totals(st, us, names):
    """Per-wave totals over every chunk (rx_diag.h DK_ACC_*: slots 20.., chunk count in 26): the median wave's µs per
    phase, the same summed over the waves as a share of their summed entry-to-exit time, and per chunk."""
    n = st[:, 26]
    life = (st[:, 15] - st[:, 0]).astype(float)
    out = {"chunks_per_wave": [int(n.min()), round(float(n.mean()), 2), int(n.max())]}
    for j, nm in enumerate(names):
        a = st[:, 20 + j].astype(float)
        out[nm] = {"median_us": round(float(np.median(us(a))), 2), "share": round(float(a.sum() / life.sum()), 3),
                   "us_per_chunk": round(float(us(a).sum() / max(n.sum(), 1)), 3)}
    return out


if __name__ == "__main__":
    main()
