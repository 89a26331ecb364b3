#!/usr/bin/env python3
"""Read/write-mix ceiling for the small-frame kernel (dk_diag_rw_probe): `--mb` MB buffers (8 rotated, past the
256 MB MALL) read in 4 KiB wave steps, with nres = 0 (reads only) and 6 (C3's six u32 result arrays per 64-byte slot:
the same write/read ratio as the 24-byte record over 64-byte frames), over several grids. One JSON line each: read,
written and total TB/s (median of --reps)."""
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
    ap.add_argument("--mb", type=int, default=64)
    ap.add_argument("--grids", default="256,512,768,1024,1536,2048")
    ap.add_argument("--nres", default="0,6")
    ap.add_argument("--iters", type=int, default=16)
    ap.add_argument("--reps", type=int, default=5)
    a = ap.parse_args()
    import torch

    from demikernel_amd import _native as N

    lib = N.load_library()
    nbytes = a.mb << 20
    bufs = [torch.randint(0, 255, (nbytes,), dtype=torch.uint8, device="cuda") for _ in range(8)]
    dst = torch.empty(6 * nbytes // 64, dtype=torch.int32, device="cuda")
    s = torch.cuda.current_stream()
    for nres in [int(x) for x in a.nres.split(",")]:
        for g in [int(x) for x in a.grids.split(",")]:
            scratch = torch.zeros(g, dtype=torch.int32, device="cuda")

            def run(k):
                rc = lib.dk_diag_rw_probe(ctypes.c_void_p(bufs[k % 8].data_ptr()), nbytes,
                                          ctypes.c_void_p(dst.data_ptr()), nres, ctypes.c_void_p(scratch.data_ptr()),
                                          g, ctypes.c_void_p(s.cuda_stream))
                assert rc == 0, rc
            ts = []
            for _ in range(a.reps):
                for k in range(3):
                    run(k)
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record(s)
                for k in range(a.iters):
                    run(k)
                e1.record(s)
                torch.cuda.synchronize()
                ts.append(e0.elapsed_time(e1) / 1e3 / a.iters)
            t = float(np.median(ts))
            wb = nres * nbytes // 16
            print(json.dumps({"probe": "rw", "nres": nres, "grid": g, "read_MB": nbytes / 1e6, "write_MB": wb / 1e6,
                              "us": round(t * 1e6, 2), "read_TBps": round(nbytes / t / 1e12, 3),
                              "total_TBps": round((nbytes + wb) / t / 1e12, 3)}), flush=True)


if __name__ == "__main__":
    main()
