#!/usr/bin/env python3
"""Interleaved A/B of dk_tcp_rx_process across library builds (tools/variants.sh) on the bench's streams: for each
connection count, the same inputs through every build, `--reps` rounds of `--iters` calls each (the connection
table restored between calls, outside the timed span), median ms per call; outputs compared with the first build's
(actions, views, deliveries, connection table).

    python tools/tcp_ab.py build/variants/a.so build/variants/b.so[:radix] --nconns 1,16,64 [--reorder 0] [--walk scan]
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
    ap.add_argument("libs", nargs="+")
    ap.add_argument("--nseg", type=int, default=1 << 20)
    ap.add_argument("--nconns", default="1")
    ap.add_argument("--reorder", type=float, default=0.0)
    ap.add_argument("--buffer-size", type=int, default=1 << 30)
    ap.add_argument("--walk", default=None)
    ap.add_argument("--iters", type=int, default=5)
    ap.add_argument("--reps", type=int, default=5)
    a = ap.parse_args()
    import torch

    from demikernel_amd import RxResults, synth
    from demikernel_amd.tcp import TcpOut, TcpReceiver

    for nconns in [int(x) for x in a.nconns.split(",")]:
        _, tr, table = synth.tcp_streams(a.nseg, nconns, 1500, buffer_size=a.buffer_size, reorder=a.reorder)
        rx = {"meta": (6 << 8 | tr.flags.astype(np.uint32) << 16 | 0x50 << 24).astype(np.uint32),
              "flow_id": tr.flow.astype(np.uint32), "tcp_seq": tr.seq, "tcp_ack": tr.ack,
              "payload": (54 | (tr.ip_len.astype(np.uint32) - 40) << 16).astype(np.uint32)}
        r = RxResults(a.nseg, 1, device=torch.device("cuda", 0), tcp_fields=True, counts=False)
        for k, v in rx.items():
            r.t[k].copy_(torch.from_numpy(v.view(np.int32)))
        runs = []
        for spec in a.libs:  # path[:radix] (the radix sort forced: dk_diag_tcp_set_sort)
            lib, _, opt = spec.partition(":")
            tcp = TcpReceiver(0, lib_path=os.path.abspath(lib), walk=a.walk, radix_sort=opt == "radix")
            pristine = tcp.conns_to_device(table)
            runs.append({"name": os.path.basename(lib)[:-3] + (":" + opt if opt else ""), "tcp": tcp,
                         "pristine": pristine,
                         "conns": pristine.clone(), "out": TcpOut(a.nseg, len(table), 0), "t": []})
        for rep in range(a.reps + 1):
            for R in runs:
                ts = []
                for _ in range(a.iters):
                    R["conns"].copy_(R["pristine"])
                    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                    e0.record()
                    R["tcp"].process(r, R["conns"], R["out"])
                    e1.record()
                    torch.cuda.synchronize()
                    ts.append(e0.elapsed_time(e1))
                if rep:
                    R["t"].append(float(np.median(ts)))
        ref = runs[0]["out"].to_numpy()
        ref_c = runs[0]["conns"].cpu()
        def valid(h):  # every array but the delivery slots past each connection's count
            d = [h["deliv"][int(s0):int(s0) + int(c)] for s0, c in zip(h["deliv_start"], h["deliv_count"])]
            return [h["action"], h["view"], h["deliv_start"], h["deliv_count"]] + d

        for R in runs:
            got = R["out"].to_numpy()
            same = all(np.array_equal(x, y) for x, y in zip(valid(ref), valid(got))) and \
                torch.equal(ref_c, R["conns"].cpu())
            print(json.dumps({"lib": R["name"], "nconns": nconns, "reorder": a.reorder, "walk": R["tcp"].last_walk,
                              "ms": round(float(np.median(R["t"])), 4), "spread": [round(min(R["t"]), 4),
                                                                                  round(max(R["t"]), 4)],
                              "same_as_first": bool(same)}), flush=True)
        for R in runs:
            R["tcp"].close()


if __name__ == "__main__":
    main()
