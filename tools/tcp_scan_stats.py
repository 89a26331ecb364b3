#!/usr/bin/env python3
"""Where the TCP scan walk's time goes: one dk_tcp_rx_process call on the bench's stream shape through a
DK_TCP_SCAN_STATS build (tools/variants.sh "tcpstats:-DDK_TCP_SCAN_STATS=1"), whose scan kernel prints per connection
its batch steps (64 decided windows each when full), slow windows (undecided: the relay's path), windows walked in the
LDS rings and batch restarts (each a fresh dependent load of three batches). Then the same call timed on that build
and on the in-tree one.

    python tools/tcp_scan_stats.py build/variants/tcpstats.so [--nconns 1] [--reorder 0] [--buffer-size 1073741824]
"""
import argparse
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("lib")
    ap.add_argument("--nseg", type=int, default=1 << 20)
    ap.add_argument("--nconns", type=int, default=1)
    ap.add_argument("--reorder", type=float, default=0.0)
    ap.add_argument("--buffer-size", type=int, default=1 << 30)
    a = ap.parse_args()
    import torch

    from demikernel_amd import RxResults, synth
    from demikernel_amd.tcp import TcpOut, TcpReceiver

    _, tr, table = synth.tcp_streams(a.nseg, a.nconns, 1500, buffer_size=a.buffer_size, reorder=a.reorder)
    rx = {"meta": (6 << 8 | tr.flags.astype(np.uint32) << 16 | 0x50 << 24).astype(np.uint32),
          "flow_id": tr.flow.astype(np.uint32), "tcp_seq": tr.seq, "tcp_ack": tr.ack,
          "payload": (54 | (tr.ip_len.astype(np.uint32) - 40) << 16).astype(np.uint32)}
    r = RxResults(a.nseg, 1, device=torch.device("cuda", 0), tcp_fields=True, counts=False)
    for k, v in rx.items():
        r.t[k].copy_(torch.from_numpy(v.view(np.int32)))
    for lib in (os.path.abspath(a.lib), None):
        tcp = TcpReceiver(0, lib_path=lib, walk="scan")
        pristine = tcp.conns_to_device(table)
        conns = pristine.clone()
        out = TcpOut(a.nseg, len(table), 0)
        ts = []
        for i in range(4 if lib is None else 1):
            conns.copy_(pristine)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            tcp.process(r, conns, out)
            e1.record()
            torch.cuda.synchronize()
            ts.append(e0.elapsed_time(e1))
        print(f'{{"lib": "{os.path.basename(lib) if lib else "in-tree"}", "ms": {min(ts):.4f}}}', flush=True)
        tcp.close()


if __name__ == "__main__":
    main()
