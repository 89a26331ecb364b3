"""dk_tcp_rx_process time per walk (lane|wave|relay|scan|rule, forced by dk_diag_tcp_set_walk) on one connection's stream, with and without the
segments that need the state machine (synth.tcp_streams dup / oow / rare fractions), to separate the walks' per-window
cost from their process() calls. One JSON line per (stream, walk): ms per call (HIP events, median)."""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import numpy as np  # noqa: E402
import torch  # noqa: E402

from demikernel_amd import RxResults, synth  # noqa: E402
from demikernel_amd.tcp import TcpOut, TcpReceiver  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--nseg", type=int, default=1 << 20)
ap.add_argument("--nconns", type=int, nargs="+", default=[1])
ap.add_argument("--walks", nargs="+", default=["relay", "wave"])
ap.add_argument("--iters", type=int, default=5)
ap.add_argument("--relay-waves", type=int, nargs="+", default=[16])
ap.add_argument("--streams", nargs="+", default=["clean", "dups", "default"],
                help="clean | dups | default (in order, 1 GB buffer) | bench (bench.py's 64-connection line: reorder 3, 16 MB)")
ap.add_argument("--libs", nargs="+", default=[None], help="libdk_rx builds to compare (default: the package's)")
a = ap.parse_args()
torch.cuda.set_device(0)
dev = torch.device("cuda", 0)
s = torch.cuda.current_stream(0)
STREAMS = {"clean": dict(dup=0.0, oow=0.0, rare=0.0, fin=0.0, rst=0.0),
           "dups": dict(dup=0.02, oow=0.0, rare=0.0, fin=0.0, rst=0.0),
           "default": dict(),
           "bench": dict(buffer_size=1 << 24, reorder=3.0)}
for nconns in a.nconns:
    for name in a.streams:
        kw = {"buffer_size": 1 << 30, "reorder": 0.0, **STREAMS[name]}
        _, tr, table = synth.tcp_streams(a.nseg, nconns, 1500, **kw)
        rx = {"meta": (6 << 8 | tr.flags.astype(np.uint32) << 16 | 0x50 << 24).astype(np.uint32),
              "flow_id": tr.flow.astype(np.uint32), "tcp_seq": tr.seq, "tcp_ack": tr.ack,
              "payload": (54 | (tr.ip_len.astype(np.uint32) - 40) << 16).astype(np.uint32)}
        r = RxResults(a.nseg, 1, device=dev, tcp_fields=True, counts=False)
        for k, v in rx.items():
            r.t[k].copy_(torch.from_numpy(v.view(np.int32)))
        ref = None
        for walk, lib in [(w + (f":{k}" if w == "relay" else ""), lib) for w in a.walks
                          for k in (a.relay_waves if w == "relay" else [0]) for lib in a.libs]:
            wname = walk.split(":")[0]
            tcp = TcpReceiver(0, lib_path=os.path.abspath(lib) if lib else None,
                              walk=None if wname == "rule" else wname,
                              relay_waves=int(walk.split(":")[1]) if walk.startswith("relay") else 8)
            pristine = tcp.conns_to_device(table)
            conns = pristine.clone()
            out = TcpOut(a.nseg, len(table), 0)
            times = []
            for i in range(a.iters + 1):
                conns.copy_(pristine)
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record(s)
                tcp.process(r, conns, out, stream=s)
                e1.record(s)
                torch.cuda.synchronize()
                if i:
                    times.append(e0.elapsed_time(e1))
            got = out.to_numpy()
            hist = np.bincount(got["action"], minlength=13)
            same = None if ref is None else bool(np.array_equal(ref, got["action"]))
            ref = got["action"] if ref is None else ref
            tcp.close()
            print(json.dumps({"stream": name, "nconns": nconns, "walk": walk, "lib": lib or "package",
                              "ms": round(float(np.median(times)), 4),
                              "mseg_s": round(a.nseg / float(np.median(times)) / 1e3, 1),
                              "hist": [int(x) for x in hist], "same_actions_as_first": same}), flush=True)
