"""dk_tcp_rx_process timing sweep (bench.tcp_rate) over segment / connection counts."""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

import bench  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--nseg", type=int, nargs="+", default=[1 << 20])
ap.add_argument("--nconns", type=int, nargs="+", default=[1 << 14])
ap.add_argument("--iters", type=int, default=10)
ap.add_argument("--cpu-seconds", type=float, default=1.0)
ap.add_argument("--buffer-size", type=int, default=1 << 24)
ap.add_argument("--reorder", type=float, default=3.0)
a = ap.parse_args()
torch.cuda.set_device(0)
s = torch.cuda.current_stream(0)
for n in a.nseg:
    for c in a.nconns:
        print(json.dumps(bench.tcp_rate(s, n, c, a.iters, a.cpu_seconds, a.buffer_size, a.reorder)), flush=True)
