#!/usr/bin/env python3
"""Ring-path (TPACKET_V3 block scan + dk_rx_process_host) and packed host-path rates of several libdk_rx.so builds,
interleaved, on bench.py's C2 slice: python tools/ring_ab.py --lib a.so --lib b.so [--frames 524288] [--reps 3]"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--lib", action="append", default=[])
    ap.add_argument("--frames", type=int, default=1 << 19)
    ap.add_argument("--reps", type=int, default=3)
    args = ap.parse_args()
    import bench
    from demikernel_amd import Config, RxEngine, synth

    base = RxEngine(Config(synth.BOB_IPV4))
    batch, flows, _ = bench.make_batch(base, "c2_tcp1500", 0, synth.SEED, 1, frames=args.frames)
    engines = []
    for lp in args.lib or [None]:
        e = RxEngine(Config(synth.BOB_IPV4), lib_path=os.path.abspath(lp) if lp else None)
        e.set_sockets(flows)
        engines.append((os.path.basename(lp)[:-3] if lp else "head", e))
    res = {n: [] for n, _ in engines}
    for _ in range(args.reps):
        for n, e in engines:
            r = bench.ring_path_rate(e, batch, flows, args.frames)
            res[n].append((r["gbps"], r["host_scan_ms"]))
    for n, v in res.items():
        v.sort()
        print(json.dumps({"lib": n, "ring_gbps": v[len(v) // 2][0], "host_scan_ms": v[len(v) // 2][1],
                          "all": v}), flush=True)


if __name__ == "__main__":
    main()
