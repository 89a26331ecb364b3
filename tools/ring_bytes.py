#!/usr/bin/env python3
"""Where the TPACKET_V3 ring path loses to the packed host path: PCIe-inclusive GB/s of the same
1500-byte frames laid out (a) in 64-byte slots, (b)-(e) shifted so the frame starts 2 bytes past each 16-byte granule
of a 64-byte line (lg = 0..3), (f) in a TPACKET_V3 ring (block scan outside the timed call: layout only) and (g) the
ring path with its scan; beside each, a host-side count of the 64-byte lines the kernel's loads touch per frame under
the quarter-wave span plan (spans from the frame's first granule, rounds 1-4) and under line-aligned spans (round 5),
counting a line once per load instruction that touches it (uncached host memory: no merging across instructions).
One library per process (--lib selects a build): python tools/ring_bytes.py [--frames N] [--lib path]"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def lines_per_frame(addr, lens, aligned_spans):
    """64-byte lines requested per frame: each quarter-wave load covers 16 granules (256 bytes)."""
    tot = 0
    for a, L in zip(addr.tolist(), lens.tolist()):
        g0 = a - (a % 16)  # the frame's first granule
        end = a + L
        start = g0 - (g0 % 64) if aligned_spans else g0
        s = start
        while s < end:
            lo, hi = max(s, g0), min(s + 256, (end + 15) // 16 * 16)
            if hi > lo:
                tot += (hi - 1) // 64 - lo // 64 + 1
            s += 256
    return tot / len(lens)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--frames", type=int, default=1 << 19)
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--lib", default=None, help="a variant libdk_rx.so (tools/variants.sh) instead of the in-tree one")
    args = ap.parse_args()
    import torch

    from demikernel_amd import Config, RxEngine, RxResults, synth
    from demikernel_amd import ring as RG

    lib = os.path.basename(args.lib or "libdk_rx.so")
    n = args.frames
    flows = synth.make_flows(1024)
    tr = synth.traffic(n, np.full(n, 1486, np.uint16), flows, seed=synth.SEED + 5)
    packed, poff, lens = synth.build_numpy(tr)
    eng = RxEngine(Config(synth.BOB_IPV4), device=0, lib_path=os.path.abspath(args.lib) if args.lib else None)
    eng.set_sockets(flows)
    res = RxResults(n, len(flows), host=True)
    nbytes = int(lens.astype(np.int64).sum())

    def pinned_desc(off, ln):  # descriptors in pinned memory, as bench.py host_path passes them
        o = torch.from_numpy(np.ascontiguousarray(off, np.uint32).view(np.int32)).pin_memory()
        l_ = torch.from_numpy(np.ascontiguousarray(ln, np.uint16).view(np.int16)).pin_memory()
        return o.numpy().view(np.uint32), l_.numpy().view(np.uint16), (o, l_)

    def timed(blob_np, off, ln):
        pinned = torch.empty(blob_np.nbytes, dtype=torch.uint8, pin_memory=True)
        pinned.numpy()[:] = blob_np
        off, ln, keep = pinned_desc(off, ln)
        rates = []
        for _ in range(args.reps + 1):
            t = time.perf_counter()
            eng.receive_batch_host(pinned.numpy(), off, ln, res)
            rates.append(nbytes / (time.perf_counter() - t) / 1e9)
        return float(np.median(rates[1:])), int(pinned.data_ptr())

    def timed_registered(blob_np, off, ln):
        """The same call over an anonymous mmap registered with hipHostRegister (as a PACKET_RX_RING mapping is),
        instead of torch's pinned allocation."""
        from demikernel_amd import _native as N
        buf = RG.page_aligned_empty(blob_np.nbytes)
        buf[:] = blob_np
        lib = N.load_library()
        assert lib.dk_ring_register(buf.ctypes.data, buf.nbytes) == 0
        off, ln, keep = pinned_desc(off, ln)
        try:
            rates = []
            for _ in range(args.reps + 1):
                t = time.perf_counter()
                eng.receive_batch_host(buf, off, ln, res)
                rates.append(nbytes / (time.perf_counter() - t) / 1e9)
        finally:
            lib.dk_ring_unregister(buf.ctypes.data)
        return float(np.median(rates[1:]))

    gb = timed_registered(packed, poff, lens)
    print(json.dumps({"lib": lib, "layout": "64-byte slots, mmap + hipHostRegister (ring-style registration)",
                      "gbps": round(gb, 2)}), flush=True)
    for shift in (0, 2, 18, 34, 50):
        blob = np.zeros(packed.nbytes + 64, np.uint8)
        blob[shift:shift + packed.nbytes] = packed
        off = (poff.astype(np.int64) + shift).astype(np.uint32)
        gbps, base = timed(blob, off, lens)
        addr = base + off.astype(np.int64)
        print(json.dumps({"lib": lib, "layout": f"64-byte slots + {shift}", "gbps": round(gbps, 2),
                          "lines_per_frame_first_granule_spans": round(lines_per_frame(addr[:4096], lens[:4096], False), 2),
                          "lines_per_frame_line_aligned_spans": round(lines_per_frame(addr[:4096], lens[:4096], True), 2)}),
              flush=True)
    block = 1 << 22
    ring, used, exp_off, elen = RG.build_tpacket3(packed, poff, lens, block)
    r = RG.TpacketRing(ring, block)
    try:
        off, ln, nb = r.scan(0, used, n)
        assert len(off) == n
        off, ln, keep = pinned_desc(off, ln)
        rates = []
        for _ in range(args.reps + 1):
            t = time.perf_counter()
            eng.receive_batch_host(ring, off, ln, res)
            rates.append(nbytes / (time.perf_counter() - t) / 1e9)
        addr = ring.ctypes.data + off.astype(np.int64)
        print(json.dumps({"lib": lib, "layout": "TPACKET_V3 ring, descriptors scanned outside the timed call",
                          "gbps": round(float(np.median(rates[1:])), 2),
                          "lines_per_frame_first_granule_spans": round(lines_per_frame(addr[:4096], ln[:4096], False), 2),
                          "lines_per_frame_line_aligned_spans": round(lines_per_frame(addr[:4096], ln[:4096], True), 2)}),
              flush=True)
        gb, _ = timed(ring, off, ln)
        print(json.dumps({"lib": lib, "layout": "TPACKET_V3 ring layout copied into torch-pinned (hipHostMalloc) memory",
                          "gbps": round(gb, 2)}), flush=True)
        rates = []
        for _ in range(args.reps + 1):
            t = time.perf_counter()
            nf, nb2 = r.receive(eng, 0, used, res)
            rates.append(nbytes / (time.perf_counter() - t) / 1e9)
        print(json.dumps({"lib": lib, "layout": "TPACKET_V3 ring path (block scan + process, as bench ring_path)",
                          "gbps": round(float(np.median(rates[1:])), 2)}), flush=True)
    finally:
        r.close()


if __name__ == "__main__":
    main()
