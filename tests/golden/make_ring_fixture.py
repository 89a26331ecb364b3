#!/usr/bin/env python3
"""Capture a live TPACKET_V3 receive ring into a fixture (tests/golden/live_ring_lo.npz), for the GPU boxes, which
lack CAP_NET_RAW. Run where AF_PACKET works (this container):

    python tests/golden/make_ring_fixture.py

Frames (IMIX sizes, 5 % corrupted, TCP and UDP over a 72-entry socket table) are injected on `lo` through a raw socket;
the kernel writes them into a PACKET_RX_RING (TPACKET_V3, 64 KiB blocks, 4 ms retire timeout) — catpowder's
receive (catpowder/linux/mod.rs:138-159) with the kernel's ring in place of one recvfrom per frame. Once every injected
frame sits in a ready block, the ready blocks are copied out byte for byte with their block descriptors and packet
headers as the kernel wrote them (other traffic on `lo` included). Stored: the ring bytes, block size and count, the
socket table, the injected frames (their bytes, to find them again), the descriptors dk_ring_scan_tpacket3 gave and
the oracle's results over them at capture time (tests/test_ring.py pins both on the CPU; the GPU test replays the
ring through dk_rx_process_tpacket3).
"""
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)

from demikernel_amd import ring as RG  # noqa: E402
from demikernel_amd import synth  # noqa: E402
from oracle.oracle import OraclePeer  # noqa: E402

OUT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "live_ring_lo.npz")
BLOCK = 1 << 16
NBLOCKS = 16


def main():
    flows = np.concatenate([synth.make_flows(64), synth.make_flows(8, kind="udp")])
    n = 300
    tr = synth.traffic(n, synth.imix_ip_lengths(n, seed=41), flows, seed=41)
    blob, off, lens = synth.build_numpy(tr)
    synth.corrupt_numpy(blob, off, synth.corruption_plan(n, 0.05, tr, seed=41))
    frames = [blob[o:o + L].tobytes() for o, L in zip(off, lens)]
    pr = RG.PacketSocketRing("lo", block_size=BLOCK, nblocks=NBLOCKS)
    try:
        RG.inject("lo", frames)
        r = RG.TpacketRing(pr.ring, BLOCK, register=False)
        want = set(frames)
        deadline = time.time() + 5.0
        while True:
            nb = 0
            while nb < NBLOCKS and pr.block_ready(nb):
                nb += 1
            soff, sln, used = r.scan(0, nb, 1 << 16) if nb else (np.zeros(0, np.uint32), np.zeros(0, np.uint16), 0)
            seen = [k for k in range(len(soff)) if pr.ring[soff[k]:soff[k] + sln[k]].tobytes() in want]
            if len(seen) >= n or time.time() > deadline:
                break
            time.sleep(0.01)
        assert len(seen) == n, f"only {len(seen)} of {n} frames reached ready blocks"
        ring = pr.ring[: used * BLOCK].copy()
    finally:
        pr.close()
    peer = OraclePeer(synth.ipv4(synth.BOB_IPV4))
    peer.set_flows(flows)
    exp = peer.process(ring, soff, sln)
    fb = np.concatenate([np.frombuffer(f, np.uint8) for f in frames])
    flen = np.array([len(f) for f in frames], np.uint16)
    np.savez_compressed(OUT, ring=ring, block_size=np.uint32(BLOCK), nblocks=np.uint32(used),
                        flows=flows.view(np.uint8), frames=fb, frame_len=flen, scan_off=soff, scan_len=sln,
                        mine=np.array(seen, np.uint32),
                        **{"res_" + k: v for k, v in exp.items()})
    print(f"{OUT}: {used} blocks, {len(soff)} frames in the ring ({n} injected), {os.path.getsize(OUT)} bytes")


if __name__ == "__main__":
    main()
