"""A live TPACKET_V3 receive ring on the loopback interface: frames sent through a raw socket
come back through the kernel's PACKET_RX_RING blocks, and dk_ring_scan_tpacket3 / dk_rx_process_tpacket3 read them in
place (catpowder's receive, catpowder/linux/mod.rs:138-159, with the kernel's ring instead of one recvfrom per frame).
Needs CAP_NET_RAW: skipped, with that reason, where the process lacks it (e.g. an unprivileged GPU box)."""
import time

import numpy as np
import pytest

from demikernel_amd import Config, RxEngine, RxResults, synth
from demikernel_amd import ring as RG
from oracle.oracle import OraclePeer


def open_ring():
    try:
        return RG.PacketSocketRing("lo", block_size=1 << 16, nblocks=32)
    except PermissionError as e:
        pytest.skip(f"no CAP_NET_RAW for an AF_PACKET socket in this process ({e})")
    except OSError as e:
        pytest.skip(f"AF_PACKET / PACKET_RX_RING unavailable here ({e})")


def send_and_collect(pr, frames, timeout=3.0):
    """Inject `frames` on lo, wait until the ring's blocks hold them (blocks retire after 4 ms), scan the ready blocks.
    Returns (descriptors off, len of our frames in ring order, first block, blocks consumed)."""
    RG.inject("lo", frames)
    r = RG.TpacketRing(pr.ring, pr.block_size, register=False)
    want = {bytes(f) for f in frames}
    deadline = time.time() + timeout
    nb = 0
    while True:
        while nb < pr.nblocks and pr.block_ready(nb):
            nb += 1
        off, ln, used = r.scan(0, nb, 1 << 16) if nb else (np.zeros(0, np.uint32), np.zeros(0, np.uint16), 0)
        mine = [k for k in range(len(off)) if pr.ring[off[k]:off[k] + ln[k]].tobytes() in want]
        if len(mine) >= len(frames) or time.time() > deadline:
            return off, ln, mine, used
        time.sleep(0.01)


def loop_frames(n=400, seed=21):
    flows = np.concatenate([synth.make_flows(64), synth.make_flows(8, kind="udp")])
    tr = synth.traffic(n, synth.imix_ip_lengths(n, seed=seed), flows, seed=seed)
    blob, off, lens = synth.build_numpy(tr)
    synth.corrupt_numpy(blob, off, synth.corruption_plan(n, 0.05, tr, seed=seed))
    return flows, [blob[o:o + L].tobytes() for o, L in zip(off, lens)]


def test_live_loopback_ring_scan():
    """Every injected frame is in the kernel-filled ring, in order, at the offset / length the scan reports (frames at
    2 mod 16, the realigned vector path); releasing the blocks hands them back (TP_STATUS_KERNEL)."""
    pr = open_ring()
    try:
        _, frames = loop_frames()
        off, ln, mine, used = send_and_collect(pr, frames)
        assert len(mine) == len(frames), f"{len(mine)} of {len(frames)} frames seen"
        got = [pr.ring[off[k]:off[k] + ln[k]].tobytes() for k in mine]
        assert got == frames
        assert {int(off[k]) % 16 for k in mine} <= {2, 10}
        RG.TpacketRing(pr.ring, pr.block_size, register=False).release(0, used)
        assert not any(pr.block_ready(k) for k in range(used))
    finally:
        pr.close()


@pytest.mark.gpu
def test_live_loopback_ring_through_engine():
    """The same live ring through dk_rx_process_tpacket3 (block scan, H2D of the blocks' byte ranges, kernel, D2H):
    our frames' results equal the oracle's on the same ring bytes."""
    import torch

    assert torch.cuda.is_available()
    pr = open_ring()
    try:
        flows, frames = loop_frames(600, seed=22)
        off, ln, mine, used = send_and_collect(pr, frames)
        assert len(mine) == len(frames)
        eng = RxEngine(Config(synth.BOB_IPV4))
        eng.set_sockets(flows)
        r = RG.TpacketRing(pr.ring, pr.block_size, register=False)
        res = RxResults(len(off), len(flows), tcp_fields=True, host=True)
        nf, nb = r.receive(eng, 0, used, res)
        assert (nf, nb) == (len(off), used)
        peer = OraclePeer(synth.ipv4(synth.BOB_IPV4))
        peer.set_flows(flows)
        exp = peer.process(pr.ring, off, ln)
        got = res.to_numpy()
        for k in ("meta", "src_ip", "dst_ip", "ports", "payload", "flow_id", "tcp_seq", "tcp_ack", "tcp_win"):
            assert np.array_equal(got[k], exp[k]), k
        assert (got["meta"][mine] & 0xFF <= 1).mean() > 0.9
        r.release(0, used)
        eng.close()
    finally:
        pr.close()


@pytest.mark.gpu
def test_captured_live_ring_through_engine():
    """The kernel-filled ring captured on a host with CAP_NET_RAW (tests/golden/live_ring_lo.npz, made by
    tests/golden/make_ring_fixture.py: Linux's own block descriptors and tpacket3 headers) replayed through
    dk_rx_process_tpacket3 on the GPU — page-locked in place, block scan, H2D of the blocks' byte ranges, kernel, D2H —
    bit-exact against the oracle over the same ring bytes, for every frame in the ring (ours and any other traffic on
    `lo` at capture time). The GPU boxes lack CAP_NET_RAW, so this is how the live ring reaches the engine there."""
    import torch

    from demikernel_amd._native import FLOW_DTYPE
    from test_ring import load_live_fixture

    assert torch.cuda.is_available()
    g, ring = load_live_fixture()
    bs, nb = int(g["block_size"]), int(g["nblocks"])
    flows = g["flows"].view(FLOW_DTYPE)
    eng = RxEngine(Config(synth.BOB_IPV4))
    eng.set_sockets(flows)
    r = RG.TpacketRing(ring, bs)  # page-locked in place (dk_ring_register)
    try:
        n = len(g["scan_off"])
        res = RxResults(n, len(flows), tcp_fields=True, host=True)
        nf, used = r.receive(eng, 0, nb, res)
        assert (nf, used) == (n, nb)
        peer = OraclePeer(synth.ipv4(synth.BOB_IPV4))
        peer.set_flows(flows)
        exp = peer.process(ring, g["scan_off"], g["scan_len"])
        got = res.to_numpy()
        for k in ("meta", "src_ip", "dst_ip", "ports", "payload", "flow_id", "tcp_seq", "tcp_ack", "tcp_win",
                  "flow_counts", "verdict_counts"):
            e = exp[k][: len(got[k])]
            assert np.array_equal(got[k], e), k
            assert np.array_equal(got[k], g["res_" + k][: len(got[k])]), k
        assert (got["meta"] & 0xFF <= 1).mean() > 0.8
    finally:
        r.close()
        eng.close()
