"""TPACKET_V3 ring ingest (include/dk_ring.h) on CPU: the block walker gives exactly the frames a
Linux TPACKET_V3 ring holds, in ring order, and stops, wraps, caps and rejects the way dk_ring.h says. Layout facts of
the ring (48-byte block descriptor and tpacket3_hdr, 8-byte packet alignment, tp_mac) are checked against the C
structures of <linux/if_packet.h>."""
import subprocess

import numpy as np
import pytest

from demikernel_amd import ring as RG
from demikernel_amd import synth
from demikernel_amd.rx import Fail

EBADMSG, ENOSPC, EINVAL = 74, 28, 22


def frames(n, seed=3):
    flows = synth.make_flows(32)
    tr = synth.traffic(n, synth.imix_ip_lengths(n, seed=seed), flows, seed=seed)
    return synth.build_numpy(tr)


def test_linux_struct_layout(tmp_path):
    src = tmp_path / "l.c"
    src.write_text('#include <stdio.h>\n#include <stddef.h>\n#include <linux/if_packet.h>\nint main(void){'
                   'printf("%zu %zu %zu %zu %zu %zu\\n", sizeof(struct tpacket_block_desc), sizeof(struct tpacket3_hdr),'
                   'offsetof(struct tpacket_block_desc, hdr.bh1.block_status),'
                   'offsetof(struct tpacket_block_desc, hdr.bh1.num_pkts), offsetof(struct tpacket3_hdr, tp_mac),'
                   'offsetof(struct tpacket3_hdr, tp_snaplen)); return 0;}')
    exe = tmp_path / "l"
    subprocess.run(["gcc", "-o", str(exe), str(src)], check=True)
    got = subprocess.run([str(exe)], capture_output=True, text=True, check=True).stdout.split()
    assert [int(x) for x in got] == [RG.BLOCK_DESC_BYTES, RG.PKT_HDR_BYTES, 8, 12, 24, 12]


@pytest.mark.parametrize("block_size", [1 << 16, 1 << 20])
def test_scan_gives_ring_frames_in_order(block_size):
    blob, off, lens = frames(3000)
    ring, used, eoff, elen = RG.build_tpacket3(blob, off, lens, block_size)
    r = RG.TpacketRing(ring, block_size, register=False)
    o, ln, nb = r.scan(0, used, len(off))
    assert nb == used and np.array_equal(o, eoff) and np.array_equal(ln, elen)
    assert set(int(x) % 16 for x in o) <= {2, 10}  # Ethernet header at 2 mod 8, like NIC buffers
    for k in range(0, len(off), 97):
        assert ring[o[k]:o[k] + ln[k]].tobytes() == blob[off[k]:off[k] + lens[k]].tobytes()


def test_scan_stops_at_kernel_owned_block_and_wraps():
    blob, off, lens = frames(2000)
    bs = 1 << 16
    ring, used, eoff, elen = RG.build_tpacket3(blob, off, lens, bs, nblocks=None)
    assert used >= 4
    r = RG.TpacketRing(ring, bs, register=False)
    r.release(2, 1)  # block 2 handed back to the kernel: the scan stops before it
    o, ln, nb = r.scan(0, used, len(off))
    per_block = np.bincount((eoff // bs).astype(np.int64), minlength=used)
    assert nb == 2 and len(o) == per_block[:2].sum()
    # wrap: starting at the last block, two blocks = the last one then block 0
    o2, _, nb2 = r.scan(used - 1, 2, len(off))
    assert nb2 == 2 and np.array_equal(o2, np.concatenate([eoff[eoff // bs == used - 1], eoff[eoff // bs == 0]]))


def test_scan_capacity():
    blob, off, lens = frames(2000)
    bs = 1 << 16
    ring, used, eoff, _ = RG.build_tpacket3(blob, off, lens, bs)
    r = RG.TpacketRing(ring, bs, register=False)
    first = int((eoff // bs == 0).sum())
    o, _, nb = r.scan(0, used, first + 5)  # room for block 0 only
    assert nb == 1 and len(o) == first
    with pytest.raises(Fail) as e:
        r.scan(0, used, first - 1)  # not even block 0 fits
    assert e.value.errno == ENOSPC


def test_malformed_blocks_rejected():
    blob, off, lens = frames(200)
    bs = 1 << 16
    ring, used, eoff, _ = RG.build_tpacket3(blob, off, lens, bs)
    bad = ring.copy()
    first_pkt = RG.BLOCK_DESC_BYTES
    bad[first_pkt:first_pkt + 4] = 0  # tp_next_offset 0 on a packet that is not the block's last
    with pytest.raises(Fail) as e:
        RG.TpacketRing(bad, bs, register=False).scan(0, used, 10000)
    assert e.value.errno == EBADMSG
    bad = ring.copy()
    bad[first_pkt + 12:first_pkt + 16] = np.frombuffer(np.uint32(bs).tobytes(), np.uint8)  # snaplen past the block
    with pytest.raises(Fail) as e:
        RG.TpacketRing(bad, bs, register=False).scan(0, used, 10000)
    assert e.value.errno == EBADMSG
    with pytest.raises(Fail) as e:
        RG.TpacketRing(ring, bs, register=False).scan(used + 100, 1, 10)  # first block outside the ring
    assert e.value.errno == EINVAL


def test_malformed_later_block_returns_good_prefix_then_is_consumed():
    """A malformed block after good ones: the good prefix comes back (rc 0) and is consumed; the next scan starting at
    the bad block reports EBADMSG with that block counted as consumed, so releasing it unblocks the ring."""
    blob, off, lens = frames(2000)
    bs = 1 << 16
    ring, used, eoff, _ = RG.build_tpacket3(blob, off, lens, bs, nblocks=None)
    assert used >= 4
    first_pkt = bs + RG.BLOCK_DESC_BYTES  # first packet of block 1
    ring[first_pkt:first_pkt + 4] = 0     # tp_next_offset 0 on a packet that is not the block's last
    r = RG.TpacketRing(ring, bs, register=False)
    o, _, nb = r.scan(0, used, len(off))
    assert nb == 1 and np.array_equal(o, eoff[eoff // bs == 0])
    with pytest.raises(Fail) as e:
        r.scan(1, used - 1, len(off))
    assert e.value.errno == EBADMSG and e.value.blocks == 1
    r.release(1, 1)
    o3, _, nb3 = r.scan(2, used - 2, len(off))
    assert nb3 == used - 2 and np.array_equal(o3, eoff[eoff // bs >= 2])


def test_long_scan_on_several_threads():
    """A scan over many ready blocks walks them on several host threads (ring_host.cpp: >= 8 blocks and >= 32,768
    frames); the result is
    the sequential walk's: every frame in ring order, a capacity cut at a block boundary, a malformed block in a later
    thread's range returning the good prefix, and that block reported (EBADMSG, consumed) when a scan starts at it."""
    blob, off, lens = frames(40000, seed=9)
    bs = 1 << 16
    ring, used, eoff, elen = RG.build_tpacket3(blob, off, lens, bs, nblocks=None)
    assert used >= 40
    r = RG.TpacketRing(ring, bs, register=False)
    o, ln, nb = r.scan(0, used, len(off))
    assert nb == used and np.array_equal(o, eoff) and np.array_equal(ln, elen)
    per_block = np.bincount((eoff // bs).astype(np.int64), minlength=used)
    cut = int(per_block[:29].sum()) + 3  # blocks 0..28 fit, block 29 does not
    o, _, nb = r.scan(0, used, cut)
    assert nb == 29 and np.array_equal(o, eoff[eoff // bs < 29])
    bad = 31
    first_pkt = bad * bs + RG.BLOCK_DESC_BYTES
    ring[first_pkt:first_pkt + 4] = 0  # tp_next_offset 0 on a packet that is not the block's last
    o, _, nb = r.scan(0, used, len(off))
    assert nb == bad and np.array_equal(o, eoff[eoff // bs < bad])
    with pytest.raises(Fail) as e:
        r.scan(bad, used - bad, len(off))
    assert e.value.errno == EBADMSG and e.value.blocks == 1
    o, _, nb = r.scan(bad + 1, used - bad - 1, len(off))
    assert nb == used - bad - 1 and np.array_equal(o, eoff[eoff // bs > bad])


def reference_scan(ring, bs, first, nblocks, cap):
    """The walk's contract restated block by block in Python (dk_ring.h: stop at a kernel-owned block; a block that
    overflows cap ends the scan before it, ENOSPC when it is the first; the first malformed block ends the scan after
    the good ones, EBADMSG and consumed when it is the first; stop once cap is exactly full)."""
    u32 = lambda a: int(np.frombuffer(ring[a:a + 4].tobytes(), np.uint32)[0])  # noqa: E731
    u16 = lambda a: int(np.frombuffer(ring[a:a + 2].tobytes(), np.uint16)[0])  # noqa: E731
    nring = ring.nbytes // bs
    offs, lens, k = [], [], 0
    while k < min(nblocks, nring):
        base = ((first + k) % nring) * bs
        if not (u32(base + 8) & RG.TP_STATUS_USER):
            break
        npk, p = u32(base + 12), u32(base + 16)
        if npk and len(offs) + npk > cap:
            return (ENOSPC, 0, 0, [], []) if k == 0 else (0, len(offs), k, offs, lens)
        bo, bl, bad = [], [], False
        for j in range(npk):
            if p + RG.PKT_HDR_BYTES > bs:
                bad = True
                break
            f, sn = p + u16(base + p + 24), u32(base + p + 12)
            if sn > 0xFFFF or f + sn > bs:
                bad = True
                break
            bo.append(base + f)
            bl.append(sn)
            if j + 1 < npk:
                nxt = u32(base + p)
                if nxt == 0:
                    bad = True
                    break
                p += nxt
        if bad:
            return (EBADMSG, 0, 1, [], []) if k == 0 else (0, len(offs), k, offs, lens)
        offs += bo
        lens += bl
        k += 1
        if len(offs) == cap:
            break
    return 0, len(offs), k, offs, lens


def test_scan_matches_reference_walk_under_corruption():
    """The two-pass, multi-thread walk (ring_host.cpp) against reference_scan on rings of 48+ blocks with corrupted
    headers, kernel-owned blocks, wrapped starts and caps that cut anywhere: return code, frames, blocks consumed and
    every descriptor identical."""
    blob, off, lens = frames(40000, seed=21)
    bs = 1 << 16
    ring0, used, _, _ = RG.build_tpacket3(blob, off, lens, bs, nblocks=None)
    rng = np.random.default_rng(22)
    for case in range(12):
        ring = ring0.copy()
        for _ in range(int(rng.integers(0, 4))):
            blk = int(rng.integers(0, used))
            what = int(rng.integers(0, 4))
            b = blk * bs
            if what == 0:  # tp_next_offset of the block's first packet zeroed
                ring[b + RG.BLOCK_DESC_BYTES:b + RG.BLOCK_DESC_BYTES + 4] = 0
            elif what == 1:  # snaplen past the block
                ring[b + RG.BLOCK_DESC_BYTES + 12:b + RG.BLOCK_DESC_BYTES + 16] = np.frombuffer(
                    np.uint32(bs).tobytes(), np.uint8)
            elif what == 2:  # handed back to the kernel
                ring[b + 8:b + 12] = 0
            else:  # num_pkts inflated: the chain runs off the block
                ring[b + 12:b + 16] = np.frombuffer(np.uint32(100000).tobytes(), np.uint8)
        first = int(rng.integers(0, used)) if case % 3 == 0 else 0
        cap = int(rng.choice([len(off), int(rng.integers(1, len(off)))]))
        exp = reference_scan(ring, bs, first, used, cap)
        r = RG.TpacketRing(ring, bs, register=False)
        try:
            o, ln, nb = r.scan(first, used, cap)
            got = (0, len(o), nb)
        except Fail as e:
            o, ln, got = [], [], (e.errno, 0, e.blocks)
        assert got == exp[:3], (case, got, exp[:3])
        if got[0] == 0:
            assert np.array_equal(o, np.array(exp[3], np.uint32)) and np.array_equal(ln, np.array(exp[4], np.uint16))


def load_live_fixture():
    """The ring a live AF_PACKET socket on `lo` filled (tests/golden/make_ring_fixture.py), in page-aligned memory."""
    import os

    g = np.load(os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "live_ring_lo.npz"),
                allow_pickle=False)
    ring = RG.page_aligned_empty(g["ring"].nbytes)
    ring[:] = g["ring"]
    return g, ring


def test_live_ring_fixture_scan_and_oracle():
    """The captured kernel-written ring (block descriptors and tpacket3 headers exactly as Linux wrote them): the scan
    finds the descriptors it found at capture time, every injected frame in order at 2 mod 16, and the oracle's
    results over those descriptors are the ones recorded then (the GPU replay compares with the same oracle)."""
    from demikernel_amd._native import FLOW_DTYPE
    from oracle.oracle import OraclePeer

    g, ring = load_live_fixture()
    bs, nb = int(g["block_size"]), int(g["nblocks"])
    off, ln, used = RG.TpacketRing(ring, bs, register=False).scan(0, nb, 1 << 16)
    assert used == nb and np.array_equal(off, g["scan_off"]) and np.array_equal(ln, g["scan_len"])
    frames, flen = g["frames"], g["frame_len"]
    starts = np.concatenate([[0], np.cumsum(flen.astype(np.int64))[:-1]])
    for j, k in enumerate(g["mine"]):
        assert ring[off[k]:off[k] + ln[k]].tobytes() == frames[starts[j]:starts[j] + flen[j]].tobytes(), j
    assert {int(off[k]) % 16 for k in g["mine"]} <= {2, 10}
    peer = OraclePeer(synth.ipv4(synth.BOB_IPV4))
    peer.set_flows(g["flows"].view(FLOW_DTYPE))
    exp = peer.process(ring, off, ln)
    for k, v in exp.items():
        assert np.array_equal(v, g["res_" + k]), k
