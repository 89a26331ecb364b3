"""The product's host-side code under AddressSanitizer + UndefinedBehaviorSanitizer (CPU only): ring_host.cpp (the
TPACKET_V3 block walker over caller memory), demi_host.cpp (results -> demi_sgarray_t) and dk_rx_process_host's chunk
planner (rx_plan.h), built into a standalone driver (tests/host_asan). Valid, corrupted and fuzzed inputs; every
sanitizer report aborts the driver (-fno-sanitize-recover), and its outputs must equal the regular libdk_rx.so's on
the same inputs (the reference's host side is catpowder/linux/mod.rs:138-159 and runtime/memory/mod.rs:38-54)."""
import ctypes
import fcntl
import os
import subprocess

import numpy as np
import pytest

from demikernel_amd import _native as N
from demikernel_amd import ring as RG
from demikernel_amd import synth

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
EXE = os.path.join(ROOT, "build", "host_asan")
ENV = dict(os.environ, ASAN_OPTIONS="detect_leaks=0:halt_on_error=1:abort_on_error=0",
           UBSAN_OPTIONS="halt_on_error=1:print_stacktrace=1")


@pytest.fixture(scope="module")
def driver():
    # one build at a time: pytest-xdist workers would otherwise race on the same output file
    os.makedirs(os.path.join(ROOT, "build"), exist_ok=True)
    with open(os.path.join(ROOT, "build", ".host_asan.lock"), "w") as lk:
        fcntl.flock(lk, fcntl.LOCK_EX)
        subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "tests", "host_asan")], check=True)
    return EXE


def run(driver, mode, payload: bytes, tmp_path):
    i, o = tmp_path / "in.bin", tmp_path / "out.bin"
    i.write_bytes(payload)
    p = subprocess.run([driver, mode, str(i), str(o)], env=ENV, capture_output=True, text=True, timeout=120)
    assert p.returncode == 0, p.stderr[-4000:]
    assert "runtime error" not in p.stderr and "AddressSanitizer" not in p.stderr, p.stderr[-4000:]
    return o.read_bytes()


def frames(n, seed=3):
    flows = synth.make_flows(32)
    tr = synth.traffic(n, synth.imix_ip_lengths(n, seed=seed), flows, seed=seed)
    return synth.build_numpy(tr)


def lib_scan(ring, bs, first, nb, cap):
    lib = N.load_library()
    off = np.zeros(max(cap, 1), np.uint32)
    ln = np.zeros(max(cap, 1), np.uint16)
    nf, nbo = ctypes.c_uint32(), ctypes.c_uint32()
    rc = lib.dk_ring_scan_tpacket3(ring.ctypes.data, ring.nbytes, bs, first, nb, off.ctypes.data if cap else None,
                                   ln.ctypes.data if cap else None, cap, ctypes.byref(nf), ctypes.byref(nbo))
    return rc, nf.value, nbo.value, off[: nf.value], ln[: nf.value]


def asan_scan(driver, tmp_path, ring, bs, first, nb, cap):
    hdr = np.array([ring.nbytes], np.uint64).tobytes() + np.array([bs, first, nb, cap], np.uint32).tobytes()
    out = run(driver, "ring", hdr + ring.tobytes(), tmp_path)
    rc, nf, nbo = np.frombuffer(out[:12], np.int32)
    off = np.frombuffer(out[12:12 + 4 * nf], np.uint32)
    ln = np.frombuffer(out[12 + 4 * nf:12 + 6 * nf], np.uint16)
    return int(rc), int(nf), int(nbo), off, ln


def corrupt_ring(ring, bs, used, rng):
    """One random header corruption: block descriptors (status, num_pkts, offset_to_first_pkt) or packet headers
    (tp_next_offset, tp_snaplen, tp_mac) set to random or extreme values."""
    r = ring.copy()
    b = int(rng.integers(0, used))
    base = b * bs
    what = int(rng.integers(0, 6))
    w32 = lambda at, v: r.__setitem__(slice(at, at + 4), np.frombuffer(np.uint32(v).tobytes(), np.uint8))  # noqa
    extreme = [0, 1, 0xFFFF, 0x10000, bs - 1, bs, bs + 1, 0x7FFFFFFF, 0xFFFFFFFF, int(rng.integers(0, 2**32))]
    v = extreme[int(rng.integers(0, len(extreme)))]
    if what == 0:
        w32(base + 12, v)  # num_pkts
    elif what == 1:
        w32(base + 16, v)  # offset_to_first_pkt
    else:
        # a packet header of this block, found by walking the valid chain
        first = int(r[base + 16: base + 20].view(np.uint32)[0])
        npk = int(r[base + 12: base + 16].view(np.uint32)[0])
        p = first
        for _ in range(int(rng.integers(0, max(npk, 1)))):
            nxt = int(r[base + p: base + p + 4].view(np.uint32)[0])
            if nxt == 0 or p + nxt + 48 > bs:
                break
            p += nxt
        if what == 2:
            w32(base + p, v)  # tp_next_offset
        elif what == 3:
            w32(base + p + 12, v)  # tp_snaplen
        elif what == 4:
            r[base + p + 24: base + p + 26] = np.frombuffer(np.uint16(v & 0xFFFF).tobytes(), np.uint8)  # tp_mac
        else:
            w32(base + 8, v & 1)  # block_status
    return r


def test_ring_walker_valid_and_corrupted(driver, tmp_path):
    blob, off, lens = frames(3000)
    rng = np.random.default_rng(5)
    for bs in (1 << 12, 1 << 16):
        ring, used, _, _ = RG.build_tpacket3(blob, off, lens, bs, nblocks=None)
        cases = [(ring, 0, used, len(off)), (ring, used - 1, 2, len(off)), (ring, 0, used, 7), (ring, 0, used, 0),
                 (ring, used + 3, 1, 10)]
        for _ in range(150):
            cases.append((corrupt_ring(ring, bs, used, rng), int(rng.integers(0, used)), int(rng.integers(1, used + 2)),
                          int(rng.choice([0, 5, 100, len(off)]))))
        for r, first, nb, cap in cases:
            got = asan_scan(driver, tmp_path, r, bs, first, nb, cap)
            exp = lib_scan(r, bs, first, nb, cap)
            assert got[:3] == exp[:3], (bs, first, nb, cap, got[:3], exp[:3])
            assert np.array_equal(got[3], exp[3]) and np.array_equal(got[4], exp[4])
            if got[0] == 0:  # every descriptor the walker hands out lies inside the ring
                assert np.all(got[3].astype(np.int64) + got[4] <= r.nbytes)


def test_ring_release(driver, tmp_path):
    blob, off, lens = frames(800)
    bs = 1 << 12
    ring, used, _, _ = RG.build_tpacket3(blob, off, lens, bs, nblocks=None)
    for first, nb in ((0, used), (used - 1, 2), (3, 0), (used, 1), (0, used + 1)):
        hdr = np.array([ring.nbytes], np.uint64).tobytes() + np.array([bs, first, nb], np.uint32).tobytes()
        out = run(driver, "release", hdr + ring.tobytes(), tmp_path)
        rc = int(np.frombuffer(out[:4], np.int32)[0])
        exp = ring.copy()
        erc = N.load_library().dk_ring_release_tpacket3(exp.ctypes.data, exp.nbytes, bs, first, nb)
        assert rc == erc and out[4:] == exp.tobytes()


def sga_rows(raw, k, base):
    """Parse k packed 40-byte demi_sgarray_t from the product lib into the driver's output row format."""
    out = []
    for j in range(k):
        s = raw[40 * j: 40 * j + 40]
        tok = int.from_bytes(s[0:8], "little")
        ns = int.from_bytes(s[8:12], "little")
        sb = int.from_bytes(s[12:20], "little")
        sl = int.from_bytes(s[20:24], "little")
        out.append((tok, (sb - base) if sb else 2**64 - 1, sl, ns, bytes(s[24:40])))
    return out


def drv_rows(out, k, with_addr=True):
    rows, p = [], 0
    for _ in range(k):
        tok, sb = np.frombuffer(out[p:p + 16], np.uint64)
        sl, ns = np.frombuffer(out[p + 16:p + 24], np.uint32)
        addr = out[p + 24:p + 40] if with_addr else b""
        rows.append((int(tok), int(sb), int(sl), int(ns), bytes(addr)))
        p += 40 if with_addr else 24
    return rows, p


def test_udp_sgarrays_fuzzed(driver, tmp_path):
    rng = np.random.default_rng(9)
    lib = N.load_library()
    for trial in range(60):
        n = int(rng.integers(0, 300))
        blob = rng.integers(0, 256, 4096 + 70000, dtype=np.uint8)
        off = rng.integers(0, 4096, n, dtype=np.uint32)
        meta = rng.choice(np.array([0, 1, 1, 1, 25, 32], np.uint32), n).astype(np.uint32) | (17 << 8)
        src = rng.integers(0, 2**32, n, dtype=np.uint32)
        ports = rng.integers(0, 2**32, n, dtype=np.uint32)
        payload = rng.integers(0, 2**32, n, dtype=np.uint32)
        cap = int(rng.choice([0, 1, n // 2, n + 5]))
        tokens = int(trial % 2)
        payload_in = (np.array([n, cap, tokens], np.uint32).tobytes() + np.array([blob.nbytes], np.uint64).tobytes()
                      + b"".join(a.tobytes() for a in (off, meta, src, ports, payload)) + blob.tobytes())
        out = run(driver, "udp", payload_in, tmp_path)
        rc, nout = np.frombuffer(out[:8], np.int32)
        idx = np.frombuffer(out[8:8 + 4 * nout], np.uint32)
        rows, _ = drv_rows(out[8 + 4 * nout:], int(nout))
        # the regular build on the same inputs
        arrs = (N.DemiSgarray * max(cap, 1))()
        eidx = np.zeros(max(cap, 1), np.uint32)
        enout = ctypes.c_uint32()
        tok = (ctypes.c_void_p * max(n, 1))(*[0x1000 + i for i in range(n)])
        p = lambda a: a.ctypes.data if n else None  # noqa: E731
        erc = lib.dk_rx_into_sgarrays(blob.ctypes.data, p(off), n, p(meta), p(src), p(ports), p(payload),
                                      tok if tokens else None, arrs if cap else None, eidx.ctypes.data if cap else None,
                                      cap, ctypes.byref(enout))
        assert (int(rc), int(nout)) == (erc, enout.value)
        assert np.array_equal(idx, eidx[: enout.value])
        exp = sga_rows(bytes(arrs), enout.value, blob.ctypes.data)
        if not tokens:  # the token is the frame address: compare relative to the blob
            exp = [((t - blob.ctypes.data) if t else t, *rest) for t, *rest in exp]
            rows = [((t - 0) if t else t, *rest) for t, *rest in rows]
            rows = [(r[1] - (payload[i] & 0xFFFF), *r[1:]) for r, i in zip(rows, idx)]
        assert rows == exp


def test_tcp_sgarrays_fuzzed(driver, tmp_path):
    rng = np.random.default_rng(10)
    lib = N.load_library()
    for trial in range(60):
        n = int(rng.integers(0, 200))
        count = int(rng.integers(0, 300))
        blob = rng.integers(0, 256, 8192, dtype=np.uint8)
        off = rng.integers(0, 4096, n, dtype=np.uint32)
        deliv = np.zeros(count, N.VIEW_DTYPE)
        deliv["ref"] = rng.integers(0, max(n, 1), count)
        deliv["ref"][rng.random(count) < 0.05] = N.DK_TCP_REF_EOF
        if trial % 7 == 3 and count:
            deliv["ref"][int(rng.integers(0, count))] = n  # out of range: EINVAL before anything is written
        deliv["off"] = rng.integers(0, 2000, count)
        deliv["len"] = rng.integers(0, 2000, count)
        cap = int(rng.choice([0, 1, count // 2, count + 3]))
        tokens = int(trial % 2)
        payload_in = (np.array([n, count, cap, tokens], np.uint32).tobytes()
                      + np.array([blob.nbytes], np.uint64).tobytes() + off.tobytes() + deliv.tobytes() + blob.tobytes())
        out = run(driver, "tcp", payload_in, tmp_path)
        rc, nout = np.frombuffer(out[:8], np.int32)
        rows, _ = drv_rows(out[8:], int(nout))
        arrs = (N.DemiSgarray * max(cap, 1))()
        enout = ctypes.c_uint32()
        tok = (ctypes.c_void_p * max(n, 1))(*[0x1000 + i for i in range(n)])
        erc = lib.dk_tcp_into_sgarrays(blob.ctypes.data, off.ctypes.data if n else None, n,
                                       deliv.ctypes.data if count else None, count, tok if tokens else None,
                                       arrs if cap else None, cap, ctypes.byref(enout))
        assert (int(rc), int(nout)) == (erc, enout.value)
        exp = sga_rows(bytes(arrs), enout.value, blob.ctypes.data)
        if not tokens:
            exp = [((t - blob.ctypes.data) if t else 0, *rest) for t, *rest in exp]
            rows = [((r[1] - int(deliv["off"][k])) if r[0] else 0, *r[1:]) for k, r in enumerate(rows)]
        assert rows == exp


def plan_ref(off, ln, fb, chunk_n, zc, max_bytes):
    """dk_rx_process_host's chunk rule (rx_plan.h), restated."""
    chunks, a, n = [], 0, len(off)
    chunk_n = max(chunk_n, 1)
    while a < n:
        lo, hi, e = None, 0, a
        while e < n and e - a < chunk_n:
            o, end = int(off[e]), int(off[e]) + int(ln[e])
            if end <= fb:
                nlo, nhi = (o & ~15) if lo is None else min(lo, o & ~15), max(hi, end)
                if not zc and e > a and nhi - nlo > max_bytes:
                    break
                lo, hi = nlo, nhi
            e += 1
        if lo is None:
            lo = hi = 0
        chunks.append((a, e, lo, hi))
        a = e
    return chunks


def test_host_chunk_planner(driver, tmp_path):
    rng = np.random.default_rng(11)
    for trial in range(80):
        n = int(rng.integers(0, 3000))
        fb = int(rng.integers(1, 1 << 22))
        off = rng.integers(0, fb + 5000, n, dtype=np.uint64).astype(np.uint32)
        if trial % 3 == 0:
            off[rng.random(n) < 0.1] = 0xFFFFFF00
        ln = rng.integers(0, 9000, n, dtype=np.uint16)
        chunk_n, zc = int(rng.choice([0, 1, 7, 1000, 65536])), int(trial % 4 == 0)
        max_bytes = int(rng.choice([1, 4096, 1 << 20, 256 << 20]))
        payload_in = (np.array([n], np.uint32).tobytes() + np.array([fb], np.uint64).tobytes()
                      + np.array([chunk_n, zc], np.uint32).tobytes() + np.array([max_bytes], np.uint64).tobytes()
                      + off.tobytes() + ln.tobytes())
        out = run(driver, "plan", payload_in, tmp_path)
        span = int(np.frombuffer(out[:8], np.uint64)[0])
        k = int(np.frombuffer(out[8:12], np.uint32)[0])
        got = []
        for j in range(k):
            a, e = np.frombuffer(out[12 + 24 * j: 20 + 24 * j], np.uint32)
            lo, hi = np.frombuffer(out[20 + 24 * j: 36 + 24 * j], np.uint64)
            got.append((int(a), int(e), int(lo), int(hi)))
        exp = plan_ref(off, ln, fb, chunk_n, zc, max_bytes)
        assert got == exp
        assert span == max([h - lo for _, _, lo, h in exp], default=0)
        assert sum(e - a for a, e, _, _ in got) == n  # every frame in exactly one chunk, in order


# --- the LDS Active table builder (lds_table.h) -------------------------------------------------------------------
M32 = 0xFFFFFFFF
ACTIVE = N.DK_FLOW_TCP_ACTIVE


def _flow_hash(kind, lip, rip, ports):  # rx_common.h flow_hash
    h = (kind * 0x9E3779B1) & M32
    h ^= lip
    h = (h * 0x85EBCA6B) & M32
    h ^= h >> 13
    h ^= rip
    h = (h * 0xC2B2AE35) & M32
    h ^= h >> 16
    h ^= ports
    h = (h * 0x27D4EB2F) & M32
    h ^= h >> 15
    return h


def _h2(kind, lip, rip):  # flow_hash's state just before `ports` is mixed in (the rest is a bijection of h2 ^ ports)
    h = (kind * 0x9E3779B1) & M32
    h ^= lip
    h = (h * 0x85EBCA6B) & M32
    h ^= h >> 13
    h ^= rip
    h = (h * 0xC2B2AE35) & M32
    h ^= h >> 16
    return h


def _fmix(h):
    h ^= h >> 16
    h = (h * 0x85EBCA6B) & M32
    h ^= h >> 13
    h = (h * 0xC2B2AE35) & M32
    h ^= h >> 16
    return h


def _mulhi(a, b):
    return (int(a) * int(b)) >> 32


def _lt_lookup(words, n, nb, lip, rip, ports):  # rx_kernels.hip lt_lookup, on the host
    h = _flow_hash(ACTIVE, lip, rip, ports)
    d = int(words[3 * n + _mulhi(h, nb)])
    sl = _mulhi(_fmix(h ^ ((d * 0x9E3779B1 + 0x7F4A7C15) & M32)), n)
    return int(words[2 * n + sl]) if int(words[sl]) == rip and int(words[n + sl]) == ports else None


def _ltable(driver, tmp_path, keys, cfg_ip, other=()):
    """keys: [(rip, ports, fid)] Active on cfg_ip; other: Active keys on another local address. Slots at random
    distinct positions of a power-of-two table (the builder scans slots, it does not re-probe)."""
    allk = [(cfg_ip, r, p, f) for r, p, f in keys] + list(other)
    cap = 16
    while cap < 2 * max(len(allk), 1):
        cap *= 2
    slots = np.zeros((cap, 4), np.uint32)
    pos = np.random.default_rng(len(allk)).permutation(cap)[: len(allk)]
    for (lip, r, p, f), at in zip(allk, pos):
        slots[at] = (ACTIVE << 24 | f, lip, r, p)
    out = run(driver, "ltable", np.array([cap, cfg_ip], np.uint32).tobytes() + slots.tobytes(), tmp_path)
    ok, n, nb, nw = np.frombuffer(out[:16], np.int32)
    return int(ok), int(n), int(nb), np.frombuffer(out[16:16 + 4 * nw], np.uint32)


def test_lds_table_builder(driver, tmp_path):
    """Random tables of 1..4096 keys: every key is found at its flow id, keys of another local address and keys not in
    the table are not; 4097 keys, two keys with one 32-bit hash, and a duplicated key are refused up front (the
    collision check runs before the displacement search, so a refusal is quick)."""
    import time

    rng = np.random.default_rng(5)
    cfg = 0x0201A8C0
    for nk in (1, 2, 3, 7, 64, 1000, 4096):
        rips = rng.integers(1, 2**32, nk, dtype=np.uint64).astype(np.uint32)
        ports = rng.integers(0, 2**32, nk, dtype=np.uint64).astype(np.uint32)
        keys = [(int(r), int(p), k) for k, (r, p) in enumerate(zip(rips, ports))]
        other = [(0x0A0A0A0A, int(rips[0]), int(ports[0]), nk + 5)]
        ok, n, nb, words = _ltable(driver, tmp_path, keys, cfg, other)
        assert ok and n == nk and nb == (nk + 3) // 4, (nk, ok, n, nb)
        for r, p, f in keys:
            assert _lt_lookup(words, n, nb, cfg, r, p) == f, (nk, r, p)
        for _ in range(200):
            assert _lt_lookup(words, n, nb, cfg, int(rng.integers(1, 2**32)), int(rng.integers(0, 2**32))) is None
    keys = [(k + 1, k, k) for k in range(4097)]
    assert _ltable(driver, tmp_path, keys, cfg)[0] == 0
    # two distinct keys with one flow_hash: same h2 ^ ports
    r1, p1, r2 = 0x01020304, 0x00500050, 0x0A0B0C0D
    p2 = _h2(ACTIVE, cfg, r1) ^ p1 ^ _h2(ACTIVE, cfg, r2)
    assert _flow_hash(ACTIVE, cfg, r1, p1) == _flow_hash(ACTIVE, cfg, r2, p2) and (r1, p1) != (r2, p2)
    for base in (0, 5, 900):
        extra = [(int(rng.integers(1, 2**32)), int(rng.integers(0, 2**32)), 10 + k) for k in range(base)]
        t = time.perf_counter()
        ok, *_ = _ltable(driver, tmp_path, extra + [(r1, p1, 1), (r2, p2, 2)], cfg)
        assert ok == 0 and time.perf_counter() - t < 20
    assert _ltable(driver, tmp_path, [(r1, p1, 1), (r1, p1, 2)], cfg)[0] == 0  # duplicated key


def _ub_hash(port, seed):
    h = (port * 0x9E3779B1 + seed) & 0xFFFFFFFF
    h ^= h >> 16
    h = (h * 0x85EBCA6B) & 0xFFFFFFFF
    h ^= h >> 13
    h = (h * 0xC2B2AE35) & 0xFFFFFFFF
    return h ^ (h >> 16)


def _ub_lookup(words, mask, seed, port):
    """rx_common.h ub_pick over the words of the port's two buckets."""
    h = _ub_hash(port, seed)
    b1, b2 = h & mask, (h >> 16) & mask
    for e in (int(words[2 * b1]), int(words[2 * b1 + 1]), int(words[2 * b2]), int(words[2 * b2 + 1])):
        if (e ^ port) & 0xFFFF == 0 and e >> 16 != 0xFFFF:
            return e >> 16
    return None


def test_udp_bind_table_builder(driver, tmp_path):
    """The compact UDP bind table (rx_common.h, lds_table.h build_udp_table: two-word buckets, load <= 1/2) from
    port-table words: 1..32,768 binds on consecutive and random ports (ports 0 and 65535 included), every bind found at
    its flow id and no unbound port found; the line count that picks it; refused for no binds, 32,769 binds and a flow
    id >= 0xFFFF."""
    rng = np.random.default_rng(7)
    none = 0xFFFFFFFF

    def build(local):
        out = run(driver, "utable", np.asarray(local, np.uint32).tobytes(), tmp_path)
        ok, mask, seed, lines = np.frombuffer(out[:16], np.uint32)
        return int(ok), int(mask), int(seed), int(lines), np.frombuffer(out[16:], np.uint32)

    for nb, spread in ((1, False), (3, True), (1024, False), (1024, True), (5000, True), (32768, True)):
        local = np.full(65536, none, np.uint32)
        ports = (rng.permutation(65536)[:nb] if spread else 5000 + np.arange(nb)).astype(np.int64)
        if spread and nb > 2:
            ports[0], ports[1] = 65535, 0
            ports = np.unique(ports)
        fids = rng.permutation(0xFFFF)[:len(ports)]
        local[ports] = fids
        ok, mask, seed, lines, words = build(local)
        assert ok and len(words) == 2 * (mask + 1) and mask + 1 >= len(ports) and (mask + 1) & mask == 0, (nb, ok, mask)
        assert lines == len(set(int(p) >> 5 for p in ports)), (nb, lines)
        for p, f in zip(ports, fids):
            assert _ub_lookup(words, mask, seed, int(p)) == int(f), (nb, p)
        bound = set(int(p) for p in ports)
        for p in rng.integers(0, 65536, 300):
            if int(p) not in bound:
                assert _ub_lookup(words, mask, seed, int(p)) is None
    assert build(np.full(65536, none, np.uint32))[0] == 0
    local = np.full(65536, none, np.uint32)
    local[:32769] = np.arange(32769)
    assert build(local)[0] == 0
    local = np.full(65536, none, np.uint32)
    local[80] = 0xFFFF
    assert build(local)[0] == 0
