#!/usr/bin/env python3
"""Writes the committed golden fixtures under tests/golden/ (run from the repo root: python tests/golden/make_golden.py).

What each fixture pins (DESIGN.md "Oracle and parity"):
  ipv4_unit_vectors.npz  The IPv4 datagrams of the reference's own unit tests (src/rust/inetstack/protocols/layer3/
                         ipv4/tests.rs, built with the same field values and its build_ipv4_header helper, restated in
                         tests/frames.py::ipv4_header) and the outcome each test asserts: ok (and for the good-parse
                         test the src/dst/protocol/payload it checks) or error. These expectations come from the
                         reference's test code, not from our oracle.
  udp_header_kat.npz     The UDP header bytes of layer4/udp/header.rs:206-252 (parse with offload on: ports 0x32 and
                         0x45, 8 payload bytes left).
  verdict_corpus.npz     A frame for every SURVEY.md Appendix A branch (tests/frames.py::verdict_corpus) with the verdict
                         it was built to produce (hand-derived from the reference lines cited there) and the full result
                         record the oracle computes for it.
  mixed_batch.npz        1,000 synthetic frames (TCP/UDP, IMIX sizes, 5 % corrupted) with the oracle's result arrays:
                         a regression pin for the oracle and a fixed vector set for the GPU parity test.
Inputs only depend on seeded generators; nothing here reads /root/reference.
"""
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))

import frames as F  # noqa: E402
from demikernel_amd import VERDICTS, ipv4, synth  # noqa: E402
from demikernel_amd.synth import ALICE_IPV4, BOB_IPV4  # noqa: E402
from oracle.oracle import OraclePeer  # noqa: E402

UDP = 17


def ipv4_unit_vectors():
    """(datagram bytes, expect_ok, test name) for every case of layer3/ipv4/tests.rs."""
    cases = []

    def hdr(**kw):
        base = dict(version=4, ihl=5, dscp=0, ecn=0, total_length=20, ident=0, flags=0x2, frag=0, ttl=1, proto=UDP,
                    src=ALICE_IPV4, dst=BOB_IPV4, checksum=None)
        base.update(kw)
        return F.ipv4_header(**base)

    data = bytes([1, 2, 3, 4, 5, 6, 7, 8])
    for ihl in range(5, 16):  # test_ipv4_header_parse_good (:80)
        hs = ihl * 4
        h = bytearray(hs)
        h[:] = hdr(ihl=ihl, total_length=hs + 8)[:20] + bytes(hs - 20)
        cases.append((bytes(h) + data, True, f"parse_good_ihl{ihl}"))
    for v in (0, 1, 2, 3, 5, 7, 8, 9, 10, 11, 12, 13, 14, 15):  # invalid_version (:136)
        cases.append((hdr(version=v), False, f"invalid_version_{v}"))
    for ihl in range(0, 5):  # invalid_ihl (:176)
        cases.append((hdr(ihl=ihl)[:20], False, f"invalid_ihl_{ihl}"))
    for tl in range(0, 20):  # invalid_total_length (:217)
        cases.append((hdr(total_length=tl), False, f"invalid_total_length_{tl}"))
    cases.append((hdr(ident=0x1D, flags=0x4), False, "invalid_flags_evil"))  # (:258)
    cases.append((hdr(ttl=0), False, "invalid_ttl"))  # (:296)
    for p in range(144, 252):  # invalid_protocol (:334)
        cases.append((hdr(proto=p), False, f"invalid_protocol_{p}"))
    cases.append((hdr(checksum=0x1), False, "invalid_header_checksum"))  # (:375)
    for d in range(1, 63):  # unsupported_dscp: accepted (:417)
        cases.append((hdr(dscp=d), True, f"dscp_{d}"))
    for e in range(1, 3):  # unsupported_ecn: accepted (:458)
        cases.append((hdr(ecn=e), True, f"ecn_{e}"))
    cases.append((hdr(ident=0x1D, flags=0x1), False, "unsupported_fragmentation_mf"))  # (:501)
    cases.append((hdr(ident=0x1D, flags=0x2, frag=1), False, "unsupported_fragmentation_offset"))
    for p in range(0, 143):  # unsupported_protocol (:575)
        if p in (1, 6, 17):
            continue
        cases.append((hdr(proto=p), False, f"unsupported_protocol_{p}"))
    return cases


def pack_var(items):
    lens = np.array([len(x) for x in items], np.int64)
    off = np.zeros(len(items), np.int64)
    np.cumsum(lens[:-1], out=off[1:])
    blob = np.frombuffer(b"".join(items), np.uint8) if items else np.zeros(0, np.uint8)
    return blob.copy(), off, lens


def main():
    out = {}
    iv = ipv4_unit_vectors()
    blob, off, lens = pack_var([c[0] for c in iv])
    out["ipv4_unit_vectors"] = dict(blob=blob, off=off, len=lens, expect_ok=np.array([c[1] for c in iv]),
                                    name=np.array([c[2] for c in iv]))

    hdr = bytes([0x0, 0x32, 0x0, 0x45, 0x0, 0x10, 0x0, 0x0])
    payload = bytes([0x0, 0x1, 0x0, 0x1, 0x0, 0x1, 0x0, 0x1])
    out["udp_header_kat"] = dict(segment=np.frombuffer(hdr + payload, np.uint8).copy(),
                                 src=np.uint32(ipv4("198.0.0.1")), dst=np.uint32(ipv4("198.0.0.2")),
                                 sport=np.uint16(0x32), dport=np.uint16(0x45), payload_len=np.uint32(8),
                                 serialized_header=np.frombuffer(hdr, np.uint8).copy())

    C = F.verdict_corpus()
    blob, off, lens = F.pack([c[1] for c in C])
    flows = F.corpus_flows()
    p = OraclePeer(ipv4(BOB_IPV4))
    p.set_flows(flows)
    r = p.process(blob, off, lens)
    out["verdict_corpus"] = dict(blob=blob, off=off, len=lens, flows=flows.view(np.uint8),
                                 expected_verdict=np.array([VERDICTS.index(c[2]) for c in C], np.uint8),
                                 name=np.array([c[0] for c in C]), **{f"res_{k}": v for k, v in r.items()})

    flows = np.concatenate([synth.make_flows(128), synth.make_flows(16, kind="udp")])
    n = 1000
    tr = synth.traffic(n, synth.imix_ip_lengths(n, seed=77), flows, seed=77)
    blob, off, lens = synth.build_numpy(tr, seed=77)
    synth.corrupt_numpy(blob, off, synth.corruption_plan(n, 0.05, tr, seed=77))
    p = OraclePeer(ipv4(BOB_IPV4))
    p.set_flows(flows)
    r = p.process(blob, off, lens)
    out["mixed_batch"] = dict(blob=blob, off=off, len=lens, flows=flows.view(np.uint8),
                              **{f"res_{k}": v for k, v in r.items()})

    for name, arrays in out.items():
        np.savez_compressed(os.path.join(HERE, name + ".npz"), **arrays)
        print(name, {k: v.shape for k, v in arrays.items()})


if __name__ == "__main__":
    main()
