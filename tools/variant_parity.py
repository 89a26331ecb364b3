#!/usr/bin/env python3
"""Bit-exact check of tuning-variant libraries (tools/variants.sh) against the oracle before their timings are trusted:
    python tools/variant_parity.py --lib build/variants/x.so [--lib ...]
Per library: IMIX, 576-byte, 64-byte UDP, 1078-byte and 1500-byte TCP batches with a 2 % corrupted tail, frames at 64-byte slots
(aligned) and shifted to 2 mod 16; every result array and both counters against OraclePeer. One JSON line per case."""
import argparse
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--lib", action="append", default=[])
    ap.add_argument("--frames", type=int, default=1 << 16)
    args = ap.parse_args()
    import torch

    from demikernel_amd import Config, FrameBatch, RxEngine, synth
    from oracle.oracle import OraclePeer

    bad_total = 0
    cases = [("imix", "imix", "tcp"), ("576", 562, "tcp"), ("udp64", 50, "udp"), ("c1_1078", 1064, "tcp"), ("c2_1486", 1486, "tcp")]
    for lp in args.lib:
        eng = RxEngine(Config(synth.BOB_IPV4), lib_path=os.path.abspath(lp))
        for name, ip, kind in cases:
            flows = synth.make_flows(64, kind=kind)
            n = args.frames
            ipl = synth.imix_ip_lengths(n, seed=5) if ip == "imix" else ip
            tr = synth.traffic(n, ipl, flows, seed=5)
            blob, off, lens = synth.build_numpy(tr, seed=5)
            synth.corrupt_numpy(blob, off, synth.corruption_plan(n, 0.02, tr, 5))
            for shift in (0, 2):
                b2 = np.zeros(len(blob) + 16, np.uint8)
                b2[shift:shift + len(blob)] = blob
                o2 = (off.astype(np.int64) + shift).astype(np.uint32)
                eng.set_sockets(flows)
                r = eng.results(n, tcp_fields=True)
                eng.receive_batch(FrameBatch.from_numpy(b2, o2, lens), r)
                torch.cuda.synchronize()
                got = r.to_numpy()
                ref = OraclePeer(synth.ipv4(synth.BOB_IPV4))
                ref.set_flows(flows)
                exp = ref.process(b2, o2, lens)
                diff = {k: int((v != exp[k][: len(v)]).sum()) for k, v in got.items()}
                nbad = sum(diff.values())
                bad_total += nbad
                print(json.dumps({"lib": os.path.basename(lp), "case": name, "shift": shift, "ok": nbad == 0,
                                  "mismatches": {k: v for k, v in diff.items() if v}}), flush=True)
    sys.exit(1 if bad_total else 0)


if __name__ == "__main__":
    main()
