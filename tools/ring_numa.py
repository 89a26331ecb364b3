#!/usr/bin/env python3
"""does the TPACKET_V3 ring path lose to the packed host path because of where the ring's pages
land? One process, the same 1500-byte frames in the same ring layout, the ring buffer made four ways:
  first_touch   as bench.py does: an anonymous mmap filled by the host thread (pages wherever that thread runs),
                then hipHostRegister (dk_ring_register);
  hip_host      hipHostMalloc'd (a pinned torch tensor) and filled (no registration needed);
  bind_gpu      the mmap bound to the GPU's NUMA node (mbind MPOL_BIND) before the first touch, then registered;
  bind_other    the same bound to another node (the contrast), when the host has one.
For each: the NUMA nodes of its pages (move_pages query on every 16th page), then the ring path (dk_rx_process_tpacket3,
block scan + kernel reading the ring in place (host_zc 1) / through staged copies (+staged, the default since round 6)
+ results back) `--reps` times interleaved, median GB/s of frame bytes, and the packed host path (dk_rx_process_host
from pinned memory, read in place) beside them. One JSON line per form."""
import argparse
import ctypes
import json
import mmap
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

LIBC = ctypes.CDLL(None, use_errno=True)
SYS_MBIND, SYS_MOVE_PAGES = 237, 279  # x86_64
MPOL_BIND = 2
PAGE = mmap.PAGESIZE


def gpu_numa_node(dev=0):
    import torch

    p = torch.cuda.get_device_properties(dev)
    bdf = f"{getattr(p, 'pci_domain_id', 0):04x}:{p.pci_bus_id:02x}:{p.pci_device_id:02x}.0"
    try:
        with open(f"/sys/bus/pci/devices/{bdf}/numa_node") as f:
            return int(f.read().strip()), bdf
    except OSError:
        return -1, bdf


def host_nodes():
    try:
        with open("/sys/devices/system/node/online") as f:
            spec = f.read().strip()
    except OSError:
        return [0]
    out = []
    for part in spec.split(","):
        a, _, b = part.partition("-")
        out += list(range(int(a), int(b or a) + 1))
    return out


def page_nodes(addr, nbytes, every=16):
    """Node of every `every`-th page (move_pages with nodes = NULL: query only)."""
    pages = [addr + k * PAGE for k in range(0, nbytes // PAGE, every)]
    arr = (ctypes.c_void_p * len(pages))(*pages)
    status = (ctypes.c_int * len(pages))()
    rc = LIBC.syscall(SYS_MOVE_PAGES, 0, ctypes.c_ulong(len(pages)), arr, None, status, 0)
    if rc != 0:
        return {"error": f"move_pages errno {ctypes.get_errno()}"}
    h = {}
    for s in status:
        k = str(s) if s >= 0 else f"err{-s}"
        h[k] = h.get(k, 0) + 1
    return h


def bound_mmap(nbytes, node):
    m = mmap.mmap(-1, nbytes, flags=mmap.MAP_PRIVATE | mmap.MAP_ANONYMOUS)
    a = np.frombuffer(m, np.uint8, count=nbytes)
    mask = (ctypes.c_ulong * 16)()
    mask[node // 64] = 1 << (node % 64)
    rc = LIBC.syscall(SYS_MBIND, ctypes.c_void_p(a.ctypes.data), ctypes.c_ulong(nbytes), MPOL_BIND, mask,
                      ctypes.c_ulong(16 * 64), 0)
    return a, (None if rc == 0 else f"mbind errno {ctypes.get_errno()}")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--frames", type=int, default=1 << 19)
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--block", type=int, default=1 << 22)
    a = ap.parse_args()
    import torch

    from demikernel_amd import Config, RxEngine, RxResults, synth
    from demikernel_amd import ring as RG

    n = a.frames
    flows = synth.make_flows(1024)
    tr = synth.traffic(n, np.full(n, 1486, np.uint16), flows, seed=synth.SEED + 5)
    packed, poff, lens = synth.build_numpy(tr)
    eng = RxEngine(Config(synth.BOB_IPV4), device=0, tuning={"host_zc": 1})  # the ring read in place (zero-copy)
    eng.set_sockets(flows)
    res = RxResults(n, len(flows), host=True)
    nbytes = int(lens.astype(np.int64).sum())
    gnode, bdf = gpu_numa_node()
    nodes = host_nodes()
    template, used, exp_off, elen = RG.build_tpacket3(packed, poff, lens, a.block)
    size = template.nbytes
    print(json.dumps({"gpu_bdf": bdf, "gpu_numa_node": gnode, "host_nodes": nodes, "ring_bytes": size,
                      "frames": n, "cpu": os.sched_getaffinity(0).__len__()}), flush=True)

    forms = {}
    ft = RG.page_aligned_empty(size)
    ft[:] = template
    forms["first_touch"] = (ft, True, None)
    hh = torch.empty(size, dtype=torch.uint8, pin_memory=True)
    hn = hh.numpy()
    hn[:] = template
    forms["hip_host"] = (hn, False, None)
    if gnode >= 0:
        b, err = bound_mmap(size, gnode)
        b[:] = template
        forms["bind_gpu"] = (b, True, err)
        other = [x for x in nodes if x != gnode]
        if other:
            o, err = bound_mmap(size, other[0])
            o[:] = template
            forms["bind_other"] = (o, True, err)
    rings = {k: RG.TpacketRing(buf, a.block, register=reg) for k, (buf, reg, _) in forms.items()}
    # the same rings through staged copies (the copy engine moves each chunk's byte range to HBM: layout-blind; the
    # ring path's default since round 6)
    eng_st = RxEngine(Config(synth.BOB_IPV4), device=0, tuning={"host_zc": 0})
    eng_st.set_sockets(flows)
    # the packed host path from pinned memory, as bench.py host_path
    pin = torch.from_numpy(packed).pin_memory().numpy()
    rates = {k: [] for k in list(rings) + [k + "+staged" for k in rings] + ["packed_pinned"]}
    for rep in range(a.reps):
        for k, r in rings.items():
            for e, kk in ((eng, k), (eng_st, k + "+staged")):
                t = time.perf_counter()
                nf, nb = r.receive(e, 0, used, res)
                rates[kk].append(nbytes / (time.perf_counter() - t) / 1e9)
                assert nf == n and nb == used
        t = time.perf_counter()
        eng.receive_batch_host(pin, poff, lens, res)
        rates["packed_pinned"].append(nbytes / (time.perf_counter() - t) / 1e9)
    for k in rates:
        base = k.split("+")[0]
        buf = forms[base][0] if base in forms else pin
        row = {"form": k, "gbps": round(float(np.median(rates[k])), 2), "gbps_max": round(max(rates[k]), 2),
               "page_nodes": page_nodes(buf.ctypes.data, buf.nbytes)}
        if base in forms and forms[base][2]:
            row["bind_error"] = forms[base][2]
        print(json.dumps(row), flush=True)
    for r in rings.values():
        r.close()


if __name__ == "__main__":
    main()
