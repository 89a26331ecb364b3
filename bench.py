#!/usr/bin/env python3
"""Benchmark: device-resident receive-path transform (checksum + parse + demux) on MI355X.

    python bench.py --gpus N --steps K --warmup W          (N > 1: launched by torch.distributed.run)

A step = one dk_rx_process pass over one HBM-resident batch of the workload (default: BASELINE config 2,
1,048,576 x 1500 B IPv4/TCP frames over 1,024 flows, 1 % corrupted tail), plus, for N > 1, the RCCL all-reduce of the
per-flow packet counts (the only collective on this path). Weak scaling: every rank owns one batch (its packet shard).
`value` = sum of frame bytes processed by all ranks / max-over-ranks time.  Rank 0 prints one JSON line.
"""
from __future__ import annotations

import argparse
import ctypes
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md)
DESC_BYTES = 6         # u32 offset + u16 length per frame
RESULT_BYTES = 24      # meta, src_ip, dst_ip, ports, payload, flow_id (u32 each)

WORKLOADS = {
    # name: (description, frames, ip_len spec, flow kind, nflows)
    "c2_tcp1500": ("1M x 1500B IPv4/TCP, 1024 flows, device-resident", 1 << 20, 1486, "tcp", 1024),
    "c3_udp64": ("1M x 64B IPv4/UDP (min-size), device-resident, 8 rotating batches", 1 << 20, 50, "udp", 1024),
    "c4_imix": ("IMIX 40/576/1500 at 7:4:1, 2M frames per GPU (16M over 8 GPUs)", 1 << 21, "imix", "tcp", 1024),
    "c5_tcp1500_10k": ("1500B IPv4/TCP, 10k flows, 2M frames per GPU (16M over 8 GPUs)", 1 << 21, 1486, "tcp", 10000),
}


def dist_env():
    ws = int(os.environ.get("WORLD_SIZE", "1"))
    return int(os.environ.get("RANK", "0")), int(os.environ.get("LOCAL_RANK", "0")), ws


def make_batch(eng, name, rank, seed_base, world=1):
    """This rank's packet shard of the global batch (world x frames-per-GPU frames, weak scaling): the frame-size
    sequence is global and seeded, the shard boundaries are byte-balanced (demikernel_amd.shard), and each rank
    synthesises only its own frames on its own GPU."""
    from demikernel_amd import synth
    from demikernel_amd.shard import byte_balanced_shards

    _, n, ip_len, kind, nflows = WORKLOADS[name]
    flows = synth.make_flows(nflows, kind=kind)
    total = n * world
    ip_all = synth.imix_ip_lengths(total, seed_base) if ip_len == "imix" else np.full(total, ip_len, np.uint16)
    frame_all = np.maximum(ip_all.astype(np.int64) + 14, synth.ETH_MIN_FRAME)
    a, b = byte_balanced_shards(frame_all, world)[rank]
    seed = seed_base + 7919 * rank
    n = b - a
    tr = synth.traffic(n, ip_all[a:b], flows, seed=seed)
    eng.set_sockets(flows)
    batch = synth.build_device(tr, eng, seed=seed)
    synth.corrupt_device(batch, batch.off.cpu().numpy().view(np.uint32), synth.corruption_plan(n, 0.01, tr, seed))
    return batch, flows, tr


def time_kernel(eng, batches, res, steps, warmup, stream, dist=None, counts_allreduce=False):
    """Run warmup + timed steps. A step = the receive pass over one batch (+ for N > 1 the all-reduce of this step's
    per-flow counts). For N > 1 the counters are double-buffered and the all-reduce is issued asynchronously (RCCL runs
    on its own stream), so step k's reduction overlaps step k+1's kernel.
    Returns (wall seconds for `steps`, per-launch kernel seconds, per-step collective seconds measured unoverlapped)."""
    import torch

    gloo = dist is not None and dist.get_backend() == "gloo"
    bufs = [res.t["flow_counts"], torch.zeros_like(res.t["flow_counts"])] if counts_allreduce else []
    pending = [None, None]

    def reduce(buf, async_op):
        if gloo:  # rehearsal only: gloo reduces a host copy, synchronously
            h = buf.cpu()
            dist.all_reduce(h)
            buf.copy_(h)
            return None
        return dist.all_reduce(buf, async_op=async_op)

    def step(k):
        b = batches[k % len(batches)]
        if counts_allreduce:
            slot = k % 2
            if pending[slot] is not None:
                pending[slot].wait()  # stream dependency: the buffer's previous all-reduce has finished
                pending[slot] = None
            bufs[slot].zero_()
            res.t["flow_counts"] = bufs[slot]
        eng.receive_batch(b, res, stream=stream)
        if counts_allreduce:
            pending[k % 2] = reduce(bufs[k % 2], True)

    def drain():
        for slot in (0, 1):
            if pending[slot] is not None:
                pending[slot].wait()
                pending[slot] = None

    for k in range(warmup):
        step(k)
    drain()
    torch.cuda.synchronize()
    if dist is not None:
        dist.barrier()
    torch.cuda.synchronize()
    # HIP events bracket the timed region only (an event pair around every launch adds a marker + cache writeback per
    # step and perturbs the kernel it measures): per-launch time = region / steps, i.e. dk_rx_kernel plus the small
    # dk_flow_reduce_kernel and launch gaps (rocprofv3 kernel stats in profiles/ split the two kernels).
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    t0 = time.perf_counter()
    e0.record(stream)
    for k in range(steps):
        step(k)
    e1.record(stream)
    drain()
    torch.cuda.synchronize()
    if dist is not None:
        dist.barrier()
    torch.cuda.synchronize()
    wall = time.perf_counter() - t0
    kern = [e0.elapsed_time(e1) / 1e3 / steps]
    coll = []
    if counts_allreduce:  # the collective alone, unoverlapped, for the report
        for _ in range(5):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(stream)
            reduce(bufs[0], False)
            e1.record(stream)
            torch.cuda.synchronize()
            coll.append(e0.elapsed_time(e1) / 1e3)
    return wall, kern, coll


def cpu_baseline(batch, flows, sample_frames, min_seconds, threads=1):
    """Oracle (CPU restatement of the reference) on a bounded sample of the same workload, host cores."""
    from demikernel_amd import ipv4, synth
    from oracle.oracle import OraclePeer

    n = min(sample_frames, batch.n)
    off = batch.off[:n].cpu().numpy().view(np.uint32).copy()
    lens = batch.len[:n].cpu().numpy().view(np.uint16).copy()
    end = int(off[-1]) + int(lens[-1])
    blob = batch.blob[:end].cpu().numpy()
    peer = OraclePeer(ipv4(synth.BOB_IPV4))
    peer.set_flows(flows)
    nbytes = int(lens.astype(np.int64).sum())
    rates, used, t_all = [], 1, time.perf_counter()
    while time.perf_counter() - t_all < min_seconds or len(rates) < 3:
        t = time.perf_counter()
        if threads == 1:
            peer.process(blob, off, lens)
        else:
            _, used = peer.process_mt(blob, off, lens, threads)
        rates.append(nbytes / (time.perf_counter() - t) / 1e9)
    return float(np.median(rates)), used, n, nbytes, len(rates)


def host_path_rate(eng, batch, flows, nframes, reps=3):
    """End-to-end GB/s of frame bytes for a pinned host batch through dk_rx_process_host (PCIe-inclusive)."""
    import torch

    from demikernel_amd import RxResults

    n = min(nframes, batch.n)
    off = batch.off[:n].cpu().numpy().view(np.uint32).copy()
    lens = batch.len[:n].cpu().numpy().view(np.uint16).copy()
    end = int(off[-1]) + int(lens[-1])
    pinned = torch.empty(end, dtype=torch.uint8, pin_memory=True)
    pinned.copy_(batch.blob[:end])
    off_p = torch.from_numpy(off.view(np.int32)).pin_memory()
    len_p = torch.from_numpy(lens.view(np.int16)).pin_memory()
    res = RxResults(n, len(flows), host=True)
    nbytes = int(lens.astype(np.int64).sum())
    rates = []
    for _ in range(reps):
        t = time.perf_counter()
        eng.receive_batch_host(pinned.numpy(), off_p.numpy(), len_p.numpy(), res)
        rates.append(nbytes / (time.perf_counter() - t) / 1e9)
    return {"gbps": round(max(rates), 2), "frames": n, "bytes": nbytes, "reps": reps,
            "pipeline": "3 streams, 65536-frame chunks, pinned host memory (dk_rx_process_host)"}


def ring_path_rate(eng, batch, flows, nframes, block_size=1 << 22, reps=3):
    """end-to-end GB/s of frame bytes for frames sitting in a TPACKET_V3 receive ring (the
    layout AF_PACKET fills; page-locked with hipHostRegister): block scan on the host, H2D of the blocks' byte ranges,
    kernel, D2H of the results (dk_rx_process_tpacket3). PCIe-inclusive; reported beside `value`, never as `value`."""
    from demikernel_amd import RxResults
    from demikernel_amd import ring as RG

    n = min(nframes, batch.n)
    off = batch.off[:n].cpu().numpy().view(np.uint32).astype(np.int64)
    lens = batch.len[:n].cpu().numpy().view(np.uint16).copy()
    end = int(off[-1]) + int(lens[-1])
    blob = batch.blob[:end].cpu().numpy()
    ring, used, _, elen = RG.build_tpacket3(blob, off, lens, block_size)
    r = RG.TpacketRing(ring, block_size)
    res = RxResults(n, len(flows), host=True)
    nbytes = int(elen.astype(np.int64).sum())
    rates = []
    try:
        for _ in range(reps):
            t = time.perf_counter()
            nf, nb = r.receive(eng, 0, used, res)
            rates.append(nbytes / (time.perf_counter() - t) / 1e9)
            assert nf == n and nb == used
    finally:
        r.close()
    return {"gbps": round(max(rates), 2), "frames": n, "bytes": nbytes, "blocks": used, "block_size": block_size,
            "reps": reps, "pipeline": "TPACKET_V3 block scan + dk_rx_process_host over the registered ring"}


def tcp_rate(stream, nseg=1 << 20, nconns=1 << 14, iters=10, cpu_seconds=3.0):
    """dk_tcp_rx_process over one dk_rx batch's results (nseg 1460-byte TCP segments spread
    over nconns established connections, reordered / duplicated / stray as synth.tcp_streams makes them), Mseg/s from
    HIP events around each call (the connection table is restored from a pristine copy between calls, outside the
    timed span); the CPU restatement (oracle/dk_tcp_oracle.cpp, 1 thread) on the same arrays beside it."""
    import torch

    from demikernel_amd import RxResults, synth
    from demikernel_amd.tcp import TcpOut, TcpReceiver
    from oracle import oracle as O

    dev = stream.device
    _, tr, table = synth.tcp_streams(nseg, nconns, 1500, buffer_size=1 << 24)
    rx = {"meta": (6 << 8 | tr.flags.astype(np.uint32) << 16 | 0x50 << 24).astype(np.uint32),
          "flow_id": tr.flow.astype(np.uint32), "tcp_seq": tr.seq, "tcp_ack": tr.ack,
          "payload": (54 | (tr.ip_len.astype(np.uint32) - 40) << 16).astype(np.uint32)}
    r = RxResults(nseg, 1, device=dev, tcp_fields=True, counts=False)
    for k, v in rx.items():
        r.t[k].copy_(torch.from_numpy(v.view(np.int32)))
    tcp = TcpReceiver(dev.index or 0)
    pristine = tcp.conns_to_device(table)
    conns = pristine.clone()
    out = TcpOut(nseg, len(table), dev.index or 0)
    times = []
    with torch.cuda.stream(stream):
        for i in range(iters + 2):
            conns.copy_(pristine)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(stream)
            tcp.process(r, conns, out, stream=stream)
            e1.record(stream)
            torch.cuda.synchronize()
            if i >= 2:
                times.append(e0.elapsed_time(e1) / 1e3)
    got = out.to_numpy()
    hist = np.bincount(got["action"], minlength=13)
    t = float(np.median(times))
    tcp.close()
    # CPU restatement on the same segments (bounded: repeat until cpu_seconds)
    reps, t0 = 0, time.perf_counter()
    while True:
        O.tcp_process(table.copy(), rx)
        reps += 1
        if time.perf_counter() - t0 >= cpu_seconds:
            break
    tc = (time.perf_counter() - t0) / reps
    return {"mseg_s": round(nseg / t / 1e6, 1), "ms_avg": round(t * 1e3, 4), "segments": nseg, "connections": nconns,
            "delivered_frac": round(float(hist[1]) / nseg, 3),
            "cpu_baseline": {"mseg_s": round(nseg / tc / 1e6, 2), "cores": 1, "kind": "port", "reps": reps},
            "walk": "wave" if nseg >= 8 * nconns else "lane",
            "pipeline": "key + onesweep radix sort (rocPRIM) + ranges + per-connection walk (lanes = connections, "
                        "store in LDS; one wave per connection with a parallel 64-segment check at >= 8 "
                        "segments per connection)"}


def rx_kernel_name(frame_bytes, n):
    """The receive kernel family the host picks for a batch (rx_host.cpp launch_batch: mean blob bytes per frame; the
    blob holds 64-byte-aligned slots, so its size is rounded up per frame)."""
    per = frame_bytes // max(n, 1)
    return ("dk_rx_small_kernel" if per <= 96 else "dk_rx_split_kernel" if per >= 1024 else
            "dk_rx_kernel (staged)" if per >= 128 else "dk_rx_kernel")


def tx_rate(eng, batch, frame_bytes, stream, iters=20):
    """dk_tx_checksum kernel time over an HBM-resident batch: frame bytes read, 2 checksum fields written per frame."""
    import torch

    for _ in range(3):
        eng.tx_checksum(batch, stream=stream)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(stream)
    for _ in range(iters):
        eng.tx_checksum(batch, stream=stream)
    e1.record(stream)
    torch.cuda.synchronize()
    t = e0.elapsed_time(e1) / 1e3 / iters
    algo = frame_bytes + batch.n * (DESC_BYTES + 4)
    return {"gbps": round(frame_bytes / t / 1e9, 1), "kernel_ms_avg": round(t * 1e3, 4),
            "roofline_achieved_gbps": round(algo / t / 1e9, 1), "roofline_frac": round(algo / t / 1e9 / HBM_PEAK_GBS, 4),
            "algorithmic_bytes_per_launch": algo,
            "kernel": "dk_tx_split_kernel" if frame_bytes // max(batch.n, 1) >= 1024 else "dk_tx_kernel"}


def read_ceiling(batch, stream, iters=10):
    """On-box streaming-read ceiling: dk_diag_read_probe over the same frame blob, register loads
    (global mode 3, buffer mode 6) and LDS-DMA (mode 4), 4 and 8 waves per CU; best GB/s and its configuration."""
    import torch

    from demikernel_amd import _native as N

    lib = N.load_library()
    nbytes = batch.blob.numel() // 16 * 16
    cus = torch.cuda.get_device_properties(batch.blob.device).multi_processor_count
    best = (0.0, "")
    names = {3: "global_load register", 4: "LDS-DMA", 6: "buffer_load register"}
    for mode in (3, 4, 6):
        for per_cu in (4, 8):
            grid = per_cu * cus // 4  # 256-thread workgroups: 4 waves each
            scratch = torch.zeros(grid, dtype=torch.int32, device=batch.blob.device)
            call = lambda: lib.dk_diag_read_probe(ctypes.c_void_p(batch.blob.data_ptr()), nbytes,  # noqa: E731
                                                  ctypes.c_void_p(scratch.data_ptr()), grid, mode,
                                                  ctypes.c_void_p(stream.cuda_stream))
            for _ in range(3):
                call()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(stream)
            for _ in range(iters):
                call()
            e1.record(stream)
            torch.cuda.synchronize()
            gbs = nbytes / (e0.elapsed_time(e1) / 1e3 / iters) / 1e9
            if gbs > best[0]:
                best = (gbs, f"dk_diag_read_probe mode {mode} ({names[mode]} loads), "
                             f"{per_cu} waves/CU, {nbytes / 1e9:.2f} GB")
    return best


def load_traffic_profile(workload):
    """HBM bytes per launch from the committed rocprofv3 --pmc summary (profiles/), if one exists for this workload."""
    p = os.path.join(ROOT, "profiles", "pmc_traffic.json")
    if not os.path.exists(p):
        return None
    try:
        d = json.load(open(p))
        return d.get(workload, {}).get("hbm_bytes_per_launch")
    except Exception:
        return None


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--workload", default="c2_tcp1500", choices=sorted(WORKLOADS))
    ap.add_argument("--cpu-seconds", type=float, default=10.0)
    ap.add_argument("--cpu-sample", type=int, default=1 << 17)
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--host-frames", type=int, default=1 << 19)
    ap.add_argument("--no-extras", action="store_true")
    ap.add_argument("--backend", default="nccl", choices=["nccl", "gloo"],
                    help="collective backend for N > 1 (nccl = RCCL on ROCm; gloo only to rehearse on one GPU)")
    args = ap.parse_args()

    import torch

    rank, local_rank, world = dist_env()
    dist = None
    if world > 1:
        import torch.distributed as dist  # noqa: F811

        local_dev = local_rank % max(torch.cuda.device_count(), 1)
        torch.cuda.set_device(local_dev)
        if args.backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", local_dev))
        else:
            dist.init_process_group("gloo")
    else:
        torch.cuda.set_device(0)
    dev = torch.cuda.current_device()

    from demikernel_amd import Config, RxEngine, synth

    eng = RxEngine(Config(synth.BOB_IPV4), device=dev)
    stream = torch.cuda.current_stream(dev)
    name = args.workload
    batch, flows, tr = make_batch(eng, name, rank, synth.SEED, world)
    batches = [batch]
    if name == "c3_udp64":  # 64 B batches fit in the 256 MB MALL: rotate 8 distinct batches (> 512 MB)
        batches += [make_batch(eng, name, rank, synth.SEED + 1000 * k, world)[0] for k in range(1, 8)]
    res = eng.results(batch.n)
    frame_bytes = int(tr.frame_len.astype(np.int64).sum())

    wall, kern, coll = time_kernel(eng, batches, res, args.steps, args.warmup, stream, dist,
                                   counts_allreduce=world > 1)
    if dist is not None:
        cdev = "cuda" if args.backend == "nccl" else "cpu"
        t = torch.tensor([wall], dtype=torch.float64, device=cdev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        wall = float(t.item())
        tb = torch.tensor([frame_bytes, batch.n], dtype=torch.int64, device=cdev)
        dist.all_reduce(tb)
        total_bytes, total_frames = int(tb[0]), int(tb[1])
    else:
        total_bytes, total_frames = frame_bytes, batch.n

    value = total_bytes * args.steps / wall / 1e9
    kern_avg = float(np.mean(kern))
    algo = frame_bytes + batch.n * (DESC_BYTES + RESULT_BYTES)
    achieved = algo / kern_avg / 1e9
    traffic = load_traffic_profile(name)

    out = {
        "metric": "GB/s packet bytes checksummed+parsed (device-resident)",
        "value": round(value, 2),
        "unit": "GB/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(wall / args.steps * 1e3, 4),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "u8",
        "data": "synthetic (seeded frames generated on device; 1% corrupted tail)",
        "config": {"workload": WORKLOADS[name][0], "name": name, "frames_per_gpu": batch.n,
                   "global_frames": total_frames, "parallelism": f"packet-shard x{world}",
                   "collective": ("all_reduce(flow_counts, u64) per step, async, double-buffered (overlaps the next "
                                  "step's kernel)") if world > 1 else "none"},
        "mpkt_s": round(total_frames * args.steps / wall / 1e6, 2),
        "roofline": {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": traffic,
                     "kernel_ms_avg": round(kern_avg * 1e3, 4),
                     "algorithmic_bytes_per_launch": algo, "kernel": rx_kernel_name(frame_bytes, batch.n)},
    }
    if not args.no_extras:
        ceil_gbs, ceil_cfg = read_ceiling(batch, stream)
        out["roofline"]["measured_read_ceiling"] = {"value": round(ceil_gbs, 1), "unit": "GB/s", "probe": ceil_cfg,
                                                    "frac": round(achieved / ceil_gbs, 4)}
    if coll:
        out["collective_ms_avg"] = round(float(np.mean(coll)) * 1e3, 4)
    if rank == 0 and world == 1 and not args.no_cpu:
        gbs, used, n_s, nb_s, reps = cpu_baseline(batch, flows, args.cpu_sample, args.cpu_seconds)
        out["cpu_baseline"] = {"value": round(gbs, 3), "unit": "GB/s", "cores": used, "kind": "port",
                               "sample": f"first {n_s} frames of the same batch ({nb_s / 1e6:.0f} MB), "
                                         f"{reps} reps over >= {args.cpu_seconds:.0f} s, median; oracle/dk_oracle.cpp "
                                         f"(C++ restatement of the Rust path, clang -O3, 1 thread as the reference's "
                                         f"single-threaded LibOS)"}
        if not args.no_extras:
            # the same restatement on all host cores of this box's share (OpenMP packet shards), as a scaled figure
            threads = min(os.cpu_count() or 1, 16)
            gbs_mt, used_mt, _, _, _ = cpu_baseline(batch, flows, args.cpu_sample, max(args.cpu_seconds / 2, 1.0),
                                                    threads=threads)
            out["cpu_baseline_all_cores"] = {"value": round(gbs_mt, 3), "unit": "GB/s", "cores": used_mt}
    if rank == 0 and world == 1 and not args.no_extras and name == "c2_tcp1500":
        # secondary: 64 B UDP Mpkt/s (config 3) on rotating batches
        eng3 = RxEngine(Config(synth.BOB_IPV4), device=dev)
        b3 = [make_batch(eng3, "c3_udp64", 0, synth.SEED + 1000 * k)[0] for k in range(8)]
        r3 = eng3.results(b3[0].n)
        w3, k3, _ = time_kernel(eng3, b3, r3, 40, 4, stream)
        n3 = b3[0].n
        k3avg = float(np.mean(k3))
        algo3 = n3 * (64 + DESC_BYTES + RESULT_BYTES)
        out["c3_udp64"] = {"gbps": round(n3 * 64 * 40 / w3 / 1e9, 2), "mpkt_s": round(n3 * 40 / w3 / 1e6, 1),
                           "kernel_ms_avg": round(k3avg * 1e3, 4), "kernel": "dk_rx_small_kernel",
                           "algorithmic_bytes_per_launch": algo3,
                           "roofline_achieved_gbps": round(algo3 / k3avg / 1e9, 1),
                           "roofline_frac": round(algo3 / k3avg / 1e9 / HBM_PEAK_GBS, 4)}
        del b3, r3, eng3
        # host-resident path (NIC ring / socket buffer in pinned host memory): H2D frames + descriptors, kernel,
        # D2H results, pipelined on 3 streams (dk_rx_process_host). Reported beside `value`, never as `value`.
        out["host_path"] = host_path_rate(eng, batch, flows, args.host_frames)
        out["ring_path"] = ring_path_rate(eng, batch, flows, args.host_frames)
        # TX checksum fill (dk_tx_checksum) over the same batch (rewrites its checksum fields)
        out["tx_checksum"] = tx_rate(eng, batch, frame_bytes, stream)
        out["tx_checksum"]["traffic"] = load_traffic_profile(name + "_tx")
        out["tcp_rx"] = tcp_rate(stream)
        # few connections with many segments each (the wave-per-connection walk)
        out["tcp_rx_64conns"] = tcp_rate(stream, 1 << 20, 64, cpu_seconds=1.0)
    if rank == 0:
        print(json.dumps(out), flush=True)
    if dist is not None:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
