"""The N > 1 path on CPU: byte-balanced packet shards + one all-reduce of the per-flow/per-verdict counters (gloo,
world_size 2, 127.0.0.1). On the GPU box the same code runs one rank per GPU with the nccl (RCCL) backend."""
import os
import socket

import numpy as np
import pytest

from demikernel_amd import ipv4, synth
from demikernel_amd.shard import byte_balanced_shards


def test_byte_balanced_shards_properties():
    rng = np.random.default_rng(0)
    for world in (1, 2, 3, 8):
        for lens in (rng.integers(60, 1515, 10000), synth.imix_ip_lengths(5000) + 14, np.full(7, 100), np.zeros(0)):
            sh = byte_balanced_shards(lens, world)
            assert len(sh) == world and sh[0][0] == 0 and sh[-1][1] == len(lens)
            assert all(a <= b for a, b in sh) and all(sh[k][1] == sh[k + 1][0] for k in range(world - 1))
            if len(lens) >= 100 * world:
                tot = lens.sum()
                per = [lens[a:b].sum() for a, b in sh]
                assert max(per) - min(per) <= 2 * lens.max(), (world, per)
                assert abs(max(per) - tot / world) <= lens.max()


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, out_path):
    import torch
    import torch.distributed as dist

    from demikernel_amd.shard import allreduce_counts, broadcast_comm_id
    from oracle.oracle import OraclePeer

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    # the RCCL bootstrap id travels the way bench.py hands it out (rank 0 makes it; a stand-in id here: no GPU)
    uid = broadcast_comm_id(dist, lambda: bytes(range(128)))
    assert uid == bytes(range(128))
    flows = np.concatenate([synth.make_flows(200), synth.make_flows(20, kind="udp")])
    n = 6000
    tr = synth.traffic(n, synth.imix_ip_lengths(n), flows, seed=3)
    blob, off, lens = synth.build_numpy(tr)
    synth.corrupt_numpy(blob, off, synth.corruption_plan(n, 0.03, tr))
    a, b = byte_balanced_shards(lens.astype(np.int64), world)[rank]
    p = OraclePeer(ipv4(synth.BOB_IPV4))
    p.set_flows(flows)
    r = p.process(blob, off[a:b], lens[a:b])
    fc = torch.from_numpy(r["flow_counts"].view(np.int64).copy())
    vc = torch.from_numpy(r["verdict_counts"].view(np.int64).copy())
    allreduce_counts(fc)
    allreduce_counts(vc)
    if rank == 0:
        whole = p.process(blob, off, lens)
        np.savez(out_path, fc=fc.numpy(), vc=vc.numpy(), fc_exp=whole["flow_counts"].view(np.int64),
                 vc_exp=whole["verdict_counts"].view(np.int64))
    dist.barrier()
    dist.destroy_process_group()


def test_two_rank_gloo_counts_equal_single_rank(tmp_path):
    import torch.multiprocessing as mp

    out = str(tmp_path / "counts.npz")
    mp.spawn(_worker, args=(2, _free_port(), out), nprocs=2, join=True)
    d = np.load(out)
    assert np.array_equal(d["fc"], d["fc_exp"]) and np.array_equal(d["vc"], d["vc_exp"])
    assert d["vc"].sum() == 6000
