"""BASELINE configs 4 and 5 at their stated node-wide size — 16M frames over 8 GPUs — on one GPU.

One 16M-frame traffic stream is cut into the 8 byte-balanced contiguous shards `shard.byte_balanced_shards` gives the
8 ranks of `bench.py --gpus 8`; each shard is built on the device and received as its rank would receive it (the
24-byte record the bench times, deferred counters completed by a flush), one after another on this GPU, and checked
bit for bit against the oracle on every frame. The node-wide counters are the sum over the shards — what the RCCL
all-reduce gathers (dk_rx_flow_counts_allreduce_to; RCCL itself cannot run 8 ranks on one device) — and are checked
against the whole stream: every frame has one verdict, every intact frame is delivered to its own flow.
(A 16M-frame IMIX stream is ~6.3 GB of 64-byte slots: more than one dk_rx batch can address, DK_RX_MAX_BLOB, so the
node-wide config only exists sharded.)"""
import dataclasses

import numpy as np
import pytest

from demikernel_amd import Config, RxEngine, V, VERDICTS, ipv4, synth
from demikernel_amd.shard import byte_balanced_shards
from oracle.oracle import OraclePeer
from test_gpu_parity import assert_same

pytestmark = pytest.mark.gpu

NODE_FRAMES, RANKS = 1 << 24, 8


def shard_traffic(tr, b, e):
    return synth.Traffic(**{f.name: getattr(tr, f.name)[b:e] for f in dataclasses.fields(tr)})


def node_wide(ip_len, flows, seed):
    import torch

    assert torch.cuda.is_available()
    tr = synth.traffic(NODE_FRAMES, ip_len, flows, seed=seed)
    flen = tr.frame_len.astype(np.int64)
    shards = byte_balanced_shards(flen, RANKS)
    assert shards[0][0] == 0 and shards[-1][1] == NODE_FRAMES and all(
        shards[k][1] == shards[k + 1][0] for k in range(RANKS - 1))
    per_rank = [int(flen[b:e].sum()) for b, e in shards]
    assert max(per_rank) - min(per_rank) <= 2 * int(flen.max()), per_rank  # balanced to a frame's bytes
    eng = RxEngine(Config(synth.BOB_IPV4))
    eng.set_sockets(flows)
    ref = OraclePeer(ipv4(synth.BOB_IPV4))
    ref.set_flows(flows)
    node_flow = np.zeros(len(flows), np.uint64)
    node_verdict = np.zeros(len(VERDICTS), np.uint64)
    delivered_flows = np.zeros(len(flows), np.uint64)
    intact_ok = 0
    for r, (b, e) in enumerate(shards):
        t = shard_traffic(tr, b, e)
        plan = synth.corruption_plan(t.n, 0.01, t, seed + r)
        batch = synth.build_device(t, eng, seed=seed + r)
        off = np.asarray(batch.off.cpu().numpy().view(np.uint32))
        lens = np.asarray(batch.len.cpu().numpy().view(np.uint16))
        synth.corrupt_device(batch, off, plan)
        res = eng.results(t.n)
        eng.receive_batch(batch, res, defer_counts=True)
        eng.flush_counts()
        torch.cuda.synchronize()
        got = res.to_numpy()
        exp = ref.process_par(batch.blob.cpu().numpy(), off, lens)
        assert_same(got, exp, f"rank {r} of {RANKS}, frames [{b}, {e})")
        v = got["meta"] & 0xFF
        bad = np.zeros(t.n, bool)
        bad[np.array(sorted({i for i, _, _ in plan}), np.int64)] = True
        assert np.array_equal(got["flow_id"][~bad], t.flow[~bad].astype(np.uint32))
        intact_ok += int((v[~bad] <= 1).sum())
        deliv = v <= 1
        delivered_flows += np.bincount(got["flow_id"][deliv], minlength=len(flows)).astype(np.uint64)
        node_flow += got["flow_counts"]
        node_verdict += got["verdict_counts"]
        print(f"rank {r}: frames [{b}, {e}), {per_rank[r]} B, bit-exact", flush=True)
        del batch, res
    assert int(node_verdict.sum()) == NODE_FRAMES
    assert np.array_equal(node_flow, delivered_flows)
    assert int(node_verdict[V["OK_TCP"]] + node_verdict[V["OK_UDP"]]) == int(node_flow.sum()) >= intact_ok
    assert intact_ok > 0.98 * NODE_FRAMES
    eng.close()
    return node_flow


def test_c4_imix_node_wide_16m_frames(torch_cuda_node):
    """C4: 16M IMIX frames (40/576/1500 B at 7:4:1) over 1,024 flows, 1 % corrupted per shard, as 8 ranks' shards."""
    node_wide(synth.imix_ip_lengths(NODE_FRAMES, seed=9), synth.make_flows(1024), seed=9)


def test_c5_node_wide_16m_frames_10k_flows(torch_cuda_node):
    """C5: 16M x 1500 B TCP frames over 10,000 Active flows, 1 % corrupted per shard, as 8 ranks' shards; every flow
    receives frames node-wide."""
    counts = node_wide(1486, synth.make_flows(10000), seed=10)
    assert (counts[:10000] > 0).all()


@pytest.fixture(scope="module")
def torch_cuda_node():
    import torch

    assert torch.cuda.is_available()
    return torch
