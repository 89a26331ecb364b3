"""The sharded path with the HIP library in every rank: two processes on cuda:0, each receives its byte-balanced shard
through ShardedReceiver (libdk_rx.so, per-step counters on the launch stream, the all-reduce on a side stream), the
counters summed over the ranks by torch.distributed (gloo: one GPU cannot host a 2-rank RCCL communicator; RCCL
itself is covered by test_counts_allreduce_one_rank and runs in bench.py --gpus N). Checked against the oracle over
the whole batch: every rank's per-frame results for its shard, and the reduced counters after each step."""
import json
import os
import socket

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, out_dir):
    import torch
    import torch.distributed as dist

    from demikernel_amd import Config, FrameBatch, RxEngine, ipv4, synth
    from demikernel_amd.shard import ShardedReceiver, TorchCountsAllreduce, byte_balanced_shards
    from oracle.oracle import OraclePeer

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    flows = np.concatenate([synth.make_flows(300), synth.make_flows(40, kind="udp")])
    n = 8000
    tr = synth.traffic(n, synth.imix_ip_lengths(n, seed=12), flows, seed=12)
    blob, off, lens = synth.build_numpy(tr)
    synth.corrupt_numpy(blob, off, synth.corruption_plan(n, 0.03, tr))
    a, b = byte_balanced_shards(lens.astype(np.int64), world)[rank]
    ok, msg = True, ""
    try:
        torch.cuda.set_device(0)
        eng = RxEngine(Config(synth.BOB_IPV4), device=0)
        eng.set_sockets(flows)
        batch = FrameBatch.from_numpy(blob, off[a:b], lens[a:b], device=0)
        res = eng.results(b - a)
        stream = torch.cuda.current_stream(0)
        sr = ShardedReceiver(eng, res, TorchCountsAllreduce(dist.group.WORLD), stream)
        ref = OraclePeer(ipv4(synth.BOB_IPV4))
        ref.set_flows(flows)
        whole = ref.process(blob, off, lens)
        mine = ref.process(blob, off[a:b], lens[a:b])
        for step in range(2):
            sr.step(batch)
            sr.drain()
            fc, vc = sr.counts()
            fc = fc.cpu().numpy().view(np.uint64)
            vc = vc.cpu().numpy().view(np.uint64)
            if not np.array_equal(fc, whole["flow_counts"][: len(fc)]):
                ok, msg = False, f"step {step}: reduced flow counts differ"
            if not np.array_equal(vc, whole["verdict_counts"][: len(vc)]):
                ok, msg = False, f"step {step}: reduced verdict counts differ"
        got = res.to_numpy()
        for k in ("meta", "src_ip", "ports", "payload", "flow_id"):
            if not np.array_equal(got[k], mine[k]):
                ok, msg = False, f"rank {rank}: '{k}' differs from the oracle on its shard"
    except Exception as e:  # noqa: BLE001 - reported through the result file
        ok, msg = False, f"rank {rank}: {type(e).__name__}: {e}"
    with open(os.path.join(out_dir, f"rank{rank}.json"), "w") as fh:
        json.dump({"ok": ok, "msg": msg, "frames": int(b - a)}, fh)
    dist.barrier()
    dist.destroy_process_group()


def test_two_ranks_sharded_receiver_on_gpu(tmp_path):
    import torch.multiprocessing as mp

    mp.spawn(_worker, args=(2, _free_port(), str(tmp_path)), nprocs=2, join=True)
    shard = 0
    for r in range(2):
        d = json.loads((tmp_path / f"rank{r}.json").read_text())
        assert d["ok"], d["msg"]
        assert d["frames"] > 0
        shard += d["frames"]
    assert shard == 8000
