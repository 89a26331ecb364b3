"""The sharded path with the HIP library in every rank: two processes on cuda:0, each receives its byte-balanced shard
through ShardedReceiver (libdk_rx.so, accumulating counters, the out-of-place all-reduce on a side stream), the
counters summed over the ranks by torch.distributed (gloo: one GPU cannot host a 2-rank RCCL communicator, rccl.h;
RCCL itself is covered by test_counts_allreduce_one_rank and runs in bench.py --gpus N on a node). Checked against
the oracle over the whole batch: every rank's per-frame results for its shard, and the reduced counters after each
step. The second test runs bench.py --gpus 2 itself, as the driver launches it, in fresh child processes."""
import json
import os
import socket
import subprocess
import sys

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
        for step in range(3):  # node-wide counts of every step so far (both counter sets in use from step 1)
            sr.step(batch)
            sr.drain()
            fc, vc = sr.counts()
            fc = fc.cpu().numpy().view(np.uint64)
            vc = vc.cpu().numpy().view(np.uint64)
            if not np.array_equal(fc, (step + 1) * whole["flow_counts"][: len(fc)]):
                ok, msg = False, f"step {step}: reduced flow counts differ"
            if not np.array_equal(vc, (step + 1) * whole["verdict_counts"][: len(vc)]):
                ok, msg = False, f"step {step}: reduced verdict counts differ"
        for step in range(4):  # back-to-back steps: each kernel completes the previous step's deferred counters
            sr.step(batch)
        sr.drain()
        fc, vc = sr.counts()
        if not np.array_equal(fc.cpu().numpy().view(np.uint64), 7 * whole["flow_counts"][: len(fc)]):
            ok, msg = False, "7 steps: reduced flow counts differ"
        if not np.array_equal(vc.cpu().numpy().view(np.uint64), 7 * whole["verdict_counts"][: len(vc)]):
            ok, msg = False, "7 steps: reduced verdict counts differ"
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


def test_bench_two_ranks_child_processes(tmp_path):
    """bench.py --gpus 2 as the driver runs it (torch.distributed.run, one process per rank, 127.0.0.1), both ranks on
    cuda:0 with the counters reduced through gloo (--counts-via-torch-gloo-test: RCCL refuses two ranks on one
    device). IMIX shards (byte-balanced). The JSON line reports both ranks' frames; the node-wide counters after all
    warmup + timed steps equal (warmup + steps) x the oracle's counts over the whole 2-shard batch."""
    import torch

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path.insert(0, root)
    import bench
    from demikernel_amd import Config, RxEngine, ipv4, synth
    from oracle.oracle import OraclePeer

    per, steps, warmup = 1 << 16, 3, 2
    out = tmp_path / "counts.npz"
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()), os.path.join(root, "bench.py"),
           "--gpus", "2", "--steps", str(steps), "--warmup", str(warmup), "--no-extras", "--workload", "c4_imix",
           "--frames-per-gpu", str(per), "--counts-via-torch-gloo-test", "--counts-out", str(out)]
    env = dict(os.environ, MASTER_ADDR="127.0.0.1")
    p = subprocess.run(cmd, cwd=root, env=env, capture_output=True, text=True, timeout=300)
    assert p.returncode == 0, p.stderr[-3000:]
    lines = [ln for ln in p.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, p.stdout[-2000:]
    line = json.loads(lines[0])
    assert line["n_gpus"] == 2 and line["config"]["global_frames"] == 2 * per
    assert "TEST ONLY" in line["config"]["collective"] and line["value"] > 0
    # the line proves its own rank count: no RCCL communicator in the test mode (rccl_nranks null, the stand-in
    # named), both ranks' own kernel times and shards, the gather period and the collective's own time
    assert line["rccl_nranks"] is None and "TEST ONLY" in line["collective_kind"] and line["world_size"] == 2
    assert [r["rank"] for r in line["per_rank"]] == [0, 1]
    assert sum(r["frames"] for r in line["per_rank"]) == 2 * per
    assert all(r["kernel_ms_per_step"] > 0 and r["wall_ms_per_step"] > 0 for r in line["per_rank"])
    assert line["kernel_ms_per_step_max"] >= line["kernel_ms_per_step_min"] > 0
    assert line["gather_every"] == 8 and line["collective_ms_avg"] > 0
    got = np.load(out, allow_pickle=False)
    assert int(got["steps"]) == steps + warmup
    fc = np.zeros(0, np.uint64)
    vc = np.zeros(0, np.uint64)
    frames = 0
    for rank in range(2):  # each rank's shard, rebuilt the way the bench builds it
        eng = RxEngine(Config(synth.BOB_IPV4), device=0)
        batch, flows, _ = bench.make_batch(eng, "c4_imix", rank, synth.SEED, 2, per)
        torch.cuda.synchronize()
        ref = OraclePeer(ipv4(synth.BOB_IPV4))
        ref.set_flows(flows)
        exp = ref.process_par(batch.blob.cpu().numpy(), batch.off.cpu().numpy().view(np.uint32),
                              batch.len.cpu().numpy().view(np.uint16))
        fc = exp["flow_counts"] if rank == 0 else fc + exp["flow_counts"]
        vc = exp["verdict_counts"] if rank == 0 else vc + exp["verdict_counts"]
        frames += batch.n
        eng.close()
    assert frames == 2 * per
    assert np.array_equal(got["flow_counts"], (steps + warmup) * fc[: len(got["flow_counts"])])
    assert np.array_equal(got["verdict_counts"], (steps + warmup) * vc)
