"""bench.py's multi-GPU line fields on the CPU (no GPU): the scaling evidence the driver's SCALE run carries —
the RCCL communicator's own rank count (dk_comm_count), each rank's kernel time and shard, the gather period and
the collective's time — built by bench.scale_fields from what every rank reports."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import bench  # noqa: E402


class FakeRccl:
    """Stands in for demikernel_amd.Comm: count() is dk_comm_count on the communicator."""

    def __init__(self, n):
        self.n = n

    def count(self):
        return self.n


class FakeTorchStandIn:  # shard.TorchCountsAllreduce has no count(): not the product collective
    pass


def rows(world):
    return [{"rank": r, "kernel_ms_per_step": 0.14 + 0.001 * r, "wall_ms_per_step": 0.15, "frames": 1000 + r,
             "frame_bytes": 10 ** 6, "gpu": {"device_index": r, "name": "gpu"}} for r in reversed(range(world))]


def test_rccl_line_proves_rank_count():
    f = bench.scale_fields(8, FakeRccl(8), rows(8), [0.008, 0.009], 8)
    assert f["rccl_nranks"] == 8 and f["world_size"] == 8 and f["collective_kind"].startswith("rccl")
    assert [r["rank"] for r in f["per_rank"]] == list(range(8))  # sorted by rank whatever the gather order
    assert f["gather_every"] == 8 and abs(f["collective_ms_avg"] - 8.5) < 1e-9
    assert f["kernel_ms_per_step_max"] == 0.147 and f["kernel_ms_per_step_min"] == 0.14


def test_test_mode_line_names_the_stand_in():
    f = bench.scale_fields(2, FakeTorchStandIn(), rows(2), [0.001], 8)
    assert f["rccl_nranks"] is None and "TEST ONLY" in f["collective_kind"]
    assert len(f["per_rank"]) == 2


def test_single_gpu_line():
    f = bench.scale_fields(1, None, rows(1), [], 8)
    assert f["rccl_nranks"] is None and f["collective_kind"] == "none" and f["gather_every"] is None
    assert f["collective_ms_avg"] is None and len(f["per_rank"]) == 1


def test_missized_communicator_is_refused():
    """an RCCL communicator that does not hold every rank exits non-zero (status 4), never a line."""
    import pytest

    for nranks, world in ((1, 8), (4, 8), (8, 4)):
        with pytest.raises(SystemExit) as e:
            bench.scale_fields(world, FakeRccl(nranks), rows(world), [0.008], 8)
        assert e.value.code == 4
    bench.check_comm_size(2, 2)  # the right size passes
