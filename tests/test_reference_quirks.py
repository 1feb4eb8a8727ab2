"""Regression tests for the reference quirks listed in SURVEY.md Appendix C.

Each test pins the CORRECT behaviour where the reference
(`/root/reference/torchsnapshot`) has a bug, so it cannot creep back in.
"""

from datetime import timedelta

import pytest
import torch

from hipsnapshot import Snapshot, StateDict
from hipsnapshot import knobs
from hipsnapshot.utils.test_utils import run_distributed


def test_c1_async_take_does_not_alias_live_host_tensors(tmp_path):
    """#1: reference `io_preparers/tensor.py:282,293` compared a str with an
    enum, so large/unbatched CPU tensors were written from a live memoryview."""
    big = torch.arange(4_000_000, dtype=torch.float32)  # 16 MB, not batched below
    ref = big.clone()
    with knobs.override_is_batching_disabled(True):
        pending = Snapshot.async_take(str(tmp_path / "s"), {"sd": StateDict(t=big)})
        big.fill_(-1.0)  # mutate right after return
        snap = pending.wait()
    assert torch.equal(snap.read_object("0/sd/t"), ref)


def test_c2_prepare_func_output_is_staged(tmp_path):
    """#2: the hook's output (not the original tensor) is what gets written."""
    t = torch.randn(64, 64)

    def halve(path, x, tracing):
        return (x / 2).to(torch.float16)

    Snapshot.take(str(tmp_path / "s"), {"sd": StateDict(t=t)},
                  _custom_tensor_prepare_func=halve)
    got = Snapshot(str(tmp_path / "s")).read_object("0/sd/t")
    assert got.dtype == torch.float16 and torch.equal(got, (t / 2).to(torch.float16))


def test_c3_merged_read_cost_counts_whole_span():
    """#3: reference used the last member's range for the merged buffer size."""
    from hipsnapshot.io.batcher import batch_read_requests
    from hipsnapshot.io_types import ReadReq

    class C:
        def __init__(self, n):
            self.n = n

        async def consume_buffer(self, buf, executor=None):
            pass

        def get_consuming_cost_bytes(self):
            return self.n

        def get_read_dest(self, nbytes):
            return None

    reqs = [ReadReq(path="batched/x", byte_range=(0, 100), buffer_consumer=C(100)),
            ReadReq(path="batched/x", byte_range=(4096, 4106), buffer_consumer=C(10))]
    (merged,) = batch_read_requests(reqs)
    assert merged.byte_range == (0, 4106)
    assert merged.buffer_consumer.buf_sz_bytes == 4106
    assert merged.buffer_consumer.get_consuming_cost_bytes() >= 4106


def test_c4_slab_override_touches_slab_knob_only():
    """#4: reference's override_slab_size_threshold_bytes set the SHARD knob."""
    shard = knobs.get_max_shard_size_bytes()
    with knobs.override_slab_size_threshold_bytes(12345):
        assert knobs.get_slab_size_threshold_bytes() == 12345
        assert knobs.get_max_shard_size_bytes() == shard


def test_c5_linear_barrier_depart_marks_departed():
    """#5: reference's depart() set ``arrived`` again."""
    from hipsnapshot.parallel.store import LinearBarrier

    store = torch.distributed.HashStore()
    b = LinearBarrier("c5", store, rank=0, world_size=1, leader_rank=0)
    b.arrive(timeout=timedelta(seconds=5))
    b.depart(timeout=timedelta(seconds=5))
    assert b.arrived and b.departed
    with pytest.raises(RuntimeError):
        b.arrive(timeout=timedelta(seconds=1))


@pytest.mark.parametrize("scheme", ["tensor", "channel"])
def test_c6_qtensor_codecs_check_the_qscheme_value(scheme):
    """#6: reference compared the bound method ``t.qscheme`` with a qscheme."""
    from hipsnapshot.format import serialization as ser

    x = torch.randn(8, 5)
    if scheme == "tensor":
        q = torch.quantize_per_tensor(x, 0.05, 3, torch.qint8)
        back = ser.per_tensor_qtensor_from_bytes(ser.per_tensor_qtensor_as_bytes(q))
        with pytest.raises(ValueError):
            ser.per_channel_qtensor_as_bytes(q)
    else:
        q = torch.quantize_per_channel(x, torch.rand(5) + 0.01, torch.zeros(5, dtype=torch.long),
                                       1, torch.quint8)
        back = ser.per_channel_qtensor_from_bytes(ser.per_channel_qtensor_as_bytes(q))
        with pytest.raises(ValueError):
            ser.per_tensor_qtensor_as_bytes(q)
    assert torch.equal(back.int_repr(), q.int_repr())
    assert torch.equal(back.dequantize(), q.dequantize())


def test_c8_objects_load_weights_only_by_default(tmp_path):
    """#8: arbitrary pickles are refused (not executed) unless trusted."""
    from hipsnapshot.io.object import UntrustedObjectError
    from hipsnapshot.format.serialization import torch_save_as_bytes

    class Custom:
        pass

    blob = torch_save_as_bytes({"ok": torch.ones(2)})
    assert blob  # plain containers of tensors round-trip weights-only
    Snapshot.take(str(tmp_path / "s"), {"sd": StateDict(obj=(1, torch.ones(3)))})
    got = Snapshot(str(tmp_path / "s")).read_object("0/sd/obj")
    assert got[0] == 1 and torch.equal(got[1], torch.ones(3))
    assert issubclass(UntrustedObjectError, Exception) and Custom


def test_c9_restore_computes_budget_and_manifest_once(tmp_path, monkeypatch):
    """#9: one hostname all-gather / manifest split per restore, not per stateful."""
    import hipsnapshot.engine.scheduler as sched
    import hipsnapshot.parallel.elasticity as el

    app = {f"s{i}": StateDict(t=torch.full((10,), float(i))) for i in range(5)}
    Snapshot.take(str(tmp_path / "s"), app)
    calls = {"ws": 0, "split": 0}
    orig_ws = sched.get_local_world_size
    orig_split = el._split_manifest if hasattr(el, "_split_manifest") else None

    def spy_ws(pg):
        calls["ws"] += 1
        return orig_ws(pg)

    monkeypatch.setattr(sched, "get_local_world_size", spy_ws)
    sched._budget_cache.clear()
    out = {f"s{i}": StateDict(t=torch.zeros(10)) for i in range(5)}
    snap = Snapshot(str(tmp_path / "s"))
    snap.restore(out)
    assert calls["ws"] <= 1
    for i in range(5):
        assert torch.equal(out[f"s{i}"]["t"], torch.full((10,), float(i)))
    del orig_split


def _disable_partitioner_worker(path: str) -> None:
    import os

    import torch.distributed as dist

    os.environ["TORCH_SNAPSHOT_DISABLE_PARTITIONER"] = "1"
    sd = StateDict(w=torch.arange(1000.0), mine=torch.full((3,), float(dist.get_rank())))
    Snapshot.take(path, {"sd": sd}, replicated=["sd/w"])
    out = StateDict(w=torch.zeros(1000), mine=torch.zeros(3))
    Snapshot(path).restore({"sd": out})
    assert torch.equal(out["w"], torch.arange(1000.0))
    assert torch.equal(out["mine"], torch.full((3,), float(dist.get_rank())))


def test_c10_disable_partitioner_is_supported(tmp_path):
    """#10: the reference declared the knob but raised NotImplementedError."""
    run_distributed(_disable_partitioner_worker, 2, str(tmp_path / "p"))
