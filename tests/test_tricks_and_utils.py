"""DeepSpeed trick (duck-typed fake engine), RSS profiler, knobs, NUMA helpers,
equality helpers, UVM adapter."""

import os

import torch

from hipsnapshot import knobs
from hipsnapshot.tricks.deepspeed import Zero3StateAdapter, patch_engine_to_use_hipsnapshot
from hipsnapshot.utils.rss_profiler import measure_rss_deltas


class _FakeZero3:
    def __init__(self):
        self.state = {"fp32_flat": torch.randn(1000), "step": 3}
        self.persistent_parameters = []
        self.loaded = None

    def state_dict(self):
        return self.state

    def load_state_dict(self, state_dict):
        self.state = state_dict

    def _rigid_load_state_dict(self, state_dict, load_optimizer_states=True):
        self.loaded = state_dict


_FakeZero3.__name__ = "DeepSpeedZeroOptimizer_Stage3"


class _FakeEngine:
    def __init__(self):
        self.optimizer = _FakeZero3()
        self.config = {"zero_optimization": {"stage": 3}}
        self.global_rank = 0
        self.copied = None

    def _copy_recovery_script(self, path):
        self.copied = path

    def zero_load_from_fp32_weights(self):
        return False


def test_deepspeed_trick_roundtrip(tmp_path):
    eng = _FakeEngine()
    patch_engine_to_use_hipsnapshot(eng)
    eng._save_zero_checkpoint(str(tmp_path / "z"), "tag")
    assert eng.copied == str(tmp_path / "z")
    eng2 = _FakeEngine()
    eng2._hipsnapshot_pending = eng._hipsnapshot_pending
    patch_engine_to_use_hipsnapshot(eng2)
    assert eng2._load_zero_checkpoint(str(tmp_path / "z"), "tag")
    assert torch.equal(eng2.optimizer.loaded["fp32_flat"], eng.optimizer.state["fp32_flat"])
    assert eng2.optimizer.loaded["step"] == 3


def test_deepspeed_trick_rejects_non_zero3():
    eng = _FakeEngine()
    eng.optimizer = object()
    import pytest

    with pytest.raises(RuntimeError):
        patch_engine_to_use_hipsnapshot(eng)
    assert isinstance(Zero3StateAdapter(_FakeZero3()).state_dict(), dict)


def test_rss_profiler():
    deltas = []
    with measure_rss_deltas(deltas, interval_s=0.01):
        x = torch.ones(50_000_000)  # 200 MB
        x.add_(1)
    assert max(deltas) > 100 * 2 ** 20


def test_knob_overrides_and_legacy_names(monkeypatch):
    assert knobs.get_max_chunk_size_bytes() == 512 * 1024 * 1024
    with knobs.override_max_chunk_size_bytes(123):
        assert knobs.get_max_chunk_size_bytes() == 123
    assert knobs.get_max_chunk_size_bytes() == 512 * 1024 * 1024
    monkeypatch.setenv("TORCHSNAPSHOT_SLAB_SIZE_THRESHOLD_BYTES_OVERRIDE", "77")
    assert knobs.get_slab_size_threshold_bytes() == 77
    with knobs.override_slab_size_threshold_bytes(5):
        assert knobs.get_slab_size_threshold_bytes() == 5
        assert knobs.get_max_shard_size_bytes() == 512 * 1024 * 1024
    monkeypatch.setenv("TORCHSNAPSHOT_DISABLE_BATCHING", "1")
    assert knobs.is_batching_disabled()


def test_timeline_trace(tmp_path, monkeypatch):
    import json

    from hipsnapshot import Snapshot, StateDict
    from hipsnapshot.utils import tracing

    tl = tracing.Timeline()
    tl.prefix = str(tmp_path / "tl")
    monkeypatch.setattr(tracing, "timeline", tl)
    import hipsnapshot.engine.scheduler as sched
    import hipsnapshot.snapshot as snap_mod

    monkeypatch.setattr(sched, "timeline", tl)
    monkeypatch.setattr(snap_mod, "timeline", tl)
    sd = StateDict(a=torch.randn(1000), b=torch.randn(50, 50), n=3)
    Snapshot.take(str(tmp_path / "s"), {"sd": sd})
    Snapshot(str(tmp_path / "s")).restore({"sd": sd})
    take = json.load(open(tmp_path / "tl.rank0.take0.json"))["traceEvents"]
    names = {e["name"] for e in take}
    assert {"coalesce", "prepare_write", "stage", "drain_io", "commit", "write"} <= names
    assert all(e["ph"] == "X" and e["dur"] >= 0 for e in take)
    assert sum(e["args"].get("bytes", 0) for e in take if e["name"] == "write") > 0
    rest = json.load(open(tmp_path / "tl.rank0.restore0.json"))["traceEvents"]
    assert {"load_stateful", "read"} <= {e["name"] for e in rest}


def test_numa_affinity_helpers(monkeypatch):
    from hipsnapshot.utils import affinity

    assert affinity._parse_cpulist("0-3,8,10-11\n") == {0, 1, 2, 3, 8, 10, 11}
    assert affinity._parse_cpulist("") == set()
    # unknown topology (no GPU here): nothing is bound, the reason is reported
    monkeypatch.setattr(affinity, "gpu_numa_node", lambda d: None)
    rep = affinity.bind_to_gpu_numa(0)
    assert rep["bound"] is False and "unknown" in rep["reason"]
    # too few usable CPUs on the GPU's node -> no binding
    monkeypatch.setattr(affinity, "gpu_numa_node", lambda d: 7)
    monkeypatch.setattr(affinity, "node_cpus", lambda n: set())
    rep = affinity.bind_to_gpu_numa(0)
    assert rep["bound"] is False and rep["local"] == 0
    # node covering every allowed CPU -> already local, affinity untouched
    import os

    allowed = os.sched_getaffinity(0)
    monkeypatch.setattr(affinity, "node_cpus", lambda n: set(allowed) | {10 ** 6})
    rep = affinity.bind_to_gpu_numa(0, min_cpus=1)
    assert rep["bound"] is False and rep["reason"] == "already local"
    assert os.sched_getaffinity(0) == allowed


def test_equality_helpers():
    # reference: tests/test_test_utils.py (tensor / sharded-tensor equality
    # used by every round-trip test)
    import pytest as _pytest
    import torch.distributed as dist

    from hipsnapshot.utils.test_utils import (assert_state_dict_eq, free_port,
                                              sharded_tensor_eq, tensor_eq)

    a = torch.arange(6.0).view(2, 3)
    assert tensor_eq(a, a.clone()) and not tensor_eq(a, a + 1)
    assert not tensor_eq(a, a.double()) and not tensor_eq(a, a.view(3, 2))
    q = torch.quantize_per_tensor(a, 0.5, 2, torch.qint8)
    assert tensor_eq(q, q.clone()) and not tensor_eq(q, a)
    assert not tensor_eq(q, torch.quantize_per_tensor(a, 0.25, 2, torch.qint8))
    f8 = a.to(torch.float8_e4m3fn)
    assert tensor_eq(f8, f8.clone())
    assert_state_dict_eq({"x": [a, 1, "s"], "y": {"z": a}}, {"x": [a.clone(), 1, "s"], "y": {"z": a}})
    with _pytest.raises(AssertionError):
        assert_state_dict_eq({"x": a}, {"x": a + 1})
    with _pytest.raises(AssertionError):
        assert_state_dict_eq({"x": a, "y": 1}, {"y": 1, "x": a})  # key order is part of equality
    with _pytest.raises(AssertionError):
        assert_state_dict_eq([1, 2], (1, 2))

    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    own_pg = not dist.is_initialized()
    if own_pg:
        dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{free_port()}", rank=0,
                                world_size=1)
    try:
        from torch.distributed._shard.sharded_tensor import empty as st_empty
        from torch.distributed._shard.sharding_spec import ChunkShardingSpec

        spec = ChunkShardingSpec(dim=0, placements=["rank:0/cpu", "rank:0/cpu"])
        s1, s2, s3 = (st_empty(spec, 4, 3) for _ in range(3))
        for s, v in ((s1, 1.0), (s2, 1.0), (s3, 2.0)):
            for sh in s.local_shards():
                sh.tensor.fill_(v)
        assert sharded_tensor_eq(s1, s2) and tensor_eq(s1, s2)
        assert not sharded_tensor_eq(s1, s3) and not sharded_tensor_eq(s1, a)
        other = st_empty(ChunkShardingSpec(dim=1, placements=["rank:0/cpu", "rank:0/cpu"]), 4, 3)
        for sh in other.local_shards():
            sh.tensor.fill_(1.0)
        assert not sharded_tensor_eq(s1, other)  # same values, different shard layout
    finally:
        if own_pg:
            dist.destroy_process_group()


def test_uvm_adapter_without_managed_memory():
    # reference: tests/test_uvm_tensor.py -- the adapter must be importable
    # and inert for ordinary tensors (managed allocation itself: test_gpu.py)
    from hipsnapshot.ops.uvm import is_uvm_tensor, uvm_to_cpu

    t = torch.randn(5, 3)
    assert not is_uvm_tensor(t)
    assert torch.equal(uvm_to_cpu(t), t)
    assert not is_uvm_tensor(t.t())


def test_state_dict_view_skips_dtensor_detach():
    # take() reads FSDP2 DTensor parameters as they are (no per-parameter
    # DTensor detach), detaches plain grad-requiring tensors, and leaves
    # classes with their own state_dict() alone
    import torch.distributed as dist
    import torch.nn as nn
    from torch.distributed.device_mesh import init_device_mesh
    from torch.distributed.tensor import DTensor

    from hipsnapshot.models.llama import LlamaConfig, build_fsdp_llama
    from hipsnapshot.snapshot import _state_dict_view
    from hipsnapshot.utils.test_utils import free_port

    lin = nn.Linear(4, 3)
    sd = _state_dict_view(lin)
    assert list(sd) == ["weight", "bias"] and not sd["weight"].requires_grad
    assert sd["weight"].data_ptr() == lin.weight.data_ptr()

    class Custom(nn.Module):
        def __init__(self):
            super().__init__()
            self.p = nn.Parameter(torch.ones(2))

        def state_dict(self, *a, **k):
            return {"custom": 1}

    assert _state_dict_view(Custom()) == {"custom": 1}

    own_pg = not dist.is_initialized()
    if own_pg:
        dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{free_port()}", rank=0,
                                world_size=1)
    try:
        m = build_fsdp_llama(LlamaConfig.tiny(), torch.device("cpu"), torch.float32,
                             mesh=init_device_mesh("cpu", (1,)))
        sd = _state_dict_view(m)
        ref = m.state_dict()
        assert list(sd) == list(ref)
        params = dict(m.named_parameters())
        for k, v in sd.items():
            assert isinstance(v, DTensor) and v is params[k]  # the parameter itself
            assert not v._local_tensor.requires_grad
            assert torch.equal(v._local_tensor, ref[k]._local_tensor)
        # restore fills the parameters' local tensors in place through the same view
        import tempfile

        from hipsnapshot import Snapshot

        with tempfile.TemporaryDirectory() as d:
            Snapshot.take(d, {"m": m})
            want = {k: v._local_tensor.clone() for k, v in sd.items()}
            with torch.no_grad():
                for p in m.parameters():
                    p.zero_()
            Snapshot(d).restore({"m": m})
            for k, p in m.named_parameters():
                assert torch.equal(p._local_tensor, want[k]), k
                assert p.requires_grad and not p._local_tensor.requires_grad
    finally:
        if own_pg:
            dist.destroy_process_group()


def test_worker_pools_are_reused_only_when_clean():
    from hipsnapshot.engine import scheduler
    from hipsnapshot.ops import native

    a = scheduler._acquire_pool("t", 2, 0)
    a.submit(lambda: None).result()
    scheduler._release_pool(a, reusable=True)
    b = scheduler._acquire_pool("t", 2, 0)
    assert b is a  # an idle pool comes back
    scheduler._release_pool(b, reusable=False)  # shut down, not pooled
    c = scheduler._acquire_pool("t", 2, 0)
    assert c is not a
    scheduler._release_pool(c, reusable=True)

    e1 = native.acquire_io_engine(2)
    native.release_io_engine(e1, reusable=True)
    e2 = native.acquire_io_engine(2)
    assert e2 is e1
    native.release_io_engine(e2, reusable=False)  # jobs in flight: closed
    assert e2.handle is None
    e3 = native.acquire_io_engine(2)
    assert e3 is not e1 and e3.handle
    native.release_io_engine(e3, reusable=True)


def test_plan_scope_caches_per_device_and_restores():
    from hipsnapshot.engine import staging

    assert staging.producer_stream_handle(torch.zeros(2)) is None  # host tensor
    with staging.plan_scope():
        assert staging._plan.streams == {}
        with staging.plan_scope():  # nested scopes restore the outer cache
            staging._plan.streams[0] = 123
        assert staging._plan.streams == {}
    assert getattr(staging._plan, "streams", None) is None


def test_drain_threads_avoid_the_callers_core():
    """Threads created under threads_avoiding_caller inherit a mask without
    the noted caller's core; the creating thread's mask is restored."""
    import os
    import threading

    from hipsnapshot.utils import affinity

    cpu = affinity.current_cpu()
    assert cpu is not None and cpu in affinity.core_siblings(cpu)
    before = os.sched_getaffinity(0)
    affinity.note_caller_cpu()
    seen = {}
    with affinity.threads_avoiding_caller():
        t = threading.Thread(target=lambda: seen.setdefault("mask", os.sched_getaffinity(0)))
        t.start()
        t.join()
    assert os.sched_getaffinity(0) == before
    expect = affinity.mask_avoiding_caller()
    if expect is None:  # too few CPUs here: nothing is restricted
        assert seen["mask"] == before
    else:
        assert seen["mask"] == expect
        assert not (seen["mask"] & affinity.core_siblings(affinity._caller_cpu[0]))
    with affinity.threads_avoiding_caller(enabled=False):
        assert os.sched_getaffinity(0) == before
    # "l3": the caller's whole L3 domain is excluded when enough CPUs remain
    cpu = affinity._caller_cpu[0]
    assert cpu in affinity.l3_siblings(cpu)
    m = affinity.mask_avoiding_caller("l3")
    if m is not None:
        assert not (m & affinity.core_siblings(cpu))
        if len(before - affinity.l3_siblings(cpu)) >= 2:
            assert not (m & affinity.l3_siblings(cpu))
    assert affinity.mask_avoiding_caller("") is None


def test_drain_avoid_knob_modes(monkeypatch):
    from hipsnapshot import knobs

    assert knobs.drain_avoid_caller_core() == "core"  # default
    for v, want in (("1", "core"), ("core", "core"), ("l3", "l3"), ("0", ""), ("off", "")):
        with knobs.override_knob("DRAIN_AVOID_CALLER_CORE", v):
            assert knobs.drain_avoid_caller_core() == want
    assert knobs.drain_avoid_caller_core() == "core"
