"""Async takes of host-resident UVM tables (engine/uvm_capture.py): CPU
capture on the pages' NUMA node while the trainer's stream waits on a gate
(csrc/hsgpu.hip hsg_gate_*)."""

import time

import pytest
import torch

from hipsnapshot import Snapshot, StateDict, memory_held
from hipsnapshot.ops import native

pytestmark = pytest.mark.gpu


def test_gate_holds_the_stream_until_released(gpu):
    if not native.gate_supported(0):
        pytest.skip("no hipStreamWaitValue32 on this device")
    s = torch.cuda.Stream(device=gpu)
    x = torch.zeros(1024, device=gpu)
    torch.cuda.synchronize()
    v = native.gate_arm(0, int(s.cuda_stream))
    try:
        with torch.cuda.stream(s):
            x.add_(1)
            ev = torch.cuda.Event()
            ev.record(s)
        time.sleep(0.1)
        assert not ev.query()  # held at the gate
    finally:
        native.gate_release(0, v)
    ev.synchronize()
    assert torch.all(x == 1)
    # an older value never lowers the word (a late release cannot re-block)
    native.gate_release(0, v - 1)
    assert native.gate_value(0) >= v


def _tables(gpu, n=4, rows=1 << 20, dim=64):
    from hipsnapshot.ops import uvm

    ts = []
    g = torch.Generator(device=gpu).manual_seed(5)
    for _ in range(n):
        t = uvm.new_managed_tensor([rows, dim], torch.float32, gpu.index or 0)
        t.copy_(torch.randn(rows, dim, device=gpu, generator=g))
        uvm.place(t, "host")
        ts.append(t)
    torch.cuda.synchronize()
    assert all(uvm.residency(t) == "host" for t in ts)
    return ts


def test_async_take_captures_host_uvm_tables_on_the_cpu(gpu, tmp_path):
    """The tables are copied by CPU threads, not frozen into HBM; updates the
    trainer queues right after async_take returns do not reach the snapshot;
    the restore is bitwise."""
    from hipsnapshot.engine import uvm_capture

    if not native.gate_supported(0):
        pytest.skip("no hipStreamWaitValue32 on this device")
    from hipsnapshot import release_hbm_arena

    release_hbm_arena()  # an arena an earlier test kept is not this take's
    ts = _tables(gpu)
    ref = [t.clone() for t in ts]
    sd = StateDict(**{f"t{i}": t for i, t in enumerate(ts)})
    pending = Snapshot.async_take(str(tmp_path / "a"), {"sd": sd})
    for t in ts:  # the trainer's next step: queued behind the gate
        t.add_(1.0)
    pending.wait()
    torch.cuda.synchronize()
    assert uvm_capture.last.get("bytes") == sum(t.numel() * 4 for t in ts)
    assert memory_held(gpu.index or 0)["hbm_arena_bytes"] == 0  # no HBM freeze
    assert all(torch.equal(t, r + 1.0) for t, r in zip(ts, ref))
    out = StateDict(**{f"t{i}": torch.zeros_like(r) for i, r in enumerate(ref)})
    # verify=True: the checksums the capture computed while copying match
    Snapshot(str(tmp_path / "a")).restore({"sd": out}, verify=True)
    for i, r in enumerate(ref):
        assert torch.equal(out[f"t{i}"], r), i
    # a second async take reuses the plan and captures again
    pending = Snapshot.async_take(str(tmp_path / "a"), {"sd": sd})
    pending.wait()
    Snapshot(str(tmp_path / "a")).restore({"sd": out})
    for i, t in enumerate(ts):
        assert torch.equal(out[f"t{i}"], t), i


def test_capture_off_falls_back_to_the_hbm_freeze(gpu, tmp_path):
    from hipsnapshot.knobs import override_tuning

    ts = _tables(gpu, n=2, rows=1 << 18)
    ref = [t.clone() for t in ts]
    sd = StateDict(**{f"t{i}": t for i, t in enumerate(ts)})
    with override_tuning(uvm_async_capture=False):
        pending = Snapshot.async_take(str(tmp_path / "b"), {"sd": sd})
        for t in ts:
            t.add_(1.0)
        pending.wait()
    out = StateDict(**{f"t{i}": torch.zeros_like(r) for i, r in enumerate(ref)})
    Snapshot(str(tmp_path / "b")).restore({"sd": out})
    for i, r in enumerate(ref):
        assert torch.equal(out[f"t{i}"], r), i
