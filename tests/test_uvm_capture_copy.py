"""The UVM capture's copy loop on the CPU: every table lands in its block byte
for byte, whatever the thread split (engine/uvm_capture.py ``Capture._run``).  The GPU half -- the stream gate, managed tables -- is in
tests/test_gpu_uvm_capture.py."""

import types

import pytest
import torch

from hipsnapshot.engine import uvm_capture
from hipsnapshot.knobs import TUNING


class _Block:
    def __init__(self, n):
        self.buf = torch.zeros(n, dtype=torch.uint8)
        self.ptr = self.buf.data_ptr()


@pytest.mark.parametrize("threads,overlap", [(1, False), (4, False), (32, True), (3, False)])
def test_capture_copies_every_table(monkeypatch, threads, overlap):
    released = []
    monkeypatch.setattr(uvm_capture.native, "gate_release", lambda dev, v: released.append(v))
    monkeypatch.setattr(TUNING, "uvm_capture_threads", threads)
    monkeypatch.setattr(TUNING, "uvm_capture_overlap", overlap)
    g = torch.Generator().manual_seed(0)
    sizes = [5 << 20, 1, (1 << 20) + 7, 40 << 20, 4096]  # 40 MiB: split over threads
    tables = [torch.randint(0, 256, (n,), dtype=torch.uint8, generator=g) for n in sizes]
    items = [(types.SimpleNamespace(), t, t.numel()) for t in tables]
    cap = uvm_capture.Capture(0, items)
    cap.blocks = [_Block(n) for n in sizes]
    cap.value = 7
    cap._run([])
    assert cap.error is None
    assert released == [7]  # the gate is always released
    assert all(d.is_set() for d in cap.done)
    for t, b in zip(tables, cap.blocks):
        assert torch.equal(b.buf, t)
    st = uvm_capture.last
    assert st["bytes"] == sum(sizes)
    assert st["threads_per_table"] == max(1, threads // len(sizes))
    assert [r[0] for r in st["tables"]] == sizes


def test_capture_error_still_releases_the_gate(monkeypatch):
    released = []
    monkeypatch.setattr(uvm_capture.native, "gate_release", lambda dev, v: released.append(v))
    t = torch.ones(1 << 20, dtype=torch.uint8)
    cap = uvm_capture.Capture(0, [(types.SimpleNamespace(), t, t.numel())])
    cap.blocks = [None]  # no block: the copy fails
    cap.value = 3
    cap._run([])
    assert cap.error is not None
    assert released == [3]
    assert cap.done[0].is_set()
