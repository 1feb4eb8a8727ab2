"""Drain helper process (csrc/hsdrain_helper.cpp) wire protocol, on the CPU:
startup handshake, unmap of an unknown handle, a job whose arena cannot be
mapped (reported, not fatal), restart after the helper died, EOF exit.  The
GPU tests (tests/test_gpu.py::test_drain_process_*) run real drains."""

import os
import signal

import pytest
import torch  # noqa: F401  (loads the HIP runtime the helper reuses)

from hipsnapshot import _build
from hipsnapshot.engine import drain_process
from hipsnapshot.ops import native


def _helper_or_skip():
    if not os.path.exists(_build.DRAIN_HELPER) or not os.path.exists(_build.HSGPU_SO):
        pytest.skip("native libraries not built")
    if native.hip_runtime_path() is None:
        pytest.skip("no HIP runtime loaded by torch")
    return drain_process.DrainHelper()


def test_helper_protocol_roundtrip(tmp_path):
    h = _helper_or_skip()
    try:
        h.close_handle(b"\0" * 64)  # not mapped: a no-op
        path = str(tmp_path / "x" / "blob")
        rc, written, sums, stats, map_s, msg = h.drain(
            0, b"\1" * 64, [(0, 100, path), (4096, 7, path + "2")], 1 << 20, 2, 1, 0, 8,
            close_after=True)
        assert rc == -10000 and "mapping the arena failed" in msg
        assert written == 0 and sums == [0, 0] and len(stats) == len(native.NativeDrain.STATS)
        assert map_s >= 0 and not os.path.exists(path)
    finally:
        h.shutdown()
    assert h.proc.returncode == 0  # EOF on stdin ends it cleanly


def test_helper_death_is_reported(tmp_path):
    h = _helper_or_skip()
    os.kill(h.proc.pid, signal.SIGKILL)
    h.proc.wait()
    with pytest.raises(drain_process.DrainHelperError):
        h.drain(0, b"\1" * 64, [(0, 1, str(tmp_path / "b"))], 1 << 20, 2, 1, 0, 8, False)
    h.shutdown()


def test_forget_arena_queues_unmap():
    drain_process._mapped[1234] = b"h" * 64
    try:
        drain_process.forget_arena(1234)
        drain_process.forget_arena(99)  # never mapped: nothing queued
        assert drain_process._to_close == [b"h" * 64] and 1234 not in drain_process._mapped
    finally:
        drain_process._mapped.clear()
        drain_process._to_close.clear()


def test_helper_unavailable_falls_back(monkeypatch, tmp_path):
    """No helper binary: drain() returns None (the caller drains in process)
    and the failure is remembered instead of retried on every take."""
    monkeypatch.setattr(drain_process, "_helper", None)
    monkeypatch.setattr(drain_process, "_start_failed", None)
    monkeypatch.setattr(_build, "DRAIN_HELPER", str(tmp_path / "missing_helper"))
    if native.hip_runtime_path() is None:
        pytest.skip("no HIP runtime loaded by torch")
    assert not drain_process.available()
    assert "not built" in drain_process._start_failed
    assert drain_process.drain(0, 0, False, [], 1 << 20, 2, 1, 0, 8) is None
