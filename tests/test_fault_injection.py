"""Failure paths of the read / write pipelines (a failing read must
not let the other in-flight reads' destinations go back to the pinned pool
while storage is still filling them)."""

import asyncio
import os
import threading
from unittest import mock

import pytest
import torch

from hipsnapshot import Snapshot, StateDict
from hipsnapshot.knobs import override_is_batching_disabled
from hipsnapshot.storage.fs import FSStoragePlugin, _uncancellable


def test_uncancellable_waits_for_job():
    """Cancelling a task that awaits a storage job does not end it before the
    job (which owns the caller's buffer) has completed."""

    async def main():
        loop = asyncio.get_running_loop()
        job = loop.create_future()
        order = []

        async def reader():
            try:
                await _uncancellable(job)
            finally:
                order.append(("reader_exit", job.done()))

        t = asyncio.ensure_future(reader())
        await asyncio.sleep(0.01)
        t.cancel()
        await asyncio.sleep(0.05)
        assert not t.done(), "reader left while its job was still running"
        job.set_result(7)
        with pytest.raises(asyncio.CancelledError):
            await t
        assert order == [("reader_exit", True)]

    asyncio.run(main())


def test_failing_read_drains_inflight_reads(tmp_path):
    n = 12
    sd = StateDict(**{f"t{i}": torch.randn(64 * 1024) for i in range(n)})
    path = str(tmp_path / "s")
    with override_is_batching_disabled(True):
        Snapshot.take(path, {"sd": sd})

    lock = threading.Lock()
    state = {"active": 0, "max_active": 0, "active_at_raise": None, "cancelled": 0}

    class Faulty(FSStoragePlugin):
        async def read(self, read_io):
            with lock:
                state["active"] += 1
                state["max_active"] = max(state["max_active"], state["active"])
            try:
                if read_io.path.endswith("/t3"):
                    await asyncio.sleep(0.02)
                    raise OSError("injected read failure")
                try:
                    await asyncio.sleep(0.15)  # still in flight when t3 fails
                except asyncio.CancelledError:
                    state["cancelled"] += 1
                    raise
                await super().read(read_io)
            finally:
                with lock:
                    state["active"] -= 1

    out = StateDict(**{f"t{i}": torch.zeros(64 * 1024) for i in range(n)})
    with override_is_batching_disabled(True), \
            mock.patch("hipsnapshot.storage.fs.FSStoragePlugin", Faulty):
        with pytest.raises(OSError, match="injected read failure"):
            Snapshot(path).restore({"sd": out})
        state["active_at_raise"] = state["active"]
    assert state["max_active"] > 1, "test needs several reads in flight"
    assert state["active_at_raise"] == 0, "restore raised while reads were still in flight"
    # in-flight reads are drained, not cancelled: a cancelled coroutine does
    # not stop the engine job that is still filling its destination
    assert state["cancelled"] == 0


def test_failed_restore_leaves_pinned_pool_usable(tmp_path):
    """After a restore whose blobs are missing fails, the same process can
    still take and restore (pools and engine are not left in a bad state)."""
    sd = StateDict(a=torch.arange(1000.0), b=torch.ones(10))
    path = str(tmp_path / "p")
    Snapshot.take(path, {"sd": sd})
    for root, _, files in os.walk(path):
        for f in files:
            if f != ".snapshot_metadata":
                os.remove(os.path.join(root, f))
    out = StateDict(a=torch.zeros(1000), b=torch.zeros(10))
    with pytest.raises(OSError):
        Snapshot(path).restore({"sd": out})
    Snapshot.take(path + "2", {"sd": sd})
    out2 = StateDict(a=torch.zeros(1000), b=torch.zeros(10))
    Snapshot(path + "2").restore({"sd": out2})
    assert torch.equal(out2["a"], sd["a"]) and torch.equal(out2["b"], sd["b"])
