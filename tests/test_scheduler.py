"""Engine scheduling helpers: the shared host-memory gate and I/O threads."""

import asyncio

from hipsnapshot.engine.scheduler import MemoryGate, execute_write_reqs
from hipsnapshot.io_types import BufferConsumer, BufferStager, ReadReq, StagedBuffer, WriteReq
from hipsnapshot.storage.memory import MemoryStoragePlugin


class _C(BufferConsumer):
    def __init__(self, n):
        self.n = n

    async def consume_buffer(self, buf, executor=None):
        pass

    def get_consuming_cost_bytes(self):
        return self.n


def test_memory_gate_admission():
    g = MemoryGate(100)
    assert g.try_admit(150)        # nothing held: an oversized request still runs
    assert not g.try_admit(1)
    g.release(150)
    assert g.try_admit(60) and g.try_admit(40) and not g.try_admit(1)


class _Stager(BufferStager):
    def __init__(self, n, log):
        self.n, self.log = n, log

    async def stage_buffer(self, executor=None):
        self.log.append(("stage", self.n))
        await asyncio.sleep(0)
        return StagedBuffer(bytearray(self.n))

    def get_staging_cost_bytes(self):
        return self.n


def test_two_pipelines_share_one_budget():
    """The deferred pipeline of an async take only stages what the first
    pipeline's unwritten buffers left of the budget."""

    async def main():
        storage = MemoryStoragePlugin(root="gate")
        gate = MemoryGate(100)
        held = []
        log = []
        first = await execute_write_reqs([WriteReq(f"a{i}", _Stager(40, log)) for i in range(2)],
                                         storage, 100, 0, gate=gate)
        held.append(gate.in_use)   # the first pipeline's buffers are not written yet
        second = await execute_write_reqs([WriteReq(f"b{i}", _Stager(40, log)) for i in range(3)],
                                          storage, 100, 0, gate=gate)
        await first.complete()
        await second.complete()
        return held, gate.in_use

    held, end = asyncio.run(main())
    assert held[0] <= 100 and end == 0


def test_io_threads_follow_cpu_share_and_local_ranks(monkeypatch):
    """Default native I/O workers: 2 x CPUs / ranks on the host, in [4, 16];
    an explicit HIPSNAPSHOT_IO_THREADS wins."""
    import os

    from hipsnapshot import knobs

    monkeypatch.delenv("HIPSNAPSHOT_IO_THREADS", raising=False)
    monkeypatch.delenv("TORCHSNAPSHOT_IO_THREADS", raising=False)
    monkeypatch.setattr(os, "sched_getaffinity", lambda pid: set(range(16)))
    monkeypatch.setattr(knobs, "_cgroup_cpu_quota", lambda root="": None)
    try:
        knobs.set_local_ranks_hint(1)
        assert knobs.get_io_threads() == 16
        knobs.set_local_ranks_hint(4)
        assert knobs.get_io_threads() == 8
        knobs.set_local_ranks_hint(8)
        assert knobs.get_io_threads() == 4
        knobs.set_local_ranks_hint(64)
        assert knobs.get_io_threads() == 4
        monkeypatch.setenv("HIPSNAPSHOT_IO_THREADS", "12")
        assert knobs.get_io_threads() == 12
    finally:
        knobs.set_local_ranks_hint(1)


class _ThreadStager(BufferStager):
    """Stager with the synchronous entry point: staged on scheduler workers."""

    thread_staging = True

    def __init__(self, n, track, fail=False):
        self.n, self.track, self.fail = n, track, fail

    async def stage_buffer(self, executor=None):
        return self.stage_buffer_sync()

    def stage_buffer_sync(self):
        import threading
        import time

        if self.fail:
            raise RuntimeError("staging failed")
        with self.track["lock"]:
            self.track["live"] += self.n
            self.track["peak"] = max(self.track["peak"], self.track["live"])
            self.track["threads"].add(threading.get_ident())
        time.sleep(0.002)

        def release():
            with self.track["lock"]:
                self.track["live"] -= self.n

        return StagedBuffer(bytearray(self.n), release=release)

    def get_staging_cost_bytes(self):
        return self.n


class _SlowStorage(MemoryStoragePlugin):
    async def write(self, write_io):
        await asyncio.sleep(0.003)
        await super().write(write_io)


def _track():
    import threading

    return {"lock": threading.Lock(), "live": 0, "peak": 0, "threads": set()}


def test_thread_staging_respects_budget_and_writes_everything():
    """Worker threads pull requests themselves: host memory held by staged,
    not yet written buffers stays within the budget (one oversized request
    aside), several workers take part, and every blob is written."""
    from hipsnapshot.storage.memory import _STORE

    track = _track()
    reqs = [WriteReq(path=f"b{i}", buffer_stager=_ThreadStager(100 + i, track))
            for i in range(40)]

    async def main():
        storage = _SlowStorage(root="tstage")
        pending = await execute_write_reqs(reqs, storage, memory_budget_bytes=350, rank=0,
                                           stage_threads=4, io_concurrency=4)
        await pending.complete()
        return pending.stats

    stats = asyncio.new_event_loop().run_until_complete(main())
    assert stats.bytes_written == sum(100 + i for i in range(40))
    assert all(f"tstage/b{i}" in _STORE for i in range(40))
    assert track["peak"] <= 350 and track["live"] == 0
    assert len(track["threads"]) > 1


def test_thread_staging_failure_stops_workers_and_releases_buffers():
    track = _track()
    reqs = [WriteReq(path=f"f{i}", buffer_stager=_ThreadStager(64, track, fail=(i == 5)))
            for i in range(30)]

    async def main():
        storage = _SlowStorage(root="tfail")
        pending = await execute_write_reqs(reqs, storage, memory_budget_bytes=256, rank=0,
                                           stage_threads=3, io_concurrency=2)
        await pending.complete()

    import pytest

    with pytest.raises(RuntimeError, match="staging failed"):
        asyncio.new_event_loop().run_until_complete(main())
    assert track["live"] == 0  # every staged buffer went back


def test_io_threads_respect_cgroup_cpu_quota(tmp_path, monkeypatch):
    """A 16-CPU quota on a 256-CPU affinity mask sizes writers by the quota:
    1 rank -> 16 workers, 8 ranks on the host -> 4 each (not 16 each)."""
    from hipsnapshot import knobs

    (tmp_path / "cpu.max").write_text("1600000 100000\n")
    assert knobs._cgroup_cpu_quota(str(tmp_path)) == 16.0
    (tmp_path / "cpu.max").write_text("max 100000\n")
    assert knobs._cgroup_cpu_quota(str(tmp_path)) is None
    v1 = tmp_path / "v1"
    (v1 / "cpu").mkdir(parents=True)
    (v1 / "cpu" / "cpu.cfs_quota_us").write_text("400000\n")
    (v1 / "cpu" / "cpu.cfs_period_us").write_text("100000\n")
    assert knobs._cgroup_cpu_quota(str(v1)) == 4.0

    monkeypatch.delenv("HIPSNAPSHOT_IO_THREADS", raising=False)
    monkeypatch.delenv("TORCHSNAPSHOT_IO_THREADS", raising=False)
    monkeypatch.setattr(knobs.os, "sched_getaffinity", lambda pid: set(range(256)))
    monkeypatch.setattr(knobs, "_cgroup_cpu_quota", lambda root="": 16.0)
    old = knobs._local_ranks_hint[0]
    try:
        knobs._local_ranks_hint[0] = 1
        assert knobs.available_cpus() == 16 and knobs.get_io_threads() == 16
        knobs._local_ranks_hint[0] = 8
        assert knobs.get_io_threads() == 4
        monkeypatch.setattr(knobs, "_cgroup_cpu_quota", lambda root="": None)
        assert knobs.get_io_threads() == 16  # 2 x 256 / 8, capped
    finally:
        knobs._local_ranks_hint[0] = old


def test_mixed_restore_budget_counts_the_native_jobs_pinned_slots(monkeypatch):
    """A restore whose HBM reads go to the native job and whose host reads
    stay in the Python pipeline: the Python part gets the host budget minus
    the job's pinned slots (it used to get all of it)."""
    from hipsnapshot.engine import native_restore, scheduler

    seen = {}

    async def fake_python(read_reqs, storage, budget, rank, *a, **k):
        seen["budget"] = budget
        return scheduler.PipelineStats()

    monkeypatch.setattr(native_restore, "split", lambda reqs, st, b: ({0: [("rr", None, [])]},
                                                                      list(reqs)))
    monkeypatch.setattr(native_restore, "run", lambda jobs, budget, verifier=None: 0)
    monkeypatch.setattr(scheduler, "_execute_python_reads", fake_python)
    budget = 1 << 30
    reqs = [ReadReq(path="x", buffer_consumer=_C(10))]
    asyncio.run(scheduler.execute_read_reqs(reqs, MemoryStoragePlugin(root="m"), budget, 0))
    assert seen["budget"] == budget - native_restore.pinned_bytes(budget)
    small = 4 << 20
    asyncio.run(scheduler.execute_read_reqs(reqs, MemoryStoragePlugin(root="m"), small, 0))
    assert seen["budget"] >= 1 and native_restore.pinned_bytes(small) <= small
