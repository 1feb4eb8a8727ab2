"""Engine scheduling helpers: the shared host-memory gate and read ordering."""

import asyncio

from hipsnapshot.engine.scheduler import MemoryGate, execute_write_reqs, order_reads_for_pipeline
from hipsnapshot.io_types import BufferConsumer, BufferStager, ReadReq, StagedBuffer, WriteReq
from hipsnapshot.storage.memory import MemoryStoragePlugin


class _C(BufferConsumer):
    def __init__(self, n):
        self.n = n

    async def consume_buffer(self, buf, executor=None):
        pass

    def get_consuming_cost_bytes(self):
        return self.n


def test_read_order_small_lead_then_largest_first():
    from hipsnapshot.knobs import override_knob

    sizes = [300, 5 << 20, 100 << 20, 2 << 20, 400 << 20, 7]
    reqs = [ReadReq(path=f"p{i}", buffer_consumer=_C(n)) for i, n in enumerate(sizes)]
    assert order_reads_for_pipeline(reqs) == reqs  # default: manifest order
    with override_knob("READ_ORDER", "pipeline"):
        out = [r.buffer_consumer.n for r in order_reads_for_pipeline(reqs)]
    assert out == [2 << 20, 400 << 20, 100 << 20, 5 << 20, 300, 7]


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
