"""engine/memory.py on the CPU: the pinned pool's cap and idle trim, and the
reporting API (the GPU halves are in tests/test_gpu_memory.py)."""

import time

import hipsnapshot
from hipsnapshot import knobs
from hipsnapshot.engine import memory


class _FakeLib:
    def __init__(self):
        self.limits = []

    def hsg_pinned_set_limit(self, n):
        self.limits.append(n)


def test_pinned_cap_is_the_rank_budget_unless_set(monkeypatch):
    from hipsnapshot.engine import scheduler

    monkeypatch.setattr(scheduler, "get_process_memory_budget_bytes", lambda pg=None: 20 << 30)
    assert memory.pinned_cap_bytes() == 20 << 30
    monkeypatch.setattr(scheduler, "get_process_memory_budget_bytes", lambda pg=None: 1 << 20)
    floor = knobs.TUNING.drain_slots * knobs.TUNING.drain_slot_bytes + \
        knobs.TUNING.restore_slots * knobs.TUNING.restore_slot_bytes
    assert memory.pinned_cap_bytes() == floor  # never below one drain + one restore
    with knobs.override_knob("PINNED_POOL_MAX_BYTES", 3 << 30):
        assert memory.pinned_cap_bytes() == 3 << 30


def test_idle_pinned_pool_is_trimmed(monkeypatch):
    from hipsnapshot.ops import native

    lib = _FakeLib()
    trims = []
    monkeypatch.setattr(native, "gpu_available", lambda: True)
    monkeypatch.setattr(native, "require_gpu_lib", lambda: lib)
    monkeypatch.setattr(native, "pinned_trim", lambda: trims.append(time.monotonic()) or 4096)
    monkeypatch.setattr(memory, "pinned_cap_bytes", lambda pg=None: 5 << 30)
    with knobs.override_tuning(pinned_idle_trim_s=0.2):
        memory.op_begin()
        assert lib.limits == [5 << 30]
        time.sleep(0.5)
        assert not trims  # an operation is running: nothing is trimmed
        memory.op_end()
        t_end = time.monotonic()
        deadline = time.monotonic() + 5
        while not trims and time.monotonic() < deadline:
            time.sleep(0.05)
        assert trims and trims[0] - t_end >= 0.19
    # the loop ends once the knob is 0
    with knobs.override_tuning(pinned_idle_trim_s=0):
        deadline = time.monotonic() + 5
        while memory._trimmer is not None and memory._trimmer.is_alive() and \
                time.monotonic() < deadline:
            time.sleep(0.05)
        assert not memory._trimmer.is_alive()


def test_memory_held_on_cpu_is_zero():
    h = hipsnapshot.memory_held()
    assert h["hbm_held_bytes"] == 0 and h["pinned_held_bytes"] == 0
    assert hipsnapshot.release_snapshot_memory() == 0
