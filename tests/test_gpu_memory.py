"""Adaptive memory retention (engine/memory.py) on the GPU: what hipsnapshot
keeps between checkpoints goes back when the trainer runs short.

Reference behaviour: `/root/reference/torchsnapshot/scheduler.py:45-65` sizes
its buffers from the memory available and keeps nothing between takes."""

import pytest
import torch

from hipsnapshot import Snapshot, StateDict, memory_held
from hipsnapshot.engine import memory
from hipsnapshot.knobs import override_knob

pytestmark = pytest.mark.gpu

GiB = 1 << 30


@pytest.fixture(autouse=True)
def _give_hbm_back():
    """These tests fill the device on purpose: hand torch's cached blocks
    back to the driver afterwards, or the next tests' worker processes (other
    processes on the same GPU) find no free HBM."""
    yield
    import gc

    from hipsnapshot import release_snapshot_memory

    gc.collect()
    release_snapshot_memory()
    torch.cuda.synchronize()
    torch.cuda.empty_cache()


def _state(dev, nbytes):
    n = nbytes // 2 // 4
    g = torch.Generator(device=dev).manual_seed(3)
    return StateDict(**{f"w{i}": torch.randn(n, device=dev, generator=g).to(torch.bfloat16)
                        for i in range(4)})


def test_trainer_allocation_after_async_take_succeeds(gpu, tmp_path):
    """After an async_take of S bytes the trainer allocates what fits only if
    the take's arena is not held: the drain's end sees the headroom below the
    reserve and hands the arena back to torch's allocator."""
    dev = gpu.index or 0
    S = 2 * GiB
    reserve = 8 * GiB
    with override_knob("HBM_STAGING_RESERVE_BYTES", reserve):
        sd = _state(gpu, S)
        pending = Snapshot.async_take(str(tmp_path / "a"), {"sd": sd})
        held = memory_held(dev)["hbm_arena_bytes"]
        assert held >= S  # the state went into the arena
        # the trainer grows while the drain runs: headroom ends 1 GiB short
        filler = torch.empty(memory.headroom(dev) - reserve + GiB, dtype=torch.uint8,
                             device=gpu)
        pending.wait()
        assert memory_held(dev)["hbm_arena_bytes"] == 0
        room = memory.headroom(dev)
        assert room >= reserve - GiB + S - 64 * (1 << 20)
        x = torch.empty(room - 256 * (1 << 20), dtype=torch.uint8, device=gpu)
        assert room - 256 * (1 << 20) > reserve - GiB  # would not fit beside the arena
        del x, filler
    # bitwise
    out = StateDict(**{k: torch.zeros_like(v) for k, v in sd.items()})
    Snapshot(str(tmp_path / "a")).restore({"sd": out})
    for k in sd:
        assert torch.equal(out[k], sd[k]), k


def test_arena_kept_with_headroom(gpu, tmp_path):
    """With room to spare the arena stays for the next take (no allocation
    beside the training step)."""
    dev = gpu.index or 0
    with override_knob("HBM_STAGING_RESERVE_BYTES", GiB):
        sd = _state(gpu, 256 << 20)
        Snapshot.async_take(str(tmp_path / "k"), {"sd": sd}).wait()
        assert memory_held(dev)["hbm_arena_bytes"] >= 256 << 20
    from hipsnapshot import release_hbm_arena

    assert release_hbm_arena() >= 256 << 20
    assert memory_held(dev)["hbm_arena_bytes"] == 0


def test_restore_pools_trimmed_under_pressure(gpu, tmp_path):
    """After a restore, the restore pools keep their rings only while the
    trainer keeps its headroom; short of it they go to 0."""
    dev = gpu.index or 0
    sd = _state(gpu, 3 * GiB)
    Snapshot.take(str(tmp_path / "r"), {"sd": sd})
    out = StateDict(**{k: torch.zeros_like(v) for k, v in sd.items()})
    with override_knob("HBM_STAGING_RESERVE_BYTES", GiB):
        Snapshot(str(tmp_path / "r")).restore({"sd": out})
        kept = memory_held(dev)["restore_pool_idle_bytes"]
        assert kept > 0  # room to spare: the rings stay
    for k in sd:
        assert torch.equal(out[k], sd[k]), k
    reserve = 8 * GiB
    with override_knob("HBM_STAGING_RESERVE_BYTES", reserve):
        filler = torch.empty(memory.headroom(dev) - reserve + GiB, dtype=torch.uint8, device=gpu)
        for v in out.values():
            v.zero_()
        Snapshot(str(tmp_path / "r")).restore({"sd": out})
        assert memory_held(dev)["restore_pool_idle_bytes"] == 0
        del filler
    for k in sd:
        assert torch.equal(out[k], sd[k]), k


def test_oom_releases_idle_snapshot_memory(gpu, tmp_path):
    """A torch OOM while hipsnapshot holds an idle arena releases it, so the
    trainer's retry succeeds."""
    dev = gpu.index or 0
    with override_knob("HBM_STAGING_RESERVE_BYTES", GiB):
        sd = _state(gpu, 2 * GiB)
        Snapshot.async_take(str(tmp_path / "o"), {"sd": sd}).wait()
        arena = memory_held(dev)["hbm_arena_bytes"]
        assert arena >= 2 * GiB
        want = memory.headroom(dev) + GiB  # fits only with the arena back
        with pytest.raises(torch.cuda.OutOfMemoryError):
            torch.empty(want, dtype=torch.uint8, device=gpu)
        assert memory_held(dev)["hbm_arena_bytes"] == 0
        x = torch.empty(want, dtype=torch.uint8, device=gpu)
        del x


def test_memory_held_reports_pinned_pool(gpu, tmp_path):
    sd = _state(gpu, 64 << 20)
    Snapshot.take(str(tmp_path / "p"), {"sd": sd})
    h = memory_held()
    assert h["pinned_held_bytes"] >= h["pinned_in_use_bytes"] >= 0
    assert h["hbm_held_bytes"] == (h["hbm_arena_bytes"] + h["restore_pool_idle_bytes"]
                                   + h["restore_pool_live_bytes"] + h["uncached_pool_bytes"])


def test_vmm_free_gives_the_memory_back(gpu):
    """hsg_rt_vmm_free unmaps and releases the physical memory (the virtual
    range stays reserved): 100 cycles of 4 GiB (400 GiB in all) leave the
    device's free memory where it was."""
    lib = __import__("hipsnapshot.ops.native", fromlist=["x"]).require_gpu_lib()
    torch.cuda.synchronize()
    free0, _ = torch.cuda.mem_get_info()
    for i in range(100):
        p = lib.hsg_rt_vmm_alloc(0, 4 * GiB, i % 2)
        assert p, lib.hsg_rt_last_error()
        assert lib.hsg_rt_vmm_free(p) == 0
    free1, _ = torch.cuda.mem_get_info()
    assert free1 >= free0 - GiB, (free0, free1)
