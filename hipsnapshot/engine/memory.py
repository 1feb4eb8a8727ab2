"""What hipsnapshot holds between checkpoints, and when it lets go.

Three kinds of memory outlive a take or a restore, each kept because a later
operation reuses it:

* the async-take HBM arena (``hbm_staging``): a torch tensor the size of the
  frozen state, so the next ``async_take`` does not allocate beside a running
  training step;
* the native restore's device pools (``csrc/hsrestore.cpp``): upload and
  scratch rings outside torch's allocator, on VMM ranges (``hshost.hip``);
* the pinned host pool (``csrc/hsgpu.hip``): registered staging and slot
  blocks.

The reference frees everything after each take and sizes its buffers from
the memory available (`/root/reference/torchsnapshot/scheduler.py:45-65`,
`/root/reference/README.md:43`).  Here the kept memory is re-checked against
what the trainer has left:

* after a drain, the idle arena is dropped (back to torch's caching
  allocator, where the trainer can use it) when the device's headroom -- free
  HBM plus torch's cached-but-unused blocks -- is below
  ``HBM_STAGING_RESERVE_BYTES``;
* after a restore, the restore pools keep ``restore_keep_bytes`` idle only if
  the headroom stays above that reserve with them; otherwise they go to 0;
* on a torch out-of-memory error, every idle block is released at once (a
  retry of the failed allocation then finds it);
* the pinned pool is capped at the rank's host memory budget and its idle
  blocks are unregistered after ``pinned_idle_trim_s`` seconds without a
  snapshot operation.

``held()`` reports all of it; ``bench.py`` prints it between takes.
"""

from __future__ import annotations

import logging
import threading
import time
from typing import Dict, Optional

import torch

from .. import knobs
from ..ops import native

logger = logging.getLogger(__name__)


def headroom(dev: int) -> int:
    """Bytes a trainer on ``dev`` can still allocate: free HBM plus the
    blocks torch's caching allocator holds unused."""
    from .hbm_staging import _cached_unused

    free, _total = torch.cuda.mem_get_info(dev)
    return int(free) + max(0, _cached_unused(dev))


def held(dev: Optional[int] = None) -> Dict[str, int]:
    """Memory hipsnapshot holds now (device ``dev``, or every device): the
    async-take arena, the restore pools (idle / in use), the uncached block
    pool, and the pinned host pool (registered / in use)."""
    from .hbm_staging import _kept

    out = {"hbm_arena_bytes": 0, "restore_pool_idle_bytes": 0, "restore_pool_live_bytes": 0,
           "uncached_pool_bytes": 0, "pinned_held_bytes": 0, "pinned_in_use_bytes": 0}
    for d, k in _kept.items():
        if dev is None or d == dev:
            out["hbm_arena_bytes"] += int(k[0].numel())
    if native.gpu_available():
        pb = native.restore_pool_bytes(-1 if dev is None else dev)
        out["restore_pool_idle_bytes"] = pb["upload_idle"] + pb["scratch_idle"]
        out["restore_pool_live_bytes"] = pb["upload_live"] + pb["scratch_live"]
        out["uncached_pool_bytes"] = native.uncached_pool_bytes()
        cached, in_use = native.pinned_stats()
        out["pinned_held_bytes"], out["pinned_in_use_bytes"] = int(cached), int(in_use)
    out["hbm_held_bytes"] = (out["hbm_arena_bytes"] + out["restore_pool_idle_bytes"]
                             + out["restore_pool_live_bytes"] + out["uncached_pool_bytes"])
    return out


def settle_arena(dev: int) -> int:
    """After a drain: drop ``dev``'s idle kept arena when the trainer's
    headroom is below the reserve.  Returns the bytes released."""
    from .hbm_staging import _drop_kept, _kept

    k = _kept.get(dev)
    if k is None or k[1]:
        return 0
    try:
        room = headroom(dev)
    except Exception:  # noqa: BLE001 - no device query: keep it
        return 0
    if room >= knobs.hbm_staging_reserve_bytes():
        return 0
    t = _kept.pop(dev)[0]
    _drop_kept(t)
    n = int(t.numel())
    del t
    logger.info(f"cuda:{dev}: headroom {room} B below the reserve: async-take arena of {n} B "
                "released")
    return n


def settle_restore_pools() -> int:
    """After a restore: trim each device's restore pools to the keep size, or
    to 0 when keeping them would leave the trainer less than the reserve.
    Returns the bytes freed."""
    if not native.gpu_available():
        return 0
    freed = 0
    keep = knobs.get_restore_keep_bytes()
    reserve = knobs.hbm_staging_reserve_bytes()
    for dev in range(torch.cuda.device_count()):
        pb = native.restore_pool_bytes(dev)
        idle = pb["upload_idle"] + pb["scratch_idle"]
        if idle == 0:
            continue
        try:
            room = headroom(dev)
        except Exception:  # noqa: BLE001
            room = reserve + idle
        k = keep if room - min(idle, 2 * keep) >= reserve else 0
        freed += native.restore_trim(dev, k)
    return freed


def release_idle(dev: Optional[int] = None) -> int:
    """Release every idle block hipsnapshot holds on the device(s): kept
    arenas, restore pool blocks, uncached blocks.  Busy ones stay."""
    from .hbm_staging import release_hbm_arena
    from .native_restore import join_prewarm

    freed = release_hbm_arena()
    if native.gpu_available():
        join_prewarm()
        devs = range(torch.cuda.device_count()) if dev is None else [dev]
        for d in devs:
            freed += native.restore_trim(d, 0)
        freed += native.uncached_trim()
    return freed


# ---- torch out-of-memory hook -------------------------------------------------

_oom_hooked = False
_oom_lock = threading.Lock()


def _on_oom(device, alloc, device_allocated, device_free) -> None:  # pragma: no cover - GPU
    try:
        n = release_idle(int(device))
        logger.warning(f"cuda:{device}: out of memory allocating {alloc} B; hipsnapshot "
                       f"released {n} B of idle snapshot memory (retry the allocation)")
    except Exception as e:  # noqa: BLE001 - never raise inside torch's allocator
        logger.debug(f"release on OOM failed: {e}")


def install_oom_hook() -> None:
    """Register ``_on_oom`` with torch's caching allocator once per process."""
    global _oom_hooked
    if _oom_hooked:
        return
    with _oom_lock:
        if _oom_hooked:
            return
        attach = getattr(torch._C, "_cuda_attach_out_of_memory_observer", None)
        if attach is not None and torch.cuda.is_available():
            try:
                attach(_on_oom)
            except Exception as e:  # noqa: BLE001
                logger.debug(f"no OOM observer: {e}")
        _oom_hooked = True


# ---- pinned pool: cap + idle trim ----------------------------------------------

_last_use = [0.0]
_trimmer: Optional[threading.Thread] = None
_trim_lock = threading.Lock()
_active = [0]


def pinned_cap_bytes(pg=None) -> int:
    """The pinned pool's cap: ``PINNED_POOL_MAX_BYTES`` when set, else the
    rank's host memory budget (never below what one drain / restore keeps in
    slots)."""
    override = knobs._get_int("PINNED_POOL_MAX_BYTES", 0)
    if override:
        return override
    from .scheduler import get_process_memory_budget_bytes

    floor = knobs.TUNING.drain_slots * knobs.TUNING.drain_slot_bytes + \
        knobs.TUNING.restore_slots * knobs.TUNING.restore_slot_bytes
    return max(floor, get_process_memory_budget_bytes(pg))


def op_begin(pg=None) -> None:
    """A snapshot operation starts: note the time, apply the pinned cap,
    hook OOM, and make sure the idle trimmer runs."""
    _active[0] += 1
    _last_use[0] = time.monotonic()
    if not native.gpu_available():
        return
    install_oom_hook()
    try:
        native.require_gpu_lib().hsg_pinned_set_limit(pinned_cap_bytes(pg))
    except Exception as e:  # noqa: BLE001
        logger.debug(f"pinned cap not applied: {e}")
    _ensure_trimmer()


def op_end() -> None:
    _active[0] = max(0, _active[0] - 1)
    _last_use[0] = time.monotonic()


def _ensure_trimmer() -> None:
    global _trimmer
    if knobs.TUNING.pinned_idle_trim_s <= 0:
        return
    with _trim_lock:
        if _trimmer is not None and _trimmer.is_alive():
            return
        _trimmer = threading.Thread(target=_trim_loop, name="hs-pinned-idle-trim", daemon=True)
        _trimmer.start()


def _trim_loop() -> None:
    while True:
        idle_s = knobs.TUNING.pinned_idle_trim_s
        if idle_s <= 0:
            return
        time.sleep(max(0.05, min(idle_s / 4, 30.0)))
        if _active[0] == 0 and time.monotonic() - _last_use[0] >= idle_s:
            try:
                n = native.pinned_trim()
                if n:
                    logger.info(f"pinned pool idle for {idle_s:.0f} s: {n} B unregistered")
            except Exception:  # noqa: BLE001 - interpreter shutdown
                return
            _last_use[0] = time.monotonic()
