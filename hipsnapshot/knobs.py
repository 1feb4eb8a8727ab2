"""Runtime configuration (environment variables + context-manager overrides).

Same knobs and defaults as the reference (`/root/reference/torchsnapshot/knobs.py:21-96`,
`scheduler.py:27-30`): 512 MiB max chunk, 512 MiB max shard piece, 128 MiB slab
threshold, batching on, per-rank memory budget min(0.6*avail/local_ws, 32 GiB).
Every variable is read as ``HIPSNAPSHOT_<NAME>`` first and the reference's
``TORCHSNAPSHOT_<NAME>`` second, so existing job scripts keep working.

MI355X-specific knobs:

* ``HIPSNAPSHOT_IO_THREADS`` (16) -- native I/O engine workers per storage plugin.
* ``HIPSNAPSHOT_COMPRESSION`` (none) -- ``hsz1`` = lossless GPU compression of
  floating-point blobs (see ``ops/codec.py``); per call via ``compression=``.
* ``HIPSNAPSHOT_READ_INFLIGHT`` (8) -- whole-blob reads in flight during restore.
* ``HIPSNAPSHOT_IO_READ_SPLIT_BYTES`` (8 MiB) -- reads larger than 1.5x this are
  split across I/O workers (parallel page-cache reads of one file; 0 = off).
* ``HIPSNAPSHOT_STAGE_THREADS`` (4) -- concurrent staging jobs (DMA/pack/serialize).
* ``HIPSNAPSHOT_FS_DIRECT_IO`` (0) -- O_DIRECT for the aligned body of blobs.
* ``HIPSNAPSHOT_FS_FSYNC`` (0) -- fdatasync every blob (durable checkpoints).
* ``HIPSNAPSHOT_ASYNC_HBM_STAGING`` (1) -- async_take snapshots device state into
  spare HBM with one gather-kernel launch and drains it in the background.
* ``HIPSNAPSHOT_HBM_STAGING_RESERVE_BYTES`` (8 GiB) -- HBM left free for training.
* ``HIPSNAPSHOT_HBM_STAGING_MAX_BYTES`` (unlimited) -- cap on the async-take HBM
  arena; requests beyond it are host-staged before ``async_take`` returns.
* ``HIPSNAPSHOT_HBM_ARENA_KEEP`` (1) -- keep the async-take HBM arena between
  takes (``hipsnapshot.release_hbm_arena()`` frees it).
* ``HIPSNAPSHOT_NATIVE_DRAIN`` (1) -- drain raw frozen blobs to local files in
  C++ threads (``csrc/hsdrain.hip``); ``HIPSNAPSHOT_DRAIN_SLOT_BYTES`` (64 MiB),
  ``_DRAIN_SLOTS`` (16), ``_DRAIN_WRITERS`` (min(16, io threads, half the rank's CPU share)),
  ``_DRAIN_NICE`` (10: nice increment of its threads), ``_DRAIN_DIRECT_IO`` (0:
  O_DIRECT files, no page-cache copy).
* ``HIPSNAPSHOT_NATIVE_RESTORE`` (1) -- reads landing in HBM go through one
  native job per device (``csrc/hsrestore.hip``): ``_RESTORE_SLOT_BYTES``
  (128 MiB), ``_RESTORE_FIRST_BYTES`` (16 MiB), ``_RESTORE_PIECE_BYTES``
  (4 MiB), ``_RESTORE_SLOTS`` (6), ``_RESTORE_READERS``,
  ``_RESTORE_DEVICE_BUDGET`` (2 GiB), ``_RESTORE_KEEP_BYTES`` (2.25 GiB),
  ``_RESTORE_PREWARM`` (1: fill its pools while the reads are planned),
  ``_RESTORE_PLAN_CACHE`` (1), ``_HSZ_DECODE2`` (``staged-pf``; ``lds`` = the
  round-3 HSZ1 decoder).
* ``HIPSNAPSHOT_ASYNC_DEVICE_CODEC`` (raw) -- ``same``: an async take encodes
  its frozen device state like a blocking take.
* ``HIPSNAPSHOT_GC_AFTER_PLAN`` (1) -- one full Python GC pass at the end of a
  take that built a new take plan, not in a later take or training step.
* ``HIPSNAPSHOT_REBALANCE`` (0) -- move whole blobs from loaded ranks to idle
  ones over xGMI before a sync take writes (``parallel/rebalance.py``).
* ``HIPSNAPSHOT_UVM_ASSUME_HOST`` (1 unless the device runs with XNACK on) -- managed tensors
  never placed with ``ops.uvm.place`` are host-resident: blocking takes write
  host-resident UVM pages in place and restores read into them, instead of
  copying them over PCIe and back.
* ``HIPSNAPSHOT_SLAB_ALIGN`` (256) -- byte alignment of slab members.
* ``HIPSNAPSHOT_TRUST_OBJECTS`` (0) -- allow full unpickling of ``object``
  entries written by OTHER tools (our own writes are trusted by the reader).
"""

from __future__ import annotations

import functools
import math
import os
from contextlib import contextmanager
from typing import Any, Generator, Optional

_PREFIXES = ("HIPSNAPSHOT_", "TORCHSNAPSHOT_")

MAX_CHUNK_SIZE = "MAX_CHUNK_SIZE_BYTES_OVERRIDE"
MAX_SHARD_SIZE = "MAX_SHARD_SIZE_BYTES_OVERRIDE"
SLAB_SIZE_THRESHOLD = "SLAB_SIZE_THRESHOLD_BYTES_OVERRIDE"
DISABLE_BATCHING = "DISABLE_BATCHING"
MEMORY_BUDGET = "PER_RANK_MEMORY_BUDGET_BYTES"

_DEFAULT_MAX_CHUNK_SIZE_BYTES = 512 * 1024 * 1024
_DEFAULT_MAX_SHARD_SIZE_BYTES = 512 * 1024 * 1024
_DEFAULT_SLAB_SIZE_THRESHOLD_BYTES = 128 * 1024 * 1024
MAX_PER_RANK_MEMORY_BUDGET_BYTES = 32 * 1024 * 1024 * 1024


def _get(name: str) -> Optional[str]:
    for p in _PREFIXES:
        v = os.environ.get(p + name)
        if v is not None:
            return v
    return None


def _get_int(name: str, default: int) -> int:
    v = _get(name)
    return default if v is None else int(v)


def _get_bool(name: str, default: bool) -> bool:
    v = _get(name)
    if v is None:
        return default
    return v.strip().lower() in ("1", "true", "yes", "on")


def get_max_chunk_size_bytes() -> int:
    return _get_int(MAX_CHUNK_SIZE, _DEFAULT_MAX_CHUNK_SIZE_BYTES)


def get_max_shard_size_bytes() -> int:
    return _get_int(MAX_SHARD_SIZE, _DEFAULT_MAX_SHARD_SIZE_BYTES)


def get_slab_size_threshold_bytes() -> int:
    return _get_int(SLAB_SIZE_THRESHOLD, _DEFAULT_SLAB_SIZE_THRESHOLD_BYTES)


def is_batching_disabled() -> bool:
    return _get_bool(DISABLE_BATCHING, False)


def get_memory_budget_override() -> Optional[int]:
    v = _get(MEMORY_BUDGET)
    return None if v is None else int(v)


_local_ranks_hint = [1]


def set_local_ranks_hint(n: int) -> None:
    """Ranks of this job on this host (learnt from the take's first
    collective); sizes the default I/O thread count."""
    _local_ranks_hint[0] = max(1, int(n))


def _cgroup_cpu_quota(root: str = "/sys/fs/cgroup") -> Optional[float]:
    """CPUs' worth of time the cgroup may use (CFS bandwidth quota / period),
    None when unlimited or unknown.  cgroup v2 ``cpu.max``, else v1
    ``cpu.cfs_quota_us`` / ``cpu.cfs_period_us``."""
    try:
        with open(os.path.join(root, "cpu.max")) as f:
            quota, period = f.read().split()[:2]
        return None if quota == "max" else int(quota) / int(period)
    except (OSError, ValueError):
        pass
    try:
        with open(os.path.join(root, "cpu", "cpu.cfs_quota_us")) as f:
            quota = int(f.read())
        with open(os.path.join(root, "cpu", "cpu.cfs_period_us")) as f:
            period = int(f.read())
        return None if quota <= 0 else quota / period
    except (OSError, ValueError):
        return None


def available_cpus() -> int:
    """CPUs this process can actually use: its affinity mask, capped by the
    cgroup's CPU quota.  (A GPU box here shows 256 CPUs in the mask and a
    16-CPU quota in ``cpu.max``: every thread above the quota only makes the
    whole group wait for the next period.)"""
    try:
        cpus = len(os.sched_getaffinity(0))
    except (AttributeError, OSError):  # pragma: no cover - non-Linux
        cpus = os.cpu_count() or 16
    quota = _cgroup_cpu_quota()
    if quota is not None:
        cpus = min(cpus, max(1, int(math.ceil(quota))))
    return cpus


def get_io_threads() -> int:
    """Native I/O workers per storage plugin: ``HIPSNAPSHOT_IO_THREADS``, else
    2 x (CPUs this process can use, ``available_cpus``) / (ranks on this
    host), within [4, 16].  Buffered writes scale with threads only up to the
    CPU share: 8 processes x 16 writer threads on 16 CPUs wrote 26 GB/s to
    the page cache, 8 x 2 threads 108 GB/s (scripts/probes/pagecache_write_probe.py,
    profiles/pagecache/)."""
    v = _get("IO_THREADS")
    if v is not None:
        return int(v)
    return max(4, min(16, 2 * available_cpus() // _local_ranks_hint[0]))


def compress_host_tensors() -> bool:
    return _get_bool("COMPRESSION_HOST", False)


def get_read_inflight() -> int:
    return max(1, _get_int("READ_INFLIGHT", 8))


def get_compression() -> str:
    return str(_get("COMPRESSION") or "none")


def get_io_read_split_bytes() -> int:
    return _get_int("IO_READ_SPLIT_BYTES", 8 * 1024 * 1024)


def get_d2h_engine() -> str:
    """Engine for bulk device -> pinned-host copies: ``blit`` = hipMemcpyAsync
    (the HIP runtime's copy kernel on the CUs), ``sdma`` = the GPU's DMA
    engines through ROCr (``csrc/hsdma.hip``; falls back to blit when ROCr
    reports no engine).  Default sdma: same PCIe-bound bandwidth, no CU time,
    +4 % on the Llama-3-8B save (profiles/dma/)."""
    v = str(_get("D2H_ENGINE") or "sdma").strip().lower()
    if v not in ("blit", "sdma"):
        raise ValueError(f"HIPSNAPSHOT_D2H_ENGINE must be blit or sdma, not {v!r}")
    return v


def get_h2d_engine() -> str:
    """Engine for a restore's uploads of encoded (HSZ1) frames: ``sdma`` (the
    DMA engines through ROCr into uncached device memory, ``csrc/hsdma.hip``)
    or ``hip`` (hipMemcpyAsync, whose calls block for milliseconds when
    several threads upload; profiles/r4/restore_trace/).  Default sdma when
    ROCr reports an engine."""
    v = str(_get("H2D_ENGINE") or "sdma").strip().lower()
    if v not in ("hip", "sdma"):
        raise ValueError(f"HIPSNAPSHOT_H2D_ENGINE must be hip or sdma, not {v!r}")
    return v


def async_dma() -> bool:
    """Staging workers submit their SDMA copy and move on; the writer waits
    for it (engine/staging.py ``d2h_staged``)."""
    return _get_bool("ASYNC_DMA", True)


def get_dma_inflight() -> int:
    """Device -> host SDMA copies in flight per device (async staging)."""
    return max(1, _get_int("DMA_INFLIGHT", 8))


def serial_encode() -> bool:
    """Staging threads take turns launching (and waiting for) HSZ1 encodes on
    a device instead of sharing the CUs (engine/staging.py ``_encode_turn``)."""
    return _get_bool("SERIAL_ENCODE", True)


def get_gil_switch_us() -> int:
    """GIL switch interval (microseconds) while a take / restore runs on the
    calling thread; 0 = leave Python's (5000)."""
    return _get_int("GIL_SWITCH_US", 0)


def thread_staging_enabled() -> bool:
    """Stage writes on long-running worker threads that pull the next request
    themselves (engine/scheduler.py ``_stage_on_threads``); 0 = one event-loop
    round trip per request (custom stagers always take that path)."""
    return _get_bool("THREAD_STAGING", True)


def checksum_enabled() -> bool:
    """Record an hs64 checksum of every blob a take writes
    (``.snapshot_checksums/<rank>``, ops/checksum.py); ``Snapshot.verify``
    checks them."""
    return _get_bool("CHECKSUM", True)


def get_hash_grid() -> int:
    """Workgroups of one blob-checksum launch (0 = whole chip).  Narrow by
    default: a full-width hash saturates HBM reads and slows the concurrent
    SDMA copies (scripts/probes/hash_probe.py); blobs only need hashing at PCIe rate."""
    return _get_int("HASH_GRID", 64)


def get_drain_cus() -> int:
    """Grid cap (workgroups, ~CUs) for the kernels of an async-take drain
    while training continues; 0 (default) = uncapped.  Measured on Llama-3-8B
    + AdamW (profiles/overlap_iso/README.md): caps of 16-128 stretch the drain
    (the encoder runs at 1.8 GB/s per workgroup) without lowering the total
    training time a checkpoint costs (250-400 ms either way), so no cap."""
    return max(0, _get_int("DRAIN_CUS", 0))


def get_read_head_bytes() -> int:
    """Whole HSZ1 blobs larger than twice this are read as a head of this
    many bytes and the rest, as two requests: the head's frames go to the GPU
    while the rest is still being read (the restore's first H2D starts after
    the head, not after the whole first blob).  0 = one read per blob."""
    return max(0, _get_int("READ_HEAD_BYTES", 16 * 1024 * 1024))


def get_read_order() -> str:
    """Restore read order: ``plan`` (manifest order, default) or ``pipeline``
    (a small lead read, then largest first).  Measured A/B on one MI355X,
    Llama-3-8B restore, median of 5: plan 70.7 / 72.8 GB/s, pipeline 65.1 /
    68.2 GB/s (profiles/timeline_r2/read_order.txt)."""
    return str(_get("READ_ORDER") or "plan")


def get_state_dict_barriers() -> str:
    """Barrier after every app-state key's ``state_dict()`` during a take
    (the reference always does, `snapshot.py:362-368`, so user
    ``state_dict()`` collectives cannot interleave across ranks).  ``auto``
    (default): skipped when EVERY rank's statefuls are of kinds whose
    ``state_dict()`` runs no collective (StateDict, RNGState, optimizers,
    modules without FSDP1 wrappers or a custom ``state_dict``); ``always``;
    ``never``."""
    v = str(_get("STATE_DICT_BARRIERS") or "auto").strip().lower()
    return {"1": "always", "true": "always", "0": "never", "false": "never"}.get(v, v)


def rebalance_enabled() -> bool:
    """Move whole blobs from heavily to lightly loaded ranks over xGMI before
    a blocking take stages (parallel/rebalance.py).  Off by default."""
    return _get_bool("REBALANCE", False)


def rebalance_host() -> bool:
    """Let the rebalancer move host (CPU) blobs too (gloo tests)."""
    return _get_bool("REBALANCE_HOST", False)


def rebalance_min_gain() -> float:
    """Stop once the load spread is below this fraction of the mean."""
    return float(_get("REBALANCE_MIN_GAIN") or 0.1)


def hbm_arena_keep() -> bool:
    """Keep the async-take HBM arena allocated between takes and reuse it
    (``hipsnapshot.release_hbm_arena()`` frees it).  Default on."""
    return _get_bool("HBM_ARENA_KEEP", True)


def native_drain_enabled() -> bool:
    """Drain an async take's raw frozen blobs to the local FS in native
    threads (engine/native_drain.py, csrc/hsdrain.hip)."""
    return _get_bool("NATIVE_DRAIN", True)


# native drain sizing: 16 writers x 16 slots of 64 MiB drain the 16 GB
# Llama-3-8B arena at the PCIe rate with an idle trainer (307 ms, was 380-475
# ms with 8 x 12 x 32 MiB; profiles/r3/s2/drain_sizing/).  The writers stay
# within half of this rank's CPU share: a drain runs next to a training
# loop, and writer threads that use up a cgroup CPU quota stall the
# trainer's thread with them (8 writers on the 16-CPU box).
def get_drain_slot_bytes() -> int:
    return max(1 << 20, _get_int("DRAIN_SLOT_BYTES", 64 << 20))


def get_drain_slots() -> int:
    """Pinned slots the native drain cycles through (slots x slot bytes of
    pinned host memory while a drain runs, outside the memory budget)."""
    return max(2, _get_int("DRAIN_SLOTS", 16))


def get_drain_writers() -> int:
    """Writer threads of an async take's native drain: 3 (at most half the
    rank's CPU share, at least 2).  The drain runs beside training: with 8
    writers a launch-bound seq-512 Llama-3-8B step ran 5-9 % slower while a
    48 GB drain was in flight, with 3 writers 2-5 % (the drain takes 2.6 s
    instead of 1.4-2.1 s; the training time lost per checkpoint is about the
    same, 0.22 vs 0.25 of a blocking take; profiles/r4/overlap_ab_writers/)."""
    share = available_cpus() // max(_local_ranks_hint[0], 1)
    return max(1, _get_int("DRAIN_WRITERS", min(3, get_io_threads(), max(2, share // 2))))


def get_drain_boost_writers() -> int:
    """Writer threads of a native drain once its caller blocks on it
    (``PendingSnapshot.wait``): the extra ones are parked until then.  With
    an idle trainer 16 writers drain 16 GB in ~310 ms, 3 in ~490 ms."""
    share = available_cpus() // max(_local_ranks_hint[0], 1)
    return max(1, _get_int("DRAIN_BOOST_WRITERS", min(16, get_io_threads(), max(2, share // 2))))


def get_drain_nice() -> int:
    """Nice increment of the native drain's threads (0-19, default 10): they
    yield a shared core to the training loop's launch thread."""
    return max(0, min(19, _get_int("DRAIN_NICE", 10)))


def _arch_features(arch_name: str) -> dict:
    """``gfx950:sramecc+:xnack-`` -> {"sramecc": "+", "xnack": "-"}."""
    feats = {}
    for f in arch_name.split(":")[1:]:
        if f and f[-1] in "+-":
            feats[f[:-1]] = f[-1]
    return feats


@functools.lru_cache(maxsize=None)
def device_xnack_enabled(index: int = 0) -> bool:
    """Whether the HIP device runs with XNACK (retryable page faults) on, read
    from the device itself (``hipDeviceProp.gcnArchName`` feature suffix), not
    from the environment.  False without a GPU."""
    try:
        import torch

        if not torch.cuda.is_available():
            return False
        name = torch.cuda.get_device_properties(index).gcnArchName
    except Exception:  # noqa: BLE001 -- no device / old torch: XNACK unknown = off
        return False
    return _arch_features(name).get("xnack") == "+"


def uvm_assume_host() -> bool:
    """Managed (UVM) tensors that were never advised / prefetched are in host
    DRAM (blocking takes write them in place).  Default: unless the device runs
    with XNACK on (``device_xnack_enabled``), where pages migrate to the GPU that
    touches them.  Measured: a never-placed table reads at 57 GB/s from a kernel
    (PCIe), 3.9 TB/s once prefetched to the GPU (profiles/r3/uvm/)."""
    if _get("UVM_ASSUME_HOST") is not None:
        return _get_bool("UVM_ASSUME_HOST", True)
    return not device_xnack_enabled()


def drain_avoid_caller_core() -> str:
    """Where the native drain's threads may NOT run, relative to the thread
    that called ``async_take`` (utils/affinity.py): ``"core"`` (default) its
    physical core -- a launch-bound training step loses issue slots to an SMT
    sibling busy with page-cache copies; ``"l3"`` every CPU sharing its L3
    (the writers' streaming copies then evict none of the trainer's cached
    interpreter and allocator state); ``""`` anywhere is fine.  Env
    ``DRAIN_AVOID_CALLER_CORE``: 0/1 or core/l3."""
    v = (_get("DRAIN_AVOID_CALLER_CORE") or "core").strip().lower()
    if v in ("0", "false", "no", "off", ""):
        return ""
    return "l3" if v == "l3" else "core"


def drain_hash_high_priority() -> bool:
    """The native drain's hs64 launches run on a high-priority stream
    (default): at normal priority a training step's GEMMs starved them
    (profiles/r3/drain_probe/)."""
    return _get_bool("DRAIN_HASH_HIGH_PRIORITY", True)


def gc_after_plan() -> bool:
    """One full Python GC pass at the end of a take that built a new take
    plan (utils/tracing.paused_gc)."""
    return _get_bool("GC_AFTER_PLAN", True)


def drain_direct_io() -> bool:
    """O_DIRECT files for the native drain of an async take: no CPU copy into
    the page cache (and none of its cache / memory-bandwidth pressure on the
    training process), at the storage device's write rate."""
    return _get_bool("DRAIN_DIRECT_IO", False)


def async_device_codec() -> str:
    """What an ``async_take`` with ``compression="hsz1"`` does with the device
    state it froze in HBM: ``raw`` (default) drains it uncompressed -- the
    encoder kernels would compete with the training step for the compute
    units (+30 % step time while they run, profiles/overlap_iso/) -- or
    ``same`` encodes it like a blocking take."""
    v = str(_get("ASYNC_DEVICE_CODEC") or "raw").lower()
    return v if v in ("raw", "same") else "raw"


def plan_cache_enabled() -> bool:
    """Reuse a take's plan for the next take of the same device-resident
    tensors (``engine/plan_cache.py``)."""
    return _get_bool("PLAN_CACHE", True)


def native_restore_enabled() -> bool:
    """Reads whose bytes all land in HBM go through ONE native job per device
    (engine/native_restore.py, csrc/hsrestore.hip): pread -> pinned slots ->
    SDMA uploads -> GPU decode / region copy, no Python per blob."""
    return _get_bool("NATIVE_RESTORE", True)


def restore_prewarm_enabled() -> bool:
    """A restore into HBM fills the native job's pinned slots and device
    rings on a thread while it plans its reads (engine/native_restore.py
    prewarm_for)."""
    return _get_bool("RESTORE_PREWARM", True)


def restore_plan_cache_enabled() -> bool:
    """A restore of the same snapshot into the same device tensors reuses the
    previous restore's native plan (engine/restore_cache.py)."""
    return _get_bool("RESTORE_PLAN_CACHE", True)


def native_io_numa_local() -> bool:
    """The native restore's reader threads run on the CPUs of their GPU's
    NUMA node (the process's own mask is left alone): unbound, one rank's
    W = 8 share restored in 42 ms, bound in 29 (profiles/r4/restore_native/)."""
    return _get_bool("NATIVE_IO_NUMA_LOCAL", True)


def get_restore_slot_bytes() -> int:
    """Pinned slot size of the native restore = the largest SDMA upload: 8
    MiB uploads ran the link at 38 GB/s, 32 MiB at 45; a request costs the
    engine a fixed ~0.1 ms (profiles/r4/restore_native/)."""
    return max(1 << 20, _get_int("RESTORE_SLOT_BYTES", 128 << 20))


def get_restore_first_bytes() -> int:
    """The job's first upload is at most this large: the link starts once it
    is read, not once a whole slot is."""
    return max(1 << 20, _get_int("RESTORE_FIRST_BYTES", 16 << 20))


def get_restore_piece_bytes() -> int:
    """Bytes one reader ``pread``s at a time: several readers fill a slot."""
    return max(256 << 10, _get_int("RESTORE_PIECE_BYTES", 4 << 20))


def get_restore_sdma_engine() -> int:
    """SDMA engine of the native restore's uploads: -1 = the one ROCr picks
    per request, -2 = the lowest engine ROCr reports free for host -> device
    copies, k = engine k (when free)."""
    return _get_int("RESTORE_SDMA_ENGINE", -1)


def get_restore_slots() -> int:
    return max(2, _get_int("RESTORE_SLOTS", 6))


def get_restore_readers() -> int:
    """pread threads of the native restore (page-cache copies of ~8 GB/s
    each feed a 57 GB/s link): ``HIPSNAPSHOT_RESTORE_READERS``, else the I/O
    thread count."""
    v = _get("RESTORE_READERS")
    return max(1, int(v)) if v is not None else max(4, min(12, get_io_threads()))


def get_restore_device_budget() -> int:
    """HBM of each of the native restore's two rings (uncached upload
    targets, decode scratch): blobs in flight between their first read and
    the end of their decode / copy kernels."""
    return max(4 << 20, _get_int("RESTORE_DEVICE_BUDGET", 2 << 30))


def get_restore_keep_bytes() -> int:
    """Idle restore blocks kept per pool after a restore: the rings of the
    next restore then allocate nothing."""
    return max(0, _get_int("RESTORE_KEEP_BYTES", (2 << 30) + (256 << 20)))


def get_stage_threads() -> int:
    return _get_int("STAGE_THREADS", 4)


def use_direct_io() -> bool:
    return _get_bool("FS_DIRECT_IO", False)


def use_fsync() -> bool:
    return _get_bool("FS_FSYNC", False)


def async_hbm_staging_enabled() -> bool:
    return _get_bool("ASYNC_HBM_STAGING", True)


def hbm_staging_reserve_bytes() -> int:
    return _get_int("HBM_STAGING_RESERVE_BYTES", 8 * 1024 ** 3)


def hbm_staging_max_bytes() -> int:
    return _get_int("HBM_STAGING_MAX_BYTES", 1 << 62)


def slab_align() -> int:
    return max(1, _get_int("SLAB_ALIGN", 256))


def trust_object_payloads() -> bool:
    return _get_bool("TRUST_OBJECTS", False)


def use_gpu_gather_for_slabs() -> bool:
    return _get_bool("GPU_SLAB_GATHER", True)


@contextmanager
def _override_env_var(name: str, value: Any) -> Generator[None, None, None]:
    key = _PREFIXES[0] + name
    prev = os.environ.get(key)
    os.environ[key] = str(value)
    try:
        yield
    finally:
        if prev is None:
            del os.environ[key]
        else:
            os.environ[key] = prev


@contextmanager
def override_max_chunk_size_bytes(n: int) -> Generator[None, None, None]:
    with _override_env_var(MAX_CHUNK_SIZE, n):
        yield


@contextmanager
def override_max_shard_size_bytes(n: int) -> Generator[None, None, None]:
    with _override_env_var(MAX_SHARD_SIZE, n):
        yield


@contextmanager
def override_slab_size_threshold_bytes(n: int) -> Generator[None, None, None]:
    # NB: the reference overrides the SHARD knob here;
    # we override the slab threshold as the name says.
    with _override_env_var(SLAB_SIZE_THRESHOLD, n):
        yield


@contextmanager
def override_is_batching_disabled(disabled: bool) -> Generator[None, None, None]:
    with _override_env_var(DISABLE_BATCHING, disabled):
        yield


@contextmanager
def override_knob(name: str, value: Any) -> Generator[None, None, None]:
    with _override_env_var(name, value):
        yield
