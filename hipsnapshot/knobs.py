"""Runtime configuration (environment variables + context-manager overrides).

Same knobs and defaults as the reference (`/root/reference/torchsnapshot/knobs.py:21-96`,
`scheduler.py:27-30`): 512 MiB max chunk, 512 MiB max shard piece, 128 MiB slab
threshold, batching on, per-rank memory budget min(0.6*avail/local_ws, 32 GiB).
Every variable is read as ``HIPSNAPSHOT_<NAME>`` first and the reference's
``TORCHSNAPSHOT_<NAME>`` second, so existing job scripts keep working.

The environment surface is ``ENV_KNOBS`` (25 names, documented in
docs/getting_started.md): the reference's five, then

* storage: ``IO_THREADS``, ``COMPRESSION`` (``none`` | ``hsz1`` |
  ``hsz1+host``), ``CHECKSUM``, ``FS_DIRECT_IO``, ``FS_FSYNC``;
* async takes: ``ASYNC_HBM_STAGING``, ``HBM_STAGING_RESERVE_BYTES``,
  ``HBM_STAGING_MAX_BYTES``, ``NATIVE_DRAIN``, ``DRAIN_WRITERS``;
* restore: ``NATIVE_RESTORE``, ``TRUST_OBJECTS``;
* distributed: ``REBALANCE``, ``STATE_DICT_BARRIERS``, ``FORCE_COLLECTIVES``;
* host: ``NUMA_BIND``, ``PINNED_POOL_MAX_BYTES``;
* format: ``FP8_FORMAT`` (``mx`` | ``block`` | ``hadamard32``);
* tracing: ``TIMELINE``, ``ROCTX``.

Everything else that used to be an environment switch -- engine sizing,
copy-engine choice, A/B variants whose measurement concluded -- is a
constant of ``TUNING`` below, each with the record that chose it.  Tests and
probes change them in-process with ``override_knob`` / ``override_tuning``;
they are not read from the environment.
"""

from __future__ import annotations

import functools
import math
import os
import threading
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


_pins = threading.local()  # .env: the knob values an async take's commit thread runs with


def _get(name: str) -> Optional[str]:
    env = getattr(_pins, "env", None)
    src = env if env is not None else os.environ
    for p in _PREFIXES:
        v = src.get(p + name)
        if v is not None:
            return v
    return None


def env_snapshot() -> dict:
    """The ``HIPSNAPSHOT_*`` / ``TORCHSNAPSHOT_*`` variables as they are now."""
    return {k: v for k, v in os.environ.items() if k.startswith(_PREFIXES)}


@contextmanager
def pinned(env: Optional[dict]) -> Generator[None, None, None]:
    """Read knobs from ``env`` (an ``env_snapshot()``) on this thread: an
    ``async_take`` drains with the configuration it was called with, even if
    the environment changes before its drain is done."""
    prev = getattr(_pins, "env", None)
    _pins.env = env
    try:
        yield
    finally:
        _pins.env = prev


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


_quota_seen: list = [None, None]  # (quota function, its value): read once per process


def _cpu_quota() -> Optional[float]:
    """``_cgroup_cpu_quota()``, read once: every take asks for it (I/O thread
    count) and the two cgroup file reads cost ~0.1 ms each."""
    fn = _cgroup_cpu_quota
    if _quota_seen[0] is not fn:
        _quota_seen[:] = [fn, fn()]
    return _quota_seen[1]


def available_cpus() -> int:
    """CPUs this process can actually use: its affinity mask, capped by the
    cgroup's CPU quota.  (A GPU box here shows 256 CPUs in the mask and a
    16-CPU quota in ``cpu.max``: every thread above the quota only makes the
    whole group wait for the next period.)"""
    try:
        cpus = len(os.sched_getaffinity(0))
    except (AttributeError, OSError):  # pragma: no cover - non-Linux
        cpus = os.cpu_count() or 16
    quota = _cpu_quota()
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


ENV_KNOBS = (
    MAX_CHUNK_SIZE, MAX_SHARD_SIZE, SLAB_SIZE_THRESHOLD, DISABLE_BATCHING, MEMORY_BUDGET,
    "IO_THREADS", "COMPRESSION", "CHECKSUM", "FS_DIRECT_IO", "FS_FSYNC",
    "ASYNC_HBM_STAGING", "HBM_STAGING_RESERVE_BYTES", "HBM_STAGING_MAX_BYTES", "NATIVE_DRAIN",
    "DRAIN_WRITERS", "NATIVE_RESTORE", "TRUST_OBJECTS", "REBALANCE", "STATE_DICT_BARRIERS",
    "FORCE_COLLECTIVES", "NUMA_BIND", "PINNED_POOL_MAX_BYTES", "FP8_FORMAT", "TIMELINE", "ROCTX",
)


class _Tuning:
    """Engine constants (not read from the environment).  Attribute =
    value; ``override_knob("RESTORE_SLOTS", 3)`` (upper-case name) or
    ``override_tuning(restore_slots=3)`` change one for a test."""

    # -- take / staging --------------------------------------------------------
    read_inflight = 8          # whole-blob reads in flight (Python read pipeline)
    io_read_split_bytes = 8 << 20   # reads > 1.5x this are split across I/O workers
    stage_threads = 4          # concurrent staging jobs
    # device -> pinned copies on the SDMA engines (falls back to blit when ROCr
    # reports none): same PCIe-bound rate, no CU time, +4 % on the Llama-3-8B
    # save (profiles/dma/)
    d2h_engine = "sdma"
    # a restore's HSZ1 uploads through SDMA into uncached blocks: hipMemcpyAsync
    # calls block for milliseconds when several threads upload
    # (profiles/r4/restore_trace/)
    h2d_engine = "sdma"
    async_dma = True           # staging workers submit the copy and move on
    dma_inflight = 8           # SDMA device -> host copies in flight per device
    serial_encode = True       # staging threads take turns on a device's HSZ1 encodes
    thread_staging = True      # long-running staging threads pull requests
    # the first blob is staged before the other workers start (rank share
    # A/B: 28.5 vs 28.8 ms, scripts/gpu_r5_z.sh; the first DMA starts sooner)
    stage_head_alone = True
    # checksum launch width: a full-chip hash slows the concurrent SDMA copies
    # (scripts/probes/hash_probe.py); blobs only need hashing at PCIe rate
    hash_grid = 64
    gpu_slab_gather = True
    slab_align = 256
    gc_after_plan = True       # one full GC pass after a take that built a plan
    plan_cache = True          # reuse a take's plan (engine/plan_cache.py)
    # async takes drain the frozen device state raw: the encoder on the CUs
    # beside a training step cost +30 % step time (profiles/overlap_iso/)
    async_device_codec = "raw"
    # the async-take arena is kept for the next take while the device keeps
    # HBM_STAGING_RESERVE_BYTES of headroom (engine/memory.py);
    # release_hbm_arena() frees it on request
    hbm_arena_keep = True
    # idle pinned pool blocks are unregistered after this long without a
    # snapshot operation (0: never)
    pinned_idle_trim_s = 300.0
    # -- native drain (csrc/hsdrain.cpp) -----------------------------------------
    # 16 slots of 64 MiB drain the 16 GB Llama-3-8B arena at the PCIe rate
    # (profiles/r3/s2/drain_sizing/)
    drain_slot_bytes = 64 << 20
    drain_slots = 16
    drain_nice = 10            # the drain's threads yield a shared core to the trainer
    drain_avoid_caller_core = "core"   # "core" | "l3" | "" (utils/affinity.py)
    drain_hash_high_priority = True    # profiles/r3/drain_probe/
    # -- restore (csrc/hsrestore.cpp) -------------------------------------------------
    # HSZ1 blobs > 2x this are read as head + rest.  (Reads go in plan order:
    # "a small lead read, then largest first" measured 65.1 / 68.2 GB/s vs
    # 70.7 / 72.8, profiles/timeline_r2/read_order.txt)
    read_head_bytes = 16 << 20
    restore_prewarm = True
    restore_plan_cache = True
    native_io_numa_local = True   # readers on their GPU's NUMA node: 42 -> 29 ms
    # 8 MiB uploads ran the link at 38 GB/s, 32 MiB at 45; a request costs the
    # engine ~0.1 ms (profiles/r4/restore_native/)
    restore_slot_bytes = 128 << 20
    restore_first_bytes = 16 << 20
    restore_piece_bytes = 4 << 20
    restore_sdma_engine = -1
    restore_slots = 6
    restore_readers = 0        # 0: max(4, min(12, I/O threads))
    restore_device_budget = 2 << 30
    # idle restore blocks kept per pool after a restore (HBM outside torch's
    # allocator): the two 2 GiB rings, so the next restore does not allocate.
    # The blocks are VMM mappings on never-reused address ranges, so freeing
    # them is safe at any time (the round-5 wrong bytes after trims were
    # stale translations of reused ranges: profiles/r6/trim/); the memory
    # policy trims them to 0 when the trainer's headroom runs short
    # (engine/memory.py), ``release_restore_memory()`` on request.
    restore_keep_bytes = (2 << 30) + (256 << 20)
    # -- distributed -------------------------------------------------------------------
    # a DTensor box replicated R ways (HSDP, DTensor DDP) at least this large
    # is written as R row ranges, one per replica; smaller boxes go whole to
    # one replica chosen by a hash of their position (io/sharded.py)
    replica_split_min_bytes = 1 << 20
    # replicated (DDP) tensors are chunked so each rank's share is >= this
    # many partitioner units (parallel/partitioner.py replicated_chunk_bytes)
    replicated_units_per_rank = 16
    rebalance_host = False     # let the rebalancer move host blobs too (gloo tests)
    rebalance_min_gain = 0.1
    # -- UVM ------------------------------------------------------------------------------
    uvm_assume_host = None     # None: unless the device runs with XNACK on
    # async takes copy host-resident UVM tables with CPU threads on the pages'
    # node while the trainer's stream waits on a gate (engine/uvm_capture.py):
    # 160-196 GB/s vs 55 GB/s for the HBM freeze over PCIe (profiles/r6/uvmcap/)
    uvm_async_capture = True
    uvm_capture_threads = 32
    # the drain writes a captured table as soon as it is copied (True) or
    # once the whole capture released the trainer's stream (False)
    uvm_capture_overlap = False


TUNING = _Tuning()


def _tuned(name: str):
    return getattr(TUNING, name)


def get_compression() -> str:
    """``none`` | ``hsz1`` (GPU-resident floating blobs) | ``hsz1+host``
    (host tensors too, with the C++ codec: worth it when storage, not host
    memory bandwidth, is the bottleneck)."""
    return str(_get("COMPRESSION") or "none").strip().lower()


def compress_host_tensors() -> bool:
    return get_compression().endswith("+host")


def get_read_inflight() -> int:
    return max(1, int(_tuned("read_inflight")))


def get_io_read_split_bytes() -> int:
    return int(_tuned("io_read_split_bytes"))


def get_d2h_engine() -> str:
    """Engine for bulk device -> pinned-host copies (``TUNING.d2h_engine``):
    ``blit`` = hipMemcpyAsync, ``sdma`` = the DMA engines (csrc/hsdma.hip)."""
    v = str(_tuned("d2h_engine")).lower()
    if v not in ("blit", "sdma"):
        raise ValueError(f"d2h engine must be blit or sdma, not {v!r}")
    return v


def get_h2d_engine() -> str:
    v = str(_tuned("h2d_engine")).lower()
    if v not in ("hip", "sdma"):
        raise ValueError(f"h2d engine must be hip or sdma, not {v!r}")
    return v


def async_dma() -> bool:
    return bool(_tuned("async_dma"))


def get_dma_inflight() -> int:
    return max(1, int(_tuned("dma_inflight")))


def serial_encode() -> bool:
    return bool(_tuned("serial_encode"))


def thread_staging_enabled() -> bool:
    return bool(_tuned("thread_staging"))


def checksum_enabled() -> bool:
    """Record an hs64 checksum of every blob a take writes
    (``.snapshot_checksums/<rank>``, ops/checksum.py); ``Snapshot.verify``
    and ``restore(verify=True)`` check them."""
    return _get_bool("CHECKSUM", True)


def get_hash_grid() -> int:
    return int(_tuned("hash_grid"))


def get_read_head_bytes() -> int:
    return max(0, int(_tuned("read_head_bytes")))


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


def force_collectives() -> bool:
    """Issue every metadata collective (and the async commit's store barrier)
    even in a one-rank process group, as the reference does
    (`pg_wrapper.py:42-56`); by default a one-rank group skips them."""
    return _get_bool("FORCE_COLLECTIVES", False)


def rebalance_enabled() -> bool:
    """Move whole blobs from heavily to lightly loaded ranks over xGMI before
    a blocking take stages (parallel/rebalance.py).  Off by default."""
    return _get_bool("REBALANCE", False)


def rebalance_host() -> bool:
    return bool(_tuned("rebalance_host"))


def rebalance_min_gain() -> float:
    return float(_tuned("rebalance_min_gain"))


def hbm_arena_keep() -> bool:
    return bool(_tuned("hbm_arena_keep"))


def native_drain_enabled() -> bool:
    """Drain an async take's raw frozen blobs to the local FS in native
    threads (engine/native_drain.py, csrc/hsdrain.cpp)."""
    return _get_bool("NATIVE_DRAIN", True)


def get_drain_slot_bytes() -> int:
    return max(1 << 20, int(_tuned("drain_slot_bytes")))


def get_drain_slots() -> int:
    """Pinned slots the native drain cycles through (slots x slot bytes of
    pinned host memory while a drain runs, outside the memory budget)."""
    return max(2, int(_tuned("drain_slots")))


def get_drain_writers() -> int:
    """Writer threads of an async take's native drain while training goes
    on: 3 (at most half the rank's CPU share, at least 2).  With 8 writers a
    launch-bound seq-512 Llama-3-8B step ran 5-9 % slower while a 48 GB drain
    was in flight, with 3 writers 2-5 % (profiles/r4/overlap_ab_writers/)."""
    share = available_cpus() // max(_local_ranks_hint[0], 1)
    return max(1, _get_int("DRAIN_WRITERS", min(3, get_io_threads(), max(2, share // 2))))


def get_drain_boost_writers() -> int:
    """Writer threads of a native drain once its caller blocks on it
    (``PendingSnapshot.wait``): the extra ones are parked until then.  Nothing
    trains while the caller waits, so they may use the rank's whole CPU share
    (not half of it): the ZeRO-3 OPT-shape save (40 GB) ran at 24 GB/s with
    8 writers and 34-49 GB/s with 16 (profiles/r5/zero3_ab/)."""
    share = available_cpus() // max(_local_ranks_hint[0], 1)
    return max(get_drain_writers(), min(16, get_io_threads(), max(2, share)))


def get_drain_nice() -> int:
    return max(0, min(19, int(_tuned("drain_nice"))))


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
    DRAM (blocking takes write them in place) -- unless the device runs with
    XNACK on (``device_xnack_enabled``), where pages migrate to the GPU that
    touches them.  Measured: a never-placed table reads at 57 GB/s from a
    kernel (PCIe), 3.9 TB/s once prefetched to the GPU (profiles/r3/uvm/)."""
    v = _tuned("uvm_assume_host")
    if v is not None:
        return bool(v)
    return not device_xnack_enabled()


def drain_avoid_caller_core() -> str:
    v = str(_tuned("drain_avoid_caller_core") or "").strip().lower()
    return "" if v in ("0", "false", "no", "off", "") else ("l3" if v == "l3" else "core")


def drain_hash_high_priority() -> bool:
    return bool(_tuned("drain_hash_high_priority"))


def gc_after_plan() -> bool:
    return bool(_tuned("gc_after_plan"))


def async_device_codec() -> str:
    v = str(_tuned("async_device_codec")).lower()
    return v if v in ("raw", "same") else "raw"


def plan_cache_enabled() -> bool:
    return bool(_tuned("plan_cache"))


def native_restore_enabled() -> bool:
    """Reads whose bytes all land in HBM go through ONE native job per device
    (engine/native_restore.py, csrc/hsrestore.cpp): pread -> pinned slots ->
    SDMA uploads -> GPU decode / region copy, no Python per blob."""
    return _get_bool("NATIVE_RESTORE", True)


def restore_prewarm_enabled() -> bool:
    return bool(_tuned("restore_prewarm"))


def restore_plan_cache_enabled() -> bool:
    return bool(_tuned("restore_plan_cache"))


def native_io_numa_local() -> bool:
    return bool(_tuned("native_io_numa_local"))


def get_restore_slot_bytes() -> int:
    return max(1 << 20, int(_tuned("restore_slot_bytes")))


def get_restore_first_bytes() -> int:
    return max(1 << 20, int(_tuned("restore_first_bytes")))


def get_restore_piece_bytes() -> int:
    return max(256 << 10, int(_tuned("restore_piece_bytes")))


def get_restore_sdma_engine() -> int:
    return int(_tuned("restore_sdma_engine"))


def get_restore_slots() -> int:
    return max(2, int(_tuned("restore_slots")))


def get_restore_readers() -> int:
    """pread threads of the native restore (page-cache copies of ~8 GB/s
    each feed a 57 GB/s link)."""
    v = int(_tuned("restore_readers"))
    return max(1, v) if v > 0 else max(4, min(12, get_io_threads()))


def get_restore_device_budget() -> int:
    """HBM of each of the native restore's two rings (uncached upload
    targets, decode scratch)."""
    return max(4 << 20, int(_tuned("restore_device_budget")))


def get_restore_keep_bytes() -> int:
    return max(0, int(_tuned("restore_keep_bytes")))


def get_stage_threads() -> int:
    return int(_tuned("stage_threads"))


def use_direct_io() -> bool:
    """O_DIRECT for blob files (take writes and the native drain): no CPU copy
    into the page cache, at the storage device's write rate."""
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
    return max(1, int(_tuned("slab_align")))


def trust_object_payloads() -> bool:
    return _get_bool("TRUST_OBJECTS", False)


def use_gpu_gather_for_slabs() -> bool:
    return bool(_tuned("gpu_slab_gather"))


def pinned_pool_max_bytes() -> int:
    """Cap of the pinned host pool (bytes kept registered across takes)
    until the first snapshot operation; from then on, unless this knob is
    set, the rank's host memory budget (engine/memory.py pinned_cap_bytes)."""
    return _get_int("PINNED_POOL_MAX_BYTES", 64 << 30)


def fp8_format() -> str:
    """Layout of ``quantize=`` blobs: ``mx`` (default: e4m3fn + E8M0 scale
    per 32 elements), ``block`` (fp32 scale per 128), ``hadamard32`` (32-wide
    Hadamard rotation on the matrix cores, then fp32-scale blocks)."""
    v = str(_get("FP8_FORMAT") or "mx").strip().lower()
    return v if v in ("mx", "block", "hadamard32") else "mx"


def plan_settings() -> tuple:
    """The configuration a take plan or a restore plan depends on (the plan
    caches' key: engine/plan_cache.py, engine/restore_cache.py) -- values,
    not every environment variable: a change of tracing or I/O thread count
    keeps the plans."""
    return (get_max_chunk_size_bytes(), get_max_shard_size_bytes(),
            get_slab_size_threshold_bytes(), is_batching_disabled(), get_compression(),
            checksum_enabled(), async_hbm_staging_enabled(), hbm_staging_reserve_bytes(),
            hbm_staging_max_bytes(), native_drain_enabled(), native_restore_enabled(),
            use_direct_io(), fp8_format(), tuple(sorted(vars(TUNING).items())))


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
def override_tuning(**values: Any) -> Generator[None, None, None]:
    old = {k: vars(TUNING).get(k, _MISSING) for k in values}
    for k, v in values.items():
        if not hasattr(_Tuning, k):
            raise AttributeError(f"no tuning constant {k!r}")
        setattr(TUNING, k, v)
    try:
        yield
    finally:
        for k, v in old.items():
            if v is _MISSING:
                delattr(TUNING, k)
            else:
                setattr(TUNING, k, v)


_MISSING = object()


@contextmanager
def override_knob(name: str, value: Any) -> Generator[None, None, None]:
    """An environment knob (``ENV_KNOBS``) or, by its upper-case name, a
    ``TUNING`` constant."""
    if name in ENV_KNOBS:
        with _override_env_var(name, value):
            yield
        return
    attr = name.lower()
    if not hasattr(_Tuning, attr):
        raise KeyError(f"unknown knob {name!r}")
    cur = getattr(TUNING, attr)
    if isinstance(cur, bool) or (cur is None and str(value) in ("0", "1")):
        value = str(value).strip().lower() in ("1", "true", "yes", "on")
    elif isinstance(cur, int):
        value = int(value)
    elif isinstance(cur, float):
        value = float(value)
    with override_tuning(**{attr: value}):
        yield
