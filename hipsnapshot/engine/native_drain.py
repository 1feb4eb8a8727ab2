"""Native drain of an async take's frozen HBM arena to the local FS.

``DeferredIOWork`` (engine/scheduler.py) hands every eligible deferred write
to ONE ``native.NativeDrain`` call (csrc/hsdrain.cpp): SDMA copies arena ->
pinned slots -> ``pwrite``, per-blob hs64 hashes on the GPU, optional
fdatasync -- in native threads, so the training loop keeps the GIL and the
compute units while a checkpoint drains.  Eligible: a raw blob (no HSZ1
codec, buffer-protocol serializer) whose bytes sit contiguously in the arena
(``frozen_region``, engine/hbm_staging.py), written by the FS plugin
(buffered, or O_DIRECT straight from the pinned slots).  Everything else drains through the Python pipeline as before.

Reference counterpart: `/root/reference/torchsnapshot/snapshot.py:891-933`
(the commit thread draining pending storage I/O) and
`/root/reference/torchsnapshot/scheduler.py:194-217`.
"""

from __future__ import annotations

import logging
import os
import threading
import time
from typing import Dict, List, Tuple

from .. import knobs
from ..io_types import StoragePlugin, WriteReq
from ..ops import checksum, native
from ..utils.tracing import timeline

logger = logging.getLogger(__name__)


last_stats: Dict[str, float] = {}  # the last drain's phase seconds (NativeDrain.STATS)

class Booster:
    """Shared by one async take's drain and its ``PendingSnapshot``: once the
    caller blocks in ``wait()`` nothing trains beside the drain any more, so
    its parked writers start (``NativeDrain.boost``)."""

    def __init__(self) -> None:
        self._lock = threading.Lock()
        self._jobs: List = []
        self.boosted = False

    def boost(self) -> None:
        with self._lock:
            self.boosted = True
            jobs = list(self._jobs)
        for job in jobs:
            job.boost()

    def attach(self, job) -> None:
        with self._lock:
            self._jobs.append(job)
            now = self.boosted
        if now:
            job.boost()

    def detach(self, job) -> None:
        with self._lock:
            self._jobs.remove(job)


def _root(storage: StoragePlugin):
    fn = getattr(storage, "native_drain_root", None)
    return fn() if fn is not None else None


def eligible(wr: WriteReq, storage: StoragePlugin) -> bool:
    from ..format.serialization import SER
    from ..io.batcher import GPUBatchedBufferStager
    from ..io.tensor import TensorBufferStager

    st = wr.buffer_stager
    if getattr(st, "frozen_region", None) is None or getattr(st, "codec", None) is not None:
        return False
    if isinstance(st, TensorBufferStager):
        if st.entry.serializer != SER.BUFFER_PROTOCOL or \
                st._tensor_prepare_func is not None:
            return False
    elif not isinstance(st, GPUBatchedBufferStager):
        return False
    return _root(storage) is not None


def split(reqs: List[WriteReq], storage: StoragePlugin) -> Tuple[List[WriteReq], List[WriteReq]]:
    """(native, python) parts of an async take's deferred writes."""
    if not knobs.native_drain_enabled() or not native.gpu_available() or _root(storage) is None:
        return [], list(reqs)
    nat, py = [], []
    for wr in reqs:
        (nat if eligible(wr, storage) else py).append(wr)
    return nat, py


def _run(dev: int, wrs: List[WriteReq], blobs, fsync: bool, want_sums: bool, direct: bool,
         booster: "Booster" = None):
    """One device's drain in this process's native threads.  Returns (hs64
    partial sums, bytes written, stats, "in_process")."""
    from ..utils.affinity import drain_thread_mask, threads_with_mask

    args = (knobs.get_drain_slot_bytes(), knobs.get_drain_slots(), knobs.get_drain_writers())
    parked = max(0, knobs.get_drain_boost_writers() - args[2])
    # the drain's threads inherit a mask without the training thread's core
    # (or L3 domain), on the GPU's NUMA node when that leaves enough CPUs
    with threads_with_mask(drain_thread_mask(dev, knobs.drain_avoid_caller_core(),
                                             knobs.native_io_numa_local())):
        job = native.NativeDrain(dev, blobs, *args, fsync, want_sums, knobs.get_hash_grid(),
                                 knobs.get_drain_nice(), direct, knobs.drain_hash_high_priority(),
                                 parked_writers=parked)
    if booster is not None:
        booster.attach(job)
    try:
        partial, written = job.wait()
    finally:
        if booster is not None:
            booster.detach(job)
    return partial, written, job.stats, "in_process"


def drain(reqs: List[WriteReq], storage: StoragePlugin, booster: "Booster" = None
          ) -> Tuple[Dict[str, int], int]:
    """Write every request's frozen region to its file; returns ({blob path:
    hs64}, bytes written).  Blocks (call it off the event loop)."""
    root, fsync, direct = _root(storage)
    by_dev: Dict[int, List[WriteReq]] = {}
    for wr in reqs:
        arena = wr.buffer_stager.frozen_region[0]
        by_dev.setdefault(arena.device.index or 0, []).append(wr)
    sums: Dict[str, int] = {}
    total = 0
    want_sums = knobs.checksum_enabled()
    for dev, wrs in by_dev.items():
        t0 = time.perf_counter()
        # the freeze copy must have landed before the engines read the arena
        for ev in {id(wr.buffer_stager.frozen_event): wr.buffer_stager.frozen_event
                   for wr in wrs}.values():
            ev.synchronize()
        blobs = []
        for wr in wrs:
            arena, off, nbytes = wr.buffer_stager.frozen_region
            blobs.append((arena.data_ptr() + off, nbytes, os.path.join(root, wr.path)))
        partial, written, stats, where = _run(dev, wrs, blobs, fsync, want_sums, direct, booster)
        total += written
        if want_sums:
            for wr, (_p, n, _path), s in zip(wrs, blobs, partial):
                sums[wr.path] = checksum.finish(s, n)
        timeline.add("native_drain", "io", t0, time.perf_counter(), n=len(wrs), bytes=written,
                     where=where, **stats)
        last_stats.clear()
        last_stats.update(stats, blobs=len(wrs), bytes=written, where=where)
    return sums, total
