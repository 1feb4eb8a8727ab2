"""Native restore of local-FS blobs whose bytes all land in HBM.

``execute_read_reqs`` (engine/scheduler.py) hands every eligible read to ONE
``native.NativeRestore`` job per device (csrc/hsrestore.cpp): reader threads
``pread`` the blobs from the page cache into pinned slots and queue their
SDMA uploads back to back, the completion thread launches each blob's HSZ1
decode and ONE region-copy kernel as soon as its bytes have landed -- no
Python (and no GIL hand-over) per blob.  Eligible: a read from the FS plugin
whose consumer exposes ``device_regions`` for all of its bytes (plain tensors,
DTensor / ShardedTensor pieces, batched slabs of them) into non-managed HBM
with casts the copy kernel does, stored raw or as an HSZ1 blob read (mostly)
whole.  Everything else keeps the Python pipeline.

The plan for a job -- destinations, descriptor tables with source offsets
relative to the uploaded / decoded bytes -- is built here on the caller's
thread; the descriptors' fast paths depend on the alignment of those offsets
only (upload and decode blocks are 2 MiB aligned).

Reference counterpart: `/root/reference/torchsnapshot/scheduler.py:384-444`
(read pipeline) and `/root/reference/torchsnapshot/io_preparers/tensor.py:294-346`.
"""

from __future__ import annotations

import logging
import os
import threading
import time
from collections import defaultdict
from typing import Dict, List, Optional, Tuple

import numpy as np

from .. import knobs
from ..io_types import ReadReq, StoragePlugin
from ..ops import native
from ..utils.tracing import timeline

logger = logging.getLogger(__name__)

last_stats: Dict[str, float] = {}  # the last job's phase seconds (NativeRestore.STATS)

_RAW, _HSZ = 0, 1


def _root(storage: StoragePlugin) -> Optional[str]:
    fn = getattr(storage, "native_read_root", None)
    return fn() if fn is not None else None


def _regions(consumer) -> Optional[list]:
    """Device regions covering every byte the consumer needs, or None."""
    from ..io.batcher import BatchedBufferConsumer

    if isinstance(consumer, BatchedBufferConsumer):
        if consumer._other or not consumer._gpu:
            return None
        out = []
        for _rng, _c, regions in consumer._gpu:
            out.extend(regions)
        return out
    fn = getattr(consumer, "device_regions", None)
    if fn is None or getattr(consumer, "_direct", False):
        return None
    return fn(0) or None


def _producers(consumer) -> List[int]:
    from ..io.batcher import BatchedBufferConsumer

    cs = [c for _r, c, _g in consumer._gpu] if isinstance(consumer, BatchedBufferConsumer) \
        else [consumer]
    out = []
    for c in cs:
        p = getattr(c, "producer", None)
        if p is not None:
            out.append(int(p))
    return out


def _plan_one(rr: ReadReq, root: str, slot_bytes: int):
    """(device, item tuple, producers) for ``NativeRestore``, or None."""
    from ..ops import codec as hsz
    from . import staging
    from .scheduler import _expected_read_bytes

    regions = _regions(rr.buffer_consumer)
    if not regions:
        return None
    devs = set()
    for src_dtype, _shape, _off, _nar, dst in regions:
        if not dst.is_cuda or staging._is_managed(dst) or dst.dim() > native.MAX_DIMS \
                or not native.can_cast_on_device(src_dtype, dst.dtype):
            return None
        devs.add(staging.device_of(dst))
    if len(devs) != 1:
        return None
    dev = devs.pop()
    path = os.path.join(root, rr.path)
    if rr.codec is None:
        n = _expected_read_bytes(rr)
        if not n:
            return None
        lo = rr.byte_range[0] if rr.byte_range is not None else 0
        codec, logical, base, direct = _RAW, n, 0, 0
        file_lo, nbytes = lo, n
    else:
        info = rr.codec
        if info.get("name", hsz.CODEC_NAME) != hsz.CODEC_NAME:
            return None
        logical = int(info["blob_bytes"])
        lo, hi = rr.byte_range if rr.byte_range is not None else (0, logical)
        nf = hsz.n_frames_for(logical, int(info["frame_bytes"]))
        # the whole blob is read and decoded: not for a small part of it
        if logical <= 0 or 2 * (hi - lo) < logical or hsz.payload_start(nf) > slot_bytes:
            return None
        try:
            nbytes = os.path.getsize(path)
        except OSError:
            return None
        codec, file_lo, base, direct = _HSZ, 0, lo, 0
        if lo == 0 and hi == logical and len(regions) == 1:
            src_dtype, src_shape, off, narrows, dst = regions[0]
            whole = off == 0 and all(st == 0 and ln == int(src_shape[d])
                                     for d, st, ln in (narrows or ()))
            if (whole and dst.dtype == src_dtype and dst.is_contiguous()
                    and dst.numel() * dst.element_size() == logical
                    and dst.data_ptr() % 16 == 0):
                direct = dst.data_ptr()
    descs = np.zeros(0, dtype=native.COPY_DESC_DTYPE)
    if not direct:
        batch = native.CopyBatch()
        for src_dtype, src_shape, off, narrows, dst in regions:
            es = staging._elem_size(src_dtype)
            if dst.dtype == src_dtype and dst.is_contiguous() and \
                    all(st == 0 and ln == int(src_shape[d]) for d, st, ln in (narrows or ())):
                # the common slab member: one contiguous byte range
                batch.add_bytes(base + off, dst.data_ptr(), dst.numel() * es)
                continue
            shape = [int(z) for z in src_shape]
            strides = staging._contig_strides(shape)
            # source offset within the uploaded (raw) / decoded (HSZ1) bytes
            ptr = base + off
            if narrows:
                for d, st, ln in narrows:
                    ptr += st * strides[d] * es
                    shape[d] = ln
            batch.add(ptr, src_dtype, strides, dst.data_ptr(), dst.dtype, dst.stride(), shape, es)
        descs = batch.pack()
    item = (path, file_lo, nbytes, codec, logical, direct, 0, descs)
    return dev, item, _producers(rr.buffer_consumer)


def sizing(budget: Optional[int]) -> Tuple[int, int, int]:
    """(slot bytes, first-span bytes, slots) of a job: the knobs, shrunk so
    the pinned slots stay within half of the host ``budget`` (a
    ``read_object`` with a memory budget must not pin 768 MiB)."""
    slot, first, n = (knobs.get_restore_slot_bytes(), knobs.get_restore_first_bytes(),
                      knobs.get_restore_slots())
    if budget:
        cap = max(2 << 20, int(budget) // 2)
        # the knob's slot count, down to 4 MiB slots: the same pinned bytes in
        # a deeper pipeline (2 slots of 25 MiB under a 100 MB budget kept one
        # read and one DMA in flight: 37-40 GB/s, where unbudgeted reads run
        # at 52 GB/s, profiles/r6/benches/)
        n = max(2, min(n, cap // (4 << 20)))
        slot = max(1 << 20, min(slot, cap // n))
    return slot, min(first, slot), n


def pinned_bytes(budget: Optional[int] = None) -> int:
    """Pinned host memory one job holds: its slots and its copy-table stage."""
    slot, _first, n = sizing(budget)
    return n * slot + table_bytes(slot)


def split(read_reqs: List[ReadReq], storage: StoragePlugin, budget: Optional[int] = None
          ) -> Tuple[Dict[int, list], List[ReadReq]]:
    """({device: [(read req, item)], ...} for native jobs, the Python part);
    ``budget``: the read's host memory budget (``sizing``)."""
    if not read_reqs or not knobs.native_restore_enabled() or _root(storage) is None \
            or not native.gpu_available():
        return {}, list(read_reqs)
    root = _root(storage)
    # an HSZ1 blob's header and frame table must fit its first upload span
    slot_bytes = sizing(budget)[1]
    jobs: Dict[int, list] = defaultdict(list)
    py: List[ReadReq] = []
    t0 = time.perf_counter()
    for rr in read_reqs:
        got = _plan_one(rr, root, slot_bytes)
        if got is None:
            py.append(rr)
        else:
            jobs[got[0]].append((rr, got[1], got[2]))
    timeline.add("native_restore_plan", "phase", t0, time.perf_counter(), n=len(read_reqs),
                 native=sum(len(v) for v in jobs.values()))
    return dict(jobs), py


_prewarm: Optional[threading.Thread] = None
_prewarm_lock = threading.Lock()


def table_bytes(slot: int) -> int:
    """The job's copy-table ring size (csrc/hsrestore.cpp kTables)."""
    return min(32 << 20, max(1 << 20, slot // 4))


def prewarm_async(dev: int, dest_bytes: int, compressed: bool,
                  budget: Optional[int] = None) -> None:
    """Start filling the restore pools for a job of ~``dest_bytes`` bytes
    into device ``dev`` on a thread, beside the caller's read planning (a
    process's first restore paid ~12 ms of pinned / uncached allocation and
    first-SDMA setup inside the job).  The device rings are warmed only when
    the job will use a whole budget's worth (smaller rings are cheap and a
    budget-sized block would not be reused for them); ``run`` joins it."""
    global _prewarm
    if dest_bytes <= 0 or not knobs.native_restore_enabled() or \
            not knobs.restore_prewarm_enabled() or not native.gpu_available():
        return
    slot, _first, nslots = sizing(budget)
    dev_budget = knobs.get_restore_device_budget()
    ring = dev_budget if dest_bytes >= 2 * dev_budget else 0
    # the job takes 2 slots at its start and allocates the rest on a helper
    # thread while its readers run: only those 2 are on its critical path
    n = 2
    with _prewarm_lock:
        if _prewarm is not None:
            return

        def work():
            t0 = time.perf_counter()
            try:  # best effort: the job allocates whatever is missing itself
                rc = native.restore_prewarm(dev, ring, ring if compressed else 0, slot, n,
                                            table_bytes(slot))
            except Exception as e:  # pragma: no cover - no GPU library
                logger.debug("restore prewarm skipped: %s", e)
                return
            timeline.add("native_restore_prewarm", "phase", t0, time.perf_counter(), rc=rc,
                         ring=ring, slots=n)

        _prewarm = threading.Thread(target=work, name="hs-restore-prewarm", daemon=True)
        _prewarm.start()


def _has_codec(entry, depth: int = 0) -> bool:
    if getattr(entry, "codec", None):
        return True
    if depth < 3:
        for attr in ("shards", "chunks"):
            for sub in getattr(entry, attr, None) or ():
                if _has_codec(getattr(sub, "tensor", sub), depth + 1):
                    return True
    return False


def prewarm_for(leaves, entries, budget: Optional[int] = None,
                storage: Optional[StoragePlugin] = None) -> None:
    """``prewarm_async`` for a restore into ``leaves`` (the stateful's
    tensors / DTensors) of manifest ``entries``: the device and bytes are
    those of the HBM destinations.  Nothing is warmed when ``storage`` is
    not one a native job reads (S3, GCS, memory): its reads take the Python
    pipeline and the pools would only hold idle HBM."""
    if storage is not None and _root(storage) is None:
        return
    try:
        from torch.distributed.tensor import DTensor
    except Exception:  # pragma: no cover
        DTensor = ()  # type: ignore[assignment]
    per_dev: Dict[int, int] = defaultdict(int)
    import torch

    for v in leaves:
        if DTensor and isinstance(v, DTensor):
            t = v._local_tensor
        elif type(v) is torch.Tensor or type(v) is torch.nn.Parameter:
            t = v
        else:  # ShardedTensor & co: not counted (an estimate only)
            continue
        if t.is_cuda:
            per_dev[t.device.index or 0] += t.numel() * t.element_size()
    if not per_dev:
        return
    dev, nbytes = max(per_dev.items(), key=lambda kv: kv[1])
    prewarm_async(dev, nbytes, any(_has_codec(e) for e in entries), budget)


def release_restore_memory() -> int:
    """Free every idle block of the native restore's device pools (the
    upload / scratch rings a restore keeps for the next one, up to 2 x
    2.25 GiB of HBM outside torch's caching allocator).  Call it when no
    restore is running on this GPU -- from any process (see
    ``knobs.TUNING.restore_keep_bytes``).  Returns the bytes freed."""
    _join_prewarm()
    if not native.gpu_available():
        return 0
    import torch

    freed = 0
    for dev in range(torch.cuda.device_count()):
        freed += native.restore_trim(dev, 0)
    return freed


def join_prewarm() -> None:
    """Wait for a pending prewarm (a restore that ran no native job)."""
    _join_prewarm()


def _join_prewarm() -> None:
    global _prewarm
    with _prewarm_lock:
        t, _prewarm = _prewarm, None
    if t is not None:
        t.join()


def _hash_plan(entries, verifier) -> Optional[List[bool]]:
    """Which items the job hashes (``restore(verify=True)``): those that read
    a whole blob (HSZ1 items always do); the blobs of the others are noted
    for a full read at the end (engine/blob_verify.py)."""
    if verifier is None:
        return None
    out = []
    for rr, item, _p in entries:
        whole = item[3] == _HSZ or (item[1] == 0 and _file_size(item[0]) == item[2])
        if not whole:
            verifier.note_partial(rr.path)
        out.append(whole)
    return out


def _file_size(path: str) -> Optional[int]:
    try:
        return os.path.getsize(path)
    except OSError:
        return None


def run(jobs: Dict[int, list], budget: Optional[int] = None, verifier=None) -> int:
    """Run the planned jobs (blocking; call off the event loop); returns the
    logical bytes restored.  Raises ``CorruptBlobError`` for rejected frames
    (and, with a ``verifier``, for blobs whose stored bytes do not match the
    take's checksums), ``OSError`` / ``HipError`` for other failures."""
    from ..ops import checksum

    _join_prewarm()
    total = 0
    slot, first, nslots = sizing(budget)
    for dev, entries in jobs.items():
        t0 = time.perf_counter()
        items = [e[1] for e in entries]
        hashed = _hash_plan(entries, verifier)
        prods = sorted({p for e in entries for p in e[2]})
        from ..utils.affinity import gpu_node_mask, threads_with_mask

        # readers (and the pinned slots they fill) on the GPU's NUMA node
        mask = gpu_node_mask(dev) if knobs.native_io_numa_local() else None
        t1 = time.perf_counter()
        with threads_with_mask(mask):
            job = native.NativeRestore(dev, items, prods, slot, knobs.get_restore_piece_bytes(),
                                       nslots, knobs.get_restore_readers(),
                                       knobs.get_restore_device_budget(),
                                       knobs.get_restore_sdma_engine(), first,
                                       hash_items=hashed, hash_grid=knobs.get_hash_grid())
        t2 = time.perf_counter()
        rc, item, msg = job.wait()
        t3 = time.perf_counter()
        bad = job.corrupt_items()
        native.restore_trim(dev, knobs.get_restore_keep_bytes())
        t4 = time.perf_counter()
        # caller-side seconds: mask / start / wait / error words + trim
        job.stats.update(py_mask=round(t1 - t0, 5), py_start=round(t2 - t1, 5),
                         py_wait=round(t3 - t2, 5), py_after=round(t4 - t3, 5))
        nbytes = sum(it[4] for it in items)
        timeline.add("native_restore", "io", t0, time.perf_counter(), n=len(items),
                     bytes=job.bytes_read, logical=nbytes, **job.stats)
        last_stats.clear()
        last_stats.update(job.stats, items=len(items), bytes=job.bytes_read, logical=nbytes)
        if bad:
            raise native.CorruptBlobError(
                "corrupt HSZ1 blob: the GPU decoder rejected a frame of "
                + ", ".join(entries[i][0].path for i in bad[:4]))
        if rc != 0:
            where = entries[item][0].path if item is not None else ""
            import errno

            if rc == -errno.EBADMSG:
                raise native.CorruptBlobError(f"corrupt HSZ1 blob {where}: {msg}")
            if rc < 0 and -rc in errno.errorcode:
                raise OSError(-rc, msg)
            raise native.HipError(f"native restore failed ({rc}): {msg}")
        if hashed:
            for (rr, item, _p), h, s in zip(entries, hashed, job.sums):
                if h:
                    verifier.check_sum(rr.path, checksum.finish(s, item[2]), item[2])
        total += nbytes
    return total
