"""Device <-> host staging on MI355X.

Every GPU byte that leaves or enters HBM goes through here:

* D2H of one tensor: pinned pool block + one bulk copy (``bulk_d2h``:
  hipMemcpyAsync on a per-thread copy stream ordered after the producer
  stream, or the SDMA engines through ROCr; no pageable bounce) --
  replaces the reference's pageable ``tensor.to("cpu")`` in a 4-thread pool
  (`/root/reference/torchsnapshot/io_preparers/tensor.py:247-254`).
* non-contiguous views are packed by the ``hs_copy_nd`` kernel straight into
  host-mapped pinned memory (K2 fused with the transfer).
* slabs of small tensors are gathered into one device buffer by ONE kernel
  launch and moved with ONE DMA (K3; reference `batcher.py:101-159` did one DtoD
  per member and a pageable ``.cpu()``).
* restore: raw bytes land in pinned memory, one H2D DMA to a device scratch,
  then ONE ``hs_copy_nd`` launch scatters (and casts) into every destination
  view (K6/K7; reference `tensor.py:329-358`, `sharded_tensor.py:278-309` did a
  host ``copy_`` per region).

CPU tensors are never moved through the GPU.
"""

from __future__ import annotations

import threading
import time
from contextlib import contextmanager
from typing import Callable, Dict, Iterator, List, Optional, Sequence, Tuple

import numpy as np
import torch

from ..format.serialization import contiguous_cpu_bytes_view, tensor_from_bytes
from ..io_types import StagedBuffer, buffer_address
from ..ops import checksum, native
from ..utils.tracing import timeline

_tls = threading.local()
_slot_lock = threading.Lock()
_next_slot = [0]
NUM_COPY_SLOTS = 4
# stream slots: copy 0..63, decode / scatter 64..127, hash 128..191 -- the
# ranges never overlap whatever the staging thread count
_MAX_COPY_SLOTS = 64
_DECODE_SLOT_BASE = 64
_HASH_SLOT_BASE = 128


def copy_slot() -> int:
    """A copy-stream slot per OS thread (concurrent DMAs from executor threads):
    at least as many slots as staging threads, so two threads never share a
    stream (a stream sync would wait for the other thread's copies too)."""
    s = getattr(_tls, "slot", None)
    if s is None:
        from .. import knobs

        n = max(NUM_COPY_SLOTS, min(_MAX_COPY_SLOTS, knobs.get_stage_threads()))
        with _slot_lock:
            s = _next_slot[0] % n
            _next_slot[0] += 1
        _tls.slot = s
    return s


def hash_slot(slot: int) -> int:
    """The stream that hashes blobs beside copy slot ``slot``'s DMAs."""
    return _HASH_SLOT_BASE + slot


def decode_slot(slot: int) -> int:
    """The stream that decodes / scatters what copy slot ``slot`` uploaded:
    the copy stream then only carries H2D copies, so the next blob's upload
    does not queue behind this one's kernels."""
    return _DECODE_SLOT_BASE + slot


_ext_streams: Dict[Tuple[int, int], "torch.cuda.ExternalStream"] = {}


def _ext_stream(dev: int, slot: int) -> "torch.cuda.ExternalStream":
    key = (dev, slot)
    st = _ext_streams.get(key)
    if st is None:
        st = _ext_streams[key] = torch.cuda.ExternalStream(native.copy_stream(dev, slot),
                                                           device=f"cuda:{dev}")
    return st


def _event_on(dev: int, slot: int) -> "torch.cuda.Event":
    ev = torch.cuda.Event()
    ev.record(_ext_stream(dev, slot))
    return ev


class _DeferredDeviceWork:
    """Device work of one read pipeline that its consumers do not wait for:
    a consumer returns once its H2D copies are done (its pinned buffer can go
    back), while decode / scatter kernels keep running on the decode stream.
    ``flush`` (end of the pipeline) waits for all of it, checks the decoders'
    error words and releases what the kernels used."""

    def __init__(self) -> None:
        self.items: List[tuple] = []
        self.lock = threading.Lock()

    def add(self, done: "torch.cuda.Event", keep, err=None, what: str = "") -> None:
        """``keep``: objects to release once ``done`` fired (``.release()``
        is called on those that have it): a launch keepalive tuple, a list."""
        if isinstance(keep, tuple):
            keep = list(keep)  # (pinned descriptor stage, device workspace): both
        with self.lock:
            self.items.append([done, keep or [], err, what])
            # finished earlier items give their buffers back now, not at the
            # end of the pipeline (uncached upload blocks, descriptor stages)
            for it in self.items[:-1]:
                if it[1] and it[0].query():
                    _release_all(it[1])
                    it[1] = []

    def flush(self, raise_errors: bool = True) -> None:
        first = None
        with self.lock:
            items, self.items = self.items, []
        for done, keep, err, what in items:
            done.synchronize()
            if err is not None:
                try:
                    err.check(what)
                except Exception as e:  # noqa: BLE001 -- the first one is raised
                    first = first or e
            _release_all(keep)
        if first is not None and raise_errors:
            raise first


def _release_all(objs) -> None:
    for o in objs:
        rel = getattr(o, "release", None)
        if rel is not None:
            rel()


_deferred_scopes: List[_DeferredDeviceWork] = []
_deferred_lock = threading.Lock()


@contextmanager
def deferred_device_work() -> Iterator[_DeferredDeviceWork]:
    """Scope of a read pipeline whose H2D consumers may leave their decode /
    scatter kernels running; everything is waited for (and corrupt frames
    raised) when the scope ends."""
    scope = _DeferredDeviceWork()
    with _deferred_lock:
        _deferred_scopes.append(scope)
    try:
        yield scope
    except BaseException:
        with _deferred_lock:
            _deferred_scopes.remove(scope)
        scope.flush(raise_errors=False)
        raise
    with _deferred_lock:
        _deferred_scopes.remove(scope)
    scope.flush()


def _current_deferred() -> Optional[_DeferredDeviceWork]:
    with _deferred_lock:
        return _deferred_scopes[-1] if _deferred_scopes else None


def device_of(t: torch.Tensor) -> int:
    idx = t.device.index
    return torch.cuda.current_device() if idx is None else idx


_plan = threading.local()


@contextmanager
def plan_scope() -> Iterator[None]:
    """One take's planning on the calling thread: a device's current stream
    cannot change inside it, so ``producer_stream_handle`` looks it up once
    per device instead of once per tensor."""
    prev = getattr(_plan, "streams", None)
    _plan.streams = {}
    try:
        yield
    finally:
        _plan.streams = prev


def producer_stream_handle(t: torch.Tensor) -> Optional[int]:
    """The stream that produces ``t`` (current stream of its device, captured
    on the calling thread -- call at plan time on the training thread).
    0 is torch's default (legacy null) stream -- a real producer that the
    non-blocking copy streams must be ordered after; None = host tensor."""
    if not t.is_cuda:
        return None
    cache = getattr(_plan, "streams", None)
    if cache is None:
        return int(torch.cuda.current_stream(t.device).cuda_stream)
    h = cache.get(t.device.index)
    if h is None:
        h = cache[t.device.index] = int(torch.cuda.current_stream(t.device).cuda_stream)
    return h


def _pinned_staged(nbytes: int) -> Tuple[native.PinnedBuffer, StagedBuffer]:
    pb = native.PinnedBuffer(nbytes)
    return pb, StagedBuffer(pb.view, pb.ptr, release=pb.release, keepalive=pb)


def _dest_staged(nbytes: int) -> StagedBuffer:
    """The final host buffer of a blob of ``nbytes`` that a DMA engine fills."""
    return _pinned_staged(nbytes)[1]


_sdma_ok: dict = {}


def _is_managed(t: torch.Tensor) -> bool:
    from ..ops.uvm import is_uvm_tensor

    return is_uvm_tensor(t)


def _checksums() -> bool:
    from .. import knobs

    return knobs.checksum_enabled()


def _hash_finish(dev: int, hslot: int, handle: int, nbytes: int) -> int:
    t_s = time.perf_counter()
    h = checksum.device_hash_result(dev, hslot, handle, nbytes)
    timeline.add("hash_wait", "d2h", t_s, time.perf_counter(), bytes=nbytes)
    return h


def _use_sdma(dev: int) -> bool:
    from .. import knobs

    if knobs.get_d2h_engine() != "sdma":
        return False
    ok = _sdma_ok.get(dev)
    if ok is None:
        ok = _sdma_ok[dev] = native.sdma_engines(dev) > 0
    return ok


def bulk_d2h(dev: int, slot: int, dst: int, src: int, nbytes: int,
             producer: Optional[int] = None) -> None:
    """Blocking device -> pinned-host copy of ``nbytes``, ordered after the
    copy stream (dev, slot) and, if given, after ``producer``.  Runs on the
    SDMA engines when ``knobs.TUNING.d2h_engine`` is ``sdma`` (no CU time taken from
    a concurrent training step), else as hipMemcpyAsync."""
    t_s = time.perf_counter()
    if nbytes and _use_sdma(dev):
        if producer is not None:
            native.memcpy(dev, slot, 0, 0, 0, native.D2H, producer, sync=False)
            producer = None  # the copy stream is ordered after it now
        try:
            native.sdma_d2h(dev, dst, src, nbytes, native.copy_stream(dev, slot))
            timeline.add("dma", "d2h", t_s, time.perf_counter(), bytes=nbytes, slot=slot)
            return
        except native.HipError as e:
            # nothing is left in flight after a failed SDMA copy (every issued
            # piece was waited for): redo it as a blit, and stop using SDMA
            import logging

            logging.getLogger(__name__).warning(
                f"SDMA device->host copy failed on cuda:{dev} ({e}); using hipMemcpyAsync")
            _sdma_ok[dev] = False
    native.memcpy(dev, slot, dst, src, nbytes, native.D2H, producer, sync=True)
    timeline.add("dma", "d2h", t_s, time.perf_counter(), bytes=nbytes, slot=slot)


_dma_limits: dict = {}


def _dma_limit(dev: int) -> threading.BoundedSemaphore:
    from .. import knobs

    n = knobs.get_dma_inflight()
    got = _dma_limits.get(dev)
    if got is None or got[0] != n:
        # (a changed knob takes effect for copies submitted from now on)
        with _slot_lock:
            got = _dma_limits.get(dev)
            if got is None or got[0] != n:
                got = _dma_limits[dev] = (n, threading.BoundedSemaphore(n))
    return got[1]


def d2h_staged(dev: int, slot: int, staged: StagedBuffer, src: int, nbytes: int,
               keep: list, hash_handle: Optional[int] = None,
               producer: Optional[int] = None) -> None:
    """Device -> pinned copy of ``nbytes`` at ``src`` into ``staged`` (and the
    hash started as ``hash_handle`` on ``hash_slot(slot)``, if any).

    On the SDMA engines (``knobs.TUNING.async_dma``, default on) the copy is
    only SUBMITTED here: ``staged.ready`` then waits for it (the writer calls
    it before writing) and the staging worker goes on to prepare its next
    blob while the engine works through its queue -- the engine no longer
    idles while every worker encodes.  ``keep`` holds the device buffers the
    copy reads; they are dropped once it is done.  At most
    ``knobs.TUNING.dma_inflight`` copies per device are in flight (device
    buffers of queued blobs stay allocated until then)."""
    from .. import knobs

    hslot = hash_slot(slot)
    if nbytes and knobs.async_dma() and _use_sdma(dev):
        if producer is not None:
            native.memcpy(dev, slot, 0, 0, 0, native.D2H, producer, sync=False)
        lim = _dma_limit(dev)
        lim.acquire()
        t_s = time.perf_counter()
        try:
            h = native.sdma_d2h_submit(dev, staged.addr, src, nbytes,
                                       native.copy_stream(dev, slot))
        except native.HipError as e:
            lim.release()
            import logging

            logging.getLogger(__name__).warning(
                f"SDMA device->host copy failed on cuda:{dev} ({e}); using hipMemcpyAsync")
            _sdma_ok[dev] = False
        else:
            done = [False]

            def ready() -> None:
                if done[0]:
                    return
                try:
                    try:
                        native.sdma_wait(h)
                    except native.HipError as e:
                        import logging

                        logging.getLogger(__name__).warning(
                            f"SDMA device->host copy failed on cuda:{dev} ({e}); "
                            "redoing it with hipMemcpyAsync")
                        _sdma_ok[dev] = False
                        native.memcpy(dev, copy_slot(), staged.addr, src, nbytes, native.D2H,
                                      None, sync=True)
                    timeline.add("dma", "d2h", t_s, time.perf_counter(), bytes=nbytes,
                                 slot=slot)
                    if hash_handle is not None:
                        staged.checksum = _hash_finish(dev, hslot, hash_handle, nbytes)
                finally:
                    done[0] = True
                    keep.clear()
                    lim.release()

            staged.ready = ready
            return
    bulk_d2h(dev, slot, staged.addr, src, nbytes, producer)
    if hash_handle is not None:
        staged.checksum = _hash_finish(dev, hslot, hash_handle, nbytes)
    keep.clear()


def wait_ready(staged: StagedBuffer) -> StagedBuffer:
    """Block until ``staged``'s bytes have arrived (asynchronous copy)."""
    ready = staged.ready
    if ready is not None:
        staged.ready = None
        ready()
    return staged


def _elem_strides_ok(t: torch.Tensor) -> bool:
    return t.dim() <= native.MAX_DIMS


def host_resident_managed(t: torch.Tensor) -> bool:
    """A managed (UVM) tensor whose pages live in host DRAM (``ops.uvm``)."""
    from ..ops import uvm

    return uvm.residency(t) == "host"


def managed_host_view(t: torch.Tensor, producer: Optional[int]) -> StagedBuffer:
    """The bytes of a contiguous host-resident managed tensor, in place: the
    writer ``pwrite``s straight from the UVM pages (one DRAM read, no DMA
    over PCIe and back, no pinned copy) and hashes them on the host.  Waits
    for the producer stream first (kernels queued before the take may still
    write the table).  Only for blocking takes: the view aliases live memory.
    Restores read into the same view (``TensorBufferConsumer.get_read_dest``)."""
    if producer is not None:
        native.sync_stream_handle(producer)
    else:
        torch.cuda.current_stream(t.device).synchronize()
    nbytes = t.numel() * t.element_size()
    import ctypes

    mv = memoryview((ctypes.c_char * nbytes).from_address(t.data_ptr())).cast("B")
    staged = StagedBuffer(mv, addr=t.data_ptr(), keepalive=t)
    # the writer copies the pages into the page cache: on their node
    from ..utils.affinity import pages_node

    staged.numa_node = pages_node(t.data_ptr(), nbytes)
    return staged


def d2h_tensor(t: torch.Tensor, producer: Optional[int],
               codec: Optional[dict] = None, alias_ok: bool = False) -> StagedBuffer:
    """Copy a CUDA tensor's logical bytes (C order) into a pinned block.

    With ``codec`` (HSZ1 info dict) the bytes are compressed on the GPU first
    and only the encoded blob crosses PCIe.  ``alias_ok`` (blocking takes): a
    contiguous managed tensor in host DRAM is handed out in place
    (``managed_host_view``) instead of copied.
    """
    if codec is not None:
        return _d2h_encoded(t, producer, codec)
    if alias_ok and t.is_contiguous() and t.numel() and host_resident_managed(t):
        t_s = time.perf_counter()
        staged = managed_host_view(t, producer)
        timeline.add("uvm_host_view", "d2h", t_s, time.perf_counter(), bytes=staged.nbytes)
        return staged
    nbytes = t.numel() * t.element_size()
    if t.is_contiguous():
        pb, staged = None, _dest_staged(nbytes)
    else:  # packed by a kernel storing into the (device-mapped) pinned block
        pb, staged = _pinned_staged(nbytes)
    if nbytes == 0:
        return staged
    dev = device_of(t)
    slot = copy_slot()
    t_s = time.perf_counter()
    try:
        if t.is_contiguous():
            hs = None
            if _checksums() and not _is_managed(t):
                # hash the bytes in HBM on a side stream (ordered after the
                # producer) while the DMA moves them; both only read them.
                # (Managed tables usually live in host memory: a GPU hash
                # would pull them over the PCIe link the DMA is using -- the
                # writer hashes the pinned copy on the host instead.)
                native.memcpy(dev, slot, 0, 0, 0, native.D2H, producer, sync=False)
                producer = None
                hs = checksum.device_hash_start(dev, hash_slot(slot), t.data_ptr(), nbytes,
                                                slot)
            d2h_staged(dev, slot, staged, t.data_ptr(), nbytes, [t], hs, producer)
        else:
            # pack-to-host: kernel stores the packed view over PCIe into the
            # host-mapped pinned block, ordered after the producer stream.
            native.memcpy(dev, slot, 0, 0, 0, native.D2H, producer, sync=False)
            batch = native.CopyBatch()
            batch.add(t.data_ptr(), t.dtype, t.stride(), pb.ptr, t.dtype,
                      _contig_strides(t.shape), list(t.shape), t.element_size())
            batch.launch(dev, native.copy_stream(dev, slot), sync=True)
    except BaseException:
        staged.release()
        raise
    timeline.add("d2h", "d2h", t_s, time.perf_counter(), bytes=nbytes, slot=slot)
    return staged


def _join_current_stream(dev: int, slot: int) -> None:
    """Order the copy stream after the current stream: memory just handed out
    by torch's caching allocator is only safe to use in that stream's order."""
    native.memcpy(dev, slot, 0, 0, 0, native.D2H,
                  int(torch.cuda.current_stream(dev).cuda_stream), sync=False)


def _read_u64_device(dev: int, slot: int, addr: int) -> int:
    pb = native.PinnedBuffer(8)
    try:
        native.memcpy(dev, slot, pb.ptr, addr, 8, native.D2H, None, sync=True)
        return int(pb.as_tensor(8).view(torch.int64)[0])
    finally:
        pb.release()


_encode_locks: dict = {}
_encode_locks_mu = threading.Lock()


@contextmanager
def _encode_turn(dev: int, nbytes: int) -> Iterator[None]:
    """Large HSZ1 encodes take turns per device (``knobs.TUNING.serial_encode``).

    Encodes launched by several staging threads at once share the CUs, so
    each finishes only when all do: at the start of a take four 512 MiB
    chunks were encoded together and the first DMA waited ~2.3 ms for them.
    Taking turns, each runs on the whole chip (~1 TB/s) and its DMA starts
    as soon as it is done; the encoder stays far ahead of PCIe either way.
    Encodes below 256 MiB (slabs) finish in ~0.1 ms and keep running
    side by side (serialising them measured slightly slower)."""
    from .. import knobs

    if nbytes < (256 << 20) or not knobs.serial_encode():
        yield
        return
    lock = _encode_locks.get(dev)
    if lock is None:
        with _encode_locks_mu:
            lock = _encode_locks.setdefault(dev, threading.Lock())
    with lock:
        yield


def _encode_device_to_host(dev: int, slot: int, src_u8: torch.Tensor, codec: dict
                           ) -> StagedBuffer:
    """HSZ1-encode a contiguous device byte tensor on the copy stream, then
    move only the encoded bytes to a pinned block (one small sync in between
    to learn the encoded size)."""
    from ..ops import codec as hsz

    stream = native.copy_stream(dev, slot)
    t_s = time.perf_counter()
    try:
        with torch.cuda.device(dev):
            out, total, meta = hsz.encode_device(src_u8, int(codec["w"]), 0,
                                                 int(codec["frame_bytes"]), launch=False)
    except torch.cuda.OutOfMemoryError:
        return _encode_on_host(dev, slot, src_u8, codec)
    t_a = time.perf_counter()
    _join_current_stream(dev, slot)
    with _encode_turn(dev, src_u8.numel()):
        hsz.launch_encode(src_u8, int(codec["w"]), stream, int(codec["frame_bytes"]), out,
                          total, meta)
        t_l = time.perf_counter()
        nbytes = _read_u64_device(dev, slot, total.data_ptr())
    t_n = time.perf_counter()
    staged = _dest_staged(nbytes)
    t_p = time.perf_counter()
    timeline.add("enc_alloc", "enc", t_s, t_a)
    timeline.add("enc_launch", "enc", t_a, t_l)
    timeline.add("enc_wait", "enc", t_l, t_n)
    timeline.add("enc_pinned", "enc", t_n, t_p)
    try:
        hs = None
        if _checksums():
            hs = checksum.device_hash_start(dev, hash_slot(slot), out.data_ptr(), nbytes, slot)
        d2h_staged(dev, slot, staged, out.data_ptr(), nbytes, [out, total, meta], hs)
    except BaseException:
        staged.release()
        raise
    del out, total, meta
    timeline.add("encode_d2h", "d2h", t_s, time.perf_counter(), bytes=nbytes,
                 logical=src_u8.numel(), slot=slot)
    return staged


def _encode_on_host(dev: int, slot: int, src_u8: torch.Tensor, codec: dict) -> StagedBuffer:
    """Fallback when HBM is short: raw D2H, then the C++ encoder."""
    from ..ops import codec as hsz

    n = src_u8.numel()
    raw_pb = native.PinnedBuffer(max(n, 1))
    try:
        if n:
            bulk_d2h(dev, slot, raw_pb.ptr, src_u8.data_ptr(), n)
        return _encode_host_bytes(raw_pb.ptr, n, codec)
    finally:
        raw_pb.release()


def encode_host_buffer(buf: StagedBuffer, codec: dict) -> StagedBuffer:
    """C++ HSZ1 encode of host bytes (host tensors / host slabs)."""
    return _encode_host_bytes(buf.addr, buf.nbytes, codec)


def _encode_host_bytes(addr: int, n: int, codec: dict) -> StagedBuffer:
    from ..ops import codec as hsz

    cap = hsz.max_encoded_bytes(n, int(codec["frame_bytes"]))
    if native.hsgpu_loaded() and native.gpu_available():
        pb, staged = _pinned_staged(cap)
        out_addr, view, release, keep = pb.ptr, pb.view, pb.release, pb
    else:
        arr = np.empty(cap, dtype=np.uint8)
        out_addr, view, release, keep = arr.ctypes.data, memoryview(arr), None, arr
    try:
        used = native.hsz_encode_cpu(addr if n else out_addr, n, int(codec["w"]),
                                     int(codec["frame_bytes"]), out_addr)
    except BaseException:
        if release is not None:
            release()
        raise
    return StagedBuffer(view[:used], out_addr, release=release, keepalive=keep)


def _d2h_encoded(t: torch.Tensor, producer: Optional[int], codec: dict) -> StagedBuffer:
    dev = device_of(t)
    slot = copy_slot()
    native.memcpy(dev, slot, 0, 0, 0, native.D2H, producer, sync=False)
    nbytes = t.numel() * t.element_size()
    if t.is_contiguous() and t.data_ptr() % 16 == 0:
        src = torch.empty(0, dtype=torch.uint8, device=t.device).set_(
            t.untyped_storage(), t.storage_offset() * t.element_size(), (nbytes,))
    else:
        src = torch.empty(nbytes, dtype=torch.uint8, device=t.device)
        _join_current_stream(dev, slot)
        if nbytes:
            batch = native.CopyBatch()
            batch.add(t.data_ptr(), t.dtype, t.stride(), src.data_ptr(), t.dtype,
                      _contig_strides(t.shape), list(t.shape), t.element_size())
            keep = batch.launch(dev, native.copy_stream(dev, slot), sync=False)
            native.stream_sync(dev, slot)
            if keep is not None:
                keep[0].release()
    return _encode_device_to_host(dev, slot, src, codec)


def _contig_strides(shape: Sequence[int]) -> List[int]:
    st = [1] * len(shape)
    for i in range(len(shape) - 2, -1, -1):
        st[i] = st[i + 1] * max(int(shape[i + 1]), 1)
    return st


def cpu_tensor_bytes(t: torch.Tensor, copy: bool) -> StagedBuffer:
    """Host bytes of a CPU tensor; zero-copy unless ``copy`` (async snapshot)."""
    t = t.detach()
    if copy or not t.is_contiguous():
        nbytes = t.numel() * t.element_size()
        if native.hsgpu_loaded() and native.gpu_available() and nbytes >= (1 << 20):
            # pinned destination: the block is reused across snapshots
            pb, staged = _pinned_staged(nbytes)
            dst = pb.as_tensor(nbytes).view(t.dtype).view(t.shape) if nbytes else None
            if dst is not None:
                dst.copy_(t)
            return staged
        out = torch.empty(t.shape, dtype=t.dtype)
        out.copy_(t)
        t = out
    mv = contiguous_cpu_bytes_view(t)
    return StagedBuffer(mv, keepalive=t)


def _add_members_zero_gaps(batch, members, base: int, dev: int) -> None:
    """Slab members at their offsets, and zeros in the alignment gaps between
    them (same launch): a slab's padding never carries stale HBM bytes, and
    every drain path writes identical blobs."""
    from .hbm_staging import add_zero_fill

    end = 0
    for t, off in sorted(members, key=lambda m: m[1]):
        if off > end:
            add_zero_fill(batch, base + end, off - end)
        batch.add_tensor(t, base + off)
        end = max(end, off + t.numel() * t.element_size())


def _launch_slab_gather(members, base: int, dev: int, stream: int,
                        pack_cache: Optional[dict]):
    """One hs_copy_nd launch gathering ``members`` (tensor, offset) into the
    slab at ``base``, gaps zeroed.  ``pack_cache`` (kept on a reused plan's
    stager): the packed descriptor table of the last launch from the same
    sources is launched again, its destinations moved to this take's slab
    address, instead of rebuilt (0.1-0.2 ms of GIL-holding work per slab,
    per take).  Every destination lies in the slab, so one offset moves all."""
    key = None
    if pack_cache is not None:
        key = tuple((t.data_ptr(), off) for t, off in members)
        if pack_cache.get("key") == key:
            arr = pack_cache["arr"]
            delta = (base - pack_cache["base"]) % (1 << 64)
            if delta:
                arr["dst"] += np.uint64(delta)  # (wraps modulo 2**64, like the pointers)
                pack_cache["base"] = base
            return native.launch_packed(arr, dev, stream, sync=False)
    batch = native.CopyBatch()
    _add_members_zero_gaps(batch, members, base, dev)
    if not len(batch):
        return None
    with timeline.span("copy_pack", n=len(batch)):
        arr = batch.pack()
    if key is not None:
        pack_cache["key"], pack_cache["arr"], pack_cache["base"] = key, arr, base
    return native.launch_packed(arr, dev, stream, sync=False)


def gather_to_host(members: Sequence[Tuple[torch.Tensor, int]], total_bytes: int,
                   producers: Sequence[int], via_device_slab: bool = True,
                   codec: Optional[dict] = None,
                   pack_cache: Optional[dict] = None) -> StagedBuffer:
    """Pack many CUDA tensors into one host slab: ``members`` = (tensor, offset).

    Default path: one ``hs_copy_nd`` launch gathers every member into a device
    slab (HBM-speed), then ONE SDMA transfer moves the slab to pinned memory.
    If the device slab cannot be allocated the kernel writes the members
    straight into host-mapped pinned memory instead.
    """
    if codec is not None and members:
        return _gather_encoded(members, total_bytes, producers, codec, pack_cache)
    if not via_device_slab or not members:
        return _gather_into_host(members, total_bytes, producers)
    staged = _dest_staged(total_bytes)
    if total_bytes == 0:
        return staged
    dev = device_of(members[0][0])
    slot = copy_slot()
    stream = native.copy_stream(dev, slot)
    t_s = time.perf_counter()
    try:
        for producer in producers:
            native.memcpy(dev, slot, 0, 0, 0, native.D2H, producer, sync=False)
        try:
            slab = torch.empty(total_bytes, dtype=torch.uint8, device=f"cuda:{dev}")
        except torch.cuda.OutOfMemoryError:
            staged.release()
            return _gather_into_host(members, total_bytes, producers)
        _join_current_stream(dev, slot)
        keep = _launch_slab_gather(members, slab.data_ptr(), dev, stream, pack_cache)
        hs = None
        if _checksums():
            hs = checksum.device_hash_start(dev, hash_slot(slot), slab.data_ptr(),
                                            total_bytes, slot)
        d2h_staged(dev, slot, staged, slab.data_ptr(), total_bytes, [slab], hs)
        if keep is not None:
            # the gather kernel is done: submitting the copy waited for it
            keep[0].release()
        del slab
    except BaseException:
        staged.release()
        raise
    timeline.add("gather_d2h", "d2h", t_s, time.perf_counter(), bytes=total_bytes,
                 members=len(members), slot=slot)
    return staged


def _gather_into_host(members: Sequence[Tuple[torch.Tensor, int]], total_bytes: int,
                      producers: Sequence[int]) -> StagedBuffer:
    """No HBM for a device slab: the gather kernel stores the members over
    PCIe straight into a (device-mapped) pinned block."""
    pb, staged = _pinned_staged(total_bytes)
    if total_bytes == 0 or not members:
        return staged
    dev = device_of(members[0][0])
    slot = copy_slot()
    t_s = time.perf_counter()
    try:
        for producer in producers:
            native.memcpy(dev, slot, 0, 0, 0, native.D2H, producer, sync=False)
        batch = native.CopyBatch()
        _add_members_zero_gaps(batch, members, pb.ptr, dev)
        keep = batch.launch(dev, native.copy_stream(dev, slot), sync=False)
        native.stream_sync(dev, slot)
        if keep is not None:
            keep[0].release()
    except BaseException:
        staged.release()
        raise
    timeline.add("gather_d2h", "d2h", t_s, time.perf_counter(), bytes=total_bytes,
                 members=len(members), slot=slot)
    return staged


def _gather_encoded(members, total_bytes: int, producers, codec: dict,
                    pack_cache: Optional[dict] = None) -> StagedBuffer:
    """Slab gather into HBM (one launch), HSZ1 encode, D2H of the encoded bytes."""
    t0 = time.perf_counter()
    dev = device_of(members[0][0])
    slot = copy_slot()
    stream = native.copy_stream(dev, slot)
    for producer in producers:
        native.memcpy(dev, slot, 0, 0, 0, native.D2H, producer, sync=False)
    t1 = time.perf_counter()
    try:
        # uninitialised: the gather launch writes the members AND zeros into
        # the alignment gaps (no separate zero-fill pass over the slab)
        slab = torch.empty(total_bytes, dtype=torch.uint8, device=f"cuda:{dev}")
        timeline.add("slab_join", "stage", t0, t1)
    except torch.cuda.OutOfMemoryError:
        # no HBM for the slab: gather into host memory, encode on the CPU
        raw = gather_to_host(members, total_bytes, producers, via_device_slab=False)
        try:
            return _encode_host_bytes(raw.addr, total_bytes, codec)
        finally:
            raw.release()
    # the slab comes from torch's allocator on the current stream: order the
    # copy stream after it (padding bytes are encoded too: zeroed below)
    _join_current_stream(dev, slot)
    keep = _launch_slab_gather(members, slab.data_ptr(), dev, stream, pack_cache)
    try:
        return _encode_device_to_host(dev, slot, slab, codec)
    finally:
        if keep is not None:
            keep[0].release()


def h2d_into(dst: torch.Tensor, host_addr: int, nbytes: int, src_dtype: torch.dtype,
             src_shape: Sequence[int], producer: Optional[int] = None) -> None:
    """Load C-order bytes at ``host_addr`` (ideally pinned) into CUDA ``dst``.

    Same dtype + contiguous destination -> one DMA.  Otherwise one DMA into a
    device scratch followed by one scatter/cast kernel launch.
    """
    dev = device_of(dst)
    slot = copy_slot()
    sdma = _current_deferred() is not None and nbytes >= _SDMA_MIN_BYTES and _sdma_uploads(dev)
    if dst.dtype == src_dtype and dst.is_contiguous() and list(dst.shape) == list(src_shape) \
            and not _is_managed(dst) and not sdma:
        native.memcpy(dev, slot, dst.data_ptr(), host_addr, nbytes, native.H2D, producer,
                      sync=True)
        return
    scatter_host_regions(host_addr, nbytes, [(src_dtype, src_shape, 0, None, dst)], dev,
                         producer)


def scatter_host_regions(host_addr: int, nbytes: int, regions, dev: int,
                         producer: Optional[int] = None) -> None:
    with timeline.span("h2d_scatter", "h2d", bytes=nbytes, regions=len(regions)):
        _scatter_host_regions(host_addr, nbytes, regions, dev, producer)


def _scatter_host_regions(host_addr: int, nbytes: int, regions, dev: int,
                          producer: Optional[int] = None) -> None:
    """One H2D of ``nbytes`` at ``host_addr`` then ONE kernel launch that copies
    every region into its destination view.

    ``regions``: list of (src_dtype, src_shape, byte_offset_in_buffer,
    narrows or None, dst_view) where ``narrows`` is a list of
    (dim, start, length) applied to the source tensor view before copying.
    """
    slot = copy_slot()
    # order after pending work on the destinations' stream (captured at plan time)
    native.memcpy(dev, slot, 0, 0, 0, native.H2D, producer, sync=False)
    scope = _current_deferred()
    if scope is not None and nbytes >= _SDMA_MIN_BYTES and _sdma_uploads(dev) and \
            all(native.can_cast_on_device(r[0], r[4].dtype) and r[4].dim() <= native.MAX_DIMS
                for r in regions):
        _scatter_host_regions_sdma(host_addr, nbytes, regions, dev, slot, scope)
        return
    # Regions whose source bytes are one contiguous range and whose destination
    # is a contiguous tensor of the same dtype/shape go host -> destination with
    # one DMA each (no scratch, no kernel: the common FSDP/DTensor restore).
    # Managed (UVM) destinations take the scratch + kernel path: a host ->
    # managed DMA ran at 4.8 GB/s into HBM-resident pages (profiles/r3/s2/),
    # the kernel writes them at HBM rate.
    kernel_regions = []
    for region in regions:
        src_dtype, src_shape, off, narrows, dst = region
        rng = _contiguous_src_range(src_dtype, src_shape, off, narrows)
        if (rng is not None and dst.dtype == src_dtype and dst.is_contiguous()
                and dst.numel() * dst.element_size() == rng[1] and not _is_managed(dst)):
            native.memcpy(dev, slot, dst.data_ptr(), host_addr + rng[0], rng[1], native.H2D,
                          None, sync=False)
        else:
            kernel_regions.append(region)
    if not kernel_regions:
        native.stream_sync(dev, slot)
        return
    scratch = torch.empty(nbytes, dtype=torch.uint8, device=f"cuda:{dev}")
    _join_current_stream(dev, slot)
    native.memcpy(dev, slot, scratch.data_ptr(), host_addr, nbytes, native.H2D, None,
                  sync=False)
    if scope is None:
        _copy_regions(scratch, kernel_regions, dev, slot)
        return
    # the copy kernel runs on the decode stream after the upload; this
    # consumer only waits for the upload (its host buffer goes back)
    h2d = _event_on(dev, slot)
    dslot = decode_slot(slot)
    native.memcpy(dev, dslot, 0, 0, 0, native.H2D, native.copy_stream(dev, slot), sync=False)
    keep = _copy_regions(scratch, kernel_regions, dev, dslot, wait=False)
    scratch.record_stream(_ext_stream(dev, dslot))
    scope.add(_event_on(dev, dslot), keep)
    t_w = time.perf_counter()
    h2d.synchronize()
    timeline.add("h2d_wait", "h2d", t_w, time.perf_counter(), bytes=nbytes)


# below this, one hipMemcpyAsync is cheaper than an uncached block + a kernel
_SDMA_MIN_BYTES = 1 << 20


def _scatter_host_regions_sdma(host_addr: int, nbytes: int, regions, dev: int, slot: int,
                               scope) -> None:
    """The whole buffer goes up on an SDMA engine into an uncached block (one
    DMA instead of a HIP copy call per region; those calls block for ms when
    several threads upload), then ONE copy kernel on the decode stream writes
    every destination view; this consumer returns once the upload is done."""
    ub = native.UncachedBlock(dev, nbytes)
    try:
        t0 = time.perf_counter()
        native.sdma_h2d(dev, ub.ptr, host_addr, nbytes)
        t1 = time.perf_counter()
        dslot = decode_slot(slot)
        native.memcpy(dev, dslot, 0, 0, 0, native.H2D, native.copy_stream(dev, slot), sync=False)
        keep = [ub]
        ck = _copy_regions(None, regions, dev, dslot, wait=False, base=ub.ptr)
        if ck is not None:
            keep.extend(ck)
    except BaseException:
        native.stream_sync(dev, decode_slot(slot))
        ub.release()
        raise
    scope.add(_event_on(dev, dslot), keep)
    timeline.add("h2d_sdma", "h2d", t0, t1, bytes=nbytes)


_elem_sizes: dict = {}


def _elem_size(dtype: torch.dtype) -> int:
    es = _elem_sizes.get(dtype)
    if es is None:
        es = _elem_sizes[dtype] = torch.empty(0, dtype=dtype).element_size()
    return es


def _copy_regions(scratch: Optional[torch.Tensor], regions, dev: int, slot: int,
                  wait: bool = True, base: Optional[int] = None):
    """ONE copy/cast launch from the device buffer ``scratch`` (region offsets
    are relative to it) into every destination view, then a stream sync.
    ``wait=False``: no sync; returns the launch's keepalive (the caller holds
    it until the stream passed the launch)."""
    t0 = time.perf_counter()
    batch = native.CopyBatch()
    fallbacks = []
    if base is None:
        base = scratch.data_ptr()
    for src_dtype, src_shape, off, narrows, dst in regions:
        es = _elem_size(src_dtype)
        if native.can_cast_on_device(src_dtype, dst.dtype) and dst.dim() <= native.MAX_DIMS:
            # the source view's pointer / shape / strides in plain integers (a
            # C-order block at ``off``, narrowed): no torch view per region
            shape = [int(z) for z in src_shape]
            strides = _contig_strides(shape)
            ptr = base + off
            if narrows:
                for d, st, ln in narrows:
                    ptr += st * strides[d] * es
                    shape[d] = ln
            batch.add(ptr, src_dtype, strides, dst.data_ptr(), dst.dtype, dst.stride(), shape,
                      es)
        else:
            n = 1
            for z in src_shape:
                n *= int(z)
            src = scratch[off: off + n * es].view(src_dtype).view(list(src_shape))
            if narrows:
                for d, st, ln in narrows:
                    src = src.narrow(d, st, ln)
            fallbacks.append((src, dst))
    t1 = time.perf_counter()
    keep = batch.launch(dev, native.copy_stream(dev, slot), sync=False)
    t2 = time.perf_counter()
    if not wait and not fallbacks:
        timeline.add("regions_build", "h2d", t0, t1, n=len(regions))
        timeline.add("regions_launch", "h2d", t1, t2)
        return keep
    native.stream_sync(dev, slot)
    t3 = time.perf_counter()
    timeline.add("regions_build", "h2d", t0, t1, n=len(regions))
    timeline.add("regions_launch", "h2d", t1, t2)
    timeline.add("dec_wait", "h2d", t2, t3)
    if keep is not None:
        keep[0].release()
    if fallbacks:
        # integer<->float and other exotic casts: ATen on the current stream
        for src, dst in fallbacks:
            dst.copy_(src)
        torch.cuda.synchronize(dev)


def scatter_compressed(span, regions, dev: int, producer: Optional[int] = None) -> None:
    """HSZ1 restore into HBM: ONE H2D of the encoded frames, ONE decode launch,
    then the same region copy as ``scatter_host_regions``.  A single region
    that is the whole blob, contiguous and of the stored dtype is decoded
    straight into its destination (no scratch, no copy)."""
    with timeline.span("h2d_decode", "h2d", bytes=span.nbytes, regions=len(regions)):
        _scatter_compressed(span, regions, dev, producer)


def _scatter_compressed(span, regions, dev: int, producer: Optional[int] = None) -> None:
    from ..ops import codec as hsz

    h = span.header
    first, last = span.first, span.last
    if last <= first:
        return
    slot = copy_slot()
    native.memcpy(dev, slot, 0, 0, 0, native.H2D, producer, sync=False)
    c_lo = h.offsets[first]
    c_n = h.offsets[last] - c_lo
    log_lo = span.frames_logical_lo
    log_n = min(last * h.frame_bytes, h.logical_size) - log_lo
    direct = None
    if len(regions) == 1:
        src_dtype, src_shape, off, narrows, dst = regions[0]
        rng = _contiguous_src_range(src_dtype, src_shape, off, narrows)
        if (rng is not None and rng[0] + span.lo == log_lo and rng[1] == log_n
                and dst.dtype == src_dtype and dst.is_contiguous()
                and dst.data_ptr() % 16 == 0):
            direct = dst
    t0 = time.perf_counter()
    # frame offsets go up from pinned memory: a pageable source would make
    # the async H2D wait for the encoded frames' copy queued before it
    n_offs = last - first + 1
    offs_pb = native.PinnedBuffer(8 * n_offs)
    offs = np.frombuffer(offs_pb.view, dtype=np.int64, count=n_offs)
    offs[:] = np.asarray(h.offsets[first:last + 1], dtype=np.int64) - c_lo
    try:
        scope = _current_deferred()
        if scope is not None and _sdma_uploads(dev):
            _decode_span_sdma(span, regions, dev, slot, direct, offs_pb, n_offs, c_n, log_lo,
                              log_n, first, last, t0, scope)
            return
        enc = torch.empty(c_n, dtype=torch.uint8, device=f"cuda:{dev}")
        _decode_span(span, regions, dev, slot, direct, enc, offs_pb, n_offs, c_n, log_lo, log_n,
                     first, last, t0)
    finally:
        del offs
        try:
            native.stream_sync(dev, slot)  # no-op normally; on errors: H2D done
        finally:
            offs_pb.release()


_sdma_ok: Dict[int, bool] = {}


def _sdma_uploads(dev: int) -> bool:
    """Encoded frames go up on the SDMA engines (``knobs.TUNING.h2d_engine``,
    default sdma, when ROCr reports an engine)."""
    from .. import knobs

    if knobs.get_h2d_engine() != "sdma":
        return False
    ok = _sdma_ok.get(dev)
    if ok is None:
        ok = _sdma_ok[dev] = native.sdma_engines(dev) > 0
    return ok


def _decode_span_sdma(span, regions, dev, slot, direct, offs_pb, n_offs, c_n, log_lo, log_n,
                      first, last, t0, scope) -> None:
    """Upload the encoded frames and their offsets on an SDMA engine into an
    uncached device block (no HIP runtime copy call: those block for ms when
    several threads upload, profiles/r4/restore_trace/), then leave decode +
    scatter running on the decode stream; the block goes back once they ran."""
    h = span.header
    offs_at = (c_n + 15) // 16 * 16
    ub = native.UncachedBlock(dev, offs_at + 8 * n_offs)
    try:
        out = None if direct is not None else torch.empty(log_n, dtype=torch.uint8,
                                                         device=f"cuda:{dev}")
        t1 = time.perf_counter()
        native.sdma_h2d(dev, ub.ptr + offs_at, offs_pb.ptr, 8 * n_offs)
        tail = span.tail
        if tail is not None and 0 < tail.offset < c_n:
            # the head's frames go up while the rest of the blob is being read
            native.sdma_h2d(dev, ub.ptr, span.buf.addr, tail.offset)
            t_w = time.perf_counter()
            tail.wait()
            timeline.add("tail_wait", "h2d", t_w, time.perf_counter())
            native.sdma_h2d(dev, ub.ptr + tail.offset, span.buf.addr + tail.offset,
                            c_n - tail.offset)
        else:
            span.wait_tail()
            native.sdma_h2d(dev, ub.ptr, span.buf.addr, c_n)
        t2 = time.perf_counter()
        kslot = decode_slot(slot)
        # after the destinations' producer (joined on the copy stream) and
        # after the current stream (``out`` comes from its allocator)
        native.memcpy(dev, kslot, 0, 0, 0, native.H2D, native.copy_stream(dev, slot), sync=False)
        _join_current_stream(dev, kslot)
        err = native.DecodeErrorWord()
        native.hsz_decode_gpu(dev, ub.ptr, ub.ptr + offs_at, first, last - first,
                              h.logical_size, h.elem_width, h.frame_bytes,
                              (direct if direct is not None else out).data_ptr(),
                              native.copy_stream(dev, kslot), err.addr)
        keep = [ub]
        if direct is None:
            ck = _copy_regions(out[span.lo - log_lo:], regions, dev, kslot, wait=False)
            if ck is not None:
                keep.extend(ck)  # descriptor stage + device workspace
            out.record_stream(_ext_stream(dev, kslot))
    except BaseException:
        native.stream_sync(dev, decode_slot(slot))
        ub.release()
        raise
    scope.add(_event_on(dev, kslot), keep, err, f"frames [{first}, {last})")
    timeline.add("dec_alloc", "h2d", t0, t1)
    timeline.add("h2d_sdma", "h2d", t1, t2, bytes=c_n)
    timeline.add("dec_launch", "h2d", t2, time.perf_counter())


def _decode_span(span, regions, dev, slot, direct, enc, offs_pb, n_offs, c_n, log_lo, log_n,
                 first, last, t0) -> None:
    h = span.header
    offs_dev = torch.empty(n_offs, dtype=torch.int64, device=f"cuda:{dev}")
    out = None if direct is not None else torch.empty(log_n, dtype=torch.uint8,
                                                     device=f"cuda:{dev}")
    t1 = time.perf_counter()
    _join_current_stream(dev, slot)
    tail = span.tail
    if tail is not None and 0 < tail.offset < c_n:
        # the head's frames go up while the rest of the blob is still being read
        native.memcpy(dev, slot, enc.data_ptr(), span.buf.addr, tail.offset, native.H2D, None,
                      sync=False)
        t_w = time.perf_counter()
        tail.wait()
        timeline.add("tail_wait", "h2d", t_w, time.perf_counter())
        native.memcpy(dev, slot, enc.data_ptr() + tail.offset, span.buf.addr + tail.offset,
                      c_n - tail.offset, native.H2D, None, sync=False)
    else:
        span.wait_tail()
        native.memcpy(dev, slot, enc.data_ptr(), span.buf.addr, c_n, native.H2D, None,
                      sync=False)
    native.memcpy(dev, slot, offs_dev.data_ptr(), offs_pb.ptr, 8 * n_offs, native.H2D, None,
                  sync=False)
    scope = _current_deferred()
    kslot = slot
    if scope is not None:
        # decode + scatter on the decode stream, after the uploads: the copy
        # stream is free for the next blob's upload at once
        h2d = _event_on(dev, slot)
        kslot = decode_slot(slot)
        native.memcpy(dev, kslot, 0, 0, 0, native.H2D, native.copy_stream(dev, slot), sync=False)
    stream = native.copy_stream(dev, kslot)
    err = native.DecodeErrorWord()
    native.hsz_decode_gpu(dev, enc.data_ptr(), offs_dev.data_ptr(), first, last - first,
                          h.logical_size, h.elem_width, h.frame_bytes,
                          (direct if direct is not None else out).data_ptr(), stream,
                          err.addr)
    t2 = time.perf_counter()
    timeline.add("dec_alloc", "h2d", t0, t1)
    timeline.add("dec_launch", "h2d", t1, t2)
    if scope is not None:
        keep = None
        if direct is None:
            keep = _copy_regions(out[span.lo - log_lo:], regions, dev, kslot, wait=False)
        ext = _ext_stream(dev, kslot)
        for t in (enc, offs_dev, out):
            if t is not None:
                t.record_stream(ext)
        scope.add(_event_on(dev, kslot), keep, err, f"frames [{first}, {last})")
        t_w = time.perf_counter()
        h2d.synchronize()  # the encoded frames and offsets are on the device
        timeline.add("h2d_wait", "h2d", t_w, time.perf_counter(), bytes=c_n)
        return
    if direct is not None:
        native.stream_sync(dev, slot)
        timeline.add("dec_wait", "h2d", t2, time.perf_counter(), bytes=c_n)
        err.check(f"frames [{first}, {last})")
        return
    shift = span.lo - log_lo
    # one stream sync for decode + copy (a failed restore leaves its targets
    # undefined either way, as on the host path)
    _copy_regions(out[shift:], regions, dev, slot)
    err.check(f"frames [{first}, {last})")


def _contiguous_src_range(src_dtype: torch.dtype, src_shape: Sequence[int], off: int, narrows):
    """(byte offset, nbytes) of a region's source when it is one contiguous
    byte range of the host buffer, else None (computed on the meta device)."""
    src = torch.empty(list(src_shape), dtype=src_dtype, device="meta")
    if narrows:
        for d, s, ln in narrows:
            src = src.narrow(d, s, ln)
    if not src.is_contiguous():
        return None
    es = src.element_size()
    return off + src.storage_offset() * es, src.numel() * es


def host_view_as_tensor(buf, dtype: torch.dtype, shape: Sequence[int]) -> torch.Tensor:
    return tensor_from_bytes(buf, dtype, shape)


def staged_from_tensor_storage(t: torch.Tensor) -> Optional[StagedBuffer]:
    """Writable host destination aliasing a contiguous CPU tensor's bytes."""
    if t.device.type != "cpu" or not t.is_contiguous() or t.is_quantized:
        return None
    if t.numel() == 0:
        return None
    mv = memoryview(t.detach().reshape(-1).view(torch.uint8).numpy()).cast("B")
    return StagedBuffer(mv, addr=t.data_ptr(), keepalive=t)


def host_buffer_addr(buf) -> int:
    if isinstance(buf, StagedBuffer):
        return buf.addr
    return buffer_address(buf)
