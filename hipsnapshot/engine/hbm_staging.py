"""Async-take "freeze" of device state into spare HBM.

The reference makes ``async_take`` consistent by finishing every DtoH copy
before returning (`/root/reference/torchsnapshot/scheduler.py:330-337`), so the
trainer is blocked for state_bytes / PCIe bandwidth (>= 4.6 s for a full
288 GB MI355X at 63 GB/s).  MI355X has 288 GB of HBM3E per GPU and ~5-6 TB/s of
copy bandwidth, so instead:

1. every CUDA source of the pending write requests (plain tensors, chunk and
   shard views, members of device slabs -- strided or not) is described in
   ONE ``hs_copy_nd`` descriptor table;
2. one kernel launch on the trainer's current stream copies them all into a
   freshly allocated HBM arena (stream order makes the copy consistent with
   everything the trainer already enqueued and everything it enqueues later,
   without any host synchronisation);
3. the stagers are re-pointed at the arena (``frozen_at``; the views are
   built lazily by the drain) and wait on an event recorded after the launch;
   the background commit thread drains the arena to storage.

The arena holds every blob exactly as it will be stored (``frozen_region``
= (arena, offset, bytes) on the write request's stager): a tensor's C-order
bytes, or a device slab with its members at their slab offsets and the gaps
zero-filled by the same launch.  Raw blobs can then go arena -> file with no
gather, through the native drain (``engine/native_drain.py``).

When the whole state does not fit in free HBM minus
``HBM_STAGING_RESERVE_BYTES`` (or ``HBM_STAGING_MAX_BYTES``), write requests are
frozen greedily in plan order until the arena is full and the rest takes the
host-staging path before ``async_take`` returns: the time-to-unblock then
scales with the bytes that did NOT fit, instead of falling back wholesale.
"""

from __future__ import annotations

import logging
import time
import weakref
from collections import defaultdict
from typing import Dict, List, Optional, Tuple

import torch

from .. import knobs
from ..io_types import WriteReq
from ..ops import native
from ..utils.tracing import timeline

logger = logging.getLogger(__name__)

_ALIGN = 256

# (descriptor keepalive, completion event) of freeze launches that may still
# be queued on the trainer's stream.  The pinned descriptor block must not go
# back to the pool before the kernel has read it -- not even when the take
# fails and drops its stagers -- so it is held here until its event completes.
_live_launches: List[tuple] = []


def _retire_launches() -> None:
    _live_launches[:] = [kd for kd in _live_launches if not kd[1].query()]


_TYPES: Optional[tuple] = None


def _types() -> tuple:
    """(TensorBufferStager, GPUBatchedBufferStager, ObjectBufferStager),
    imported once: these run per write request on the unblock path."""
    global _TYPES
    if _TYPES is None:
        from ..io.batcher import GPUBatchedBufferStager
        from ..io.object import ObjectBufferStager
        from ..io.tensor import TensorBufferStager

        _TYPES = (TensorBufferStager, GPUBatchedBufferStager, ObjectBufferStager)
    return _TYPES


def _cuda_sources(wr: WriteReq):
    """The stagers whose CUDA tensors a write request reads (empty if none)."""
    TensorBufferStager, GPUBatchedBufferStager, _ = _types()
    st = wr.buffer_stager
    if isinstance(st, TensorBufferStager) and st.tensor.is_cuda \
            and st._tensor_prepare_func is None:
        return [st]
    if isinstance(st, GPUBatchedBufferStager):
        return [m for _, m in st.members]
    return []


def _nbytes(st) -> int:
    nb = st.tensor.numel() * st.tensor.element_size()
    return (nb + _ALIGN - 1) // _ALIGN * _ALIGN


def _region(wr: WriteReq, sts) -> Tuple[int, List[int], int]:
    """(arena bytes, member offsets in the region, blob bytes) of one write
    request.  The region holds the blob exactly as it goes to storage: a
    tensor's C-order bytes, or a device slab with every member at its slab
    offset (the gaps are zero-filled by the freeze)."""
    st = wr.buffer_stager
    if isinstance(st, _types()[1]):
        offs = [lo for (lo, _hi), _m in st.members]
        return (st.total + _ALIGN - 1) // _ALIGN * _ALIGN, offs, st.total
    t = sts[0].tensor
    return _nbytes(sts[0]), [0], t.numel() * t.element_size()


def _cached_unused(dev: int) -> int:
    """Bytes torch's caching allocator holds but does not use on ``dev``.
    One nested-stats call: ``memory_reserved`` and ``memory_allocated`` each
    flatten the whole statistics dict (~0.1 ms apiece on the unblock path)."""
    try:
        st = torch._C._cuda_memoryStats(dev)
        return int(st["reserved_bytes"]["all"]["current"]) - \
            int(st["allocated_bytes"]["all"]["current"])
    except (AttributeError, KeyError, TypeError):
        return torch.cuda.memory_reserved(dev) - torch.cuda.memory_allocated(dev)


ZERO_PAGE = 4096
_zero_page: list = []  # [PinnedBuffer]: kept for the life of the process


def zero_page_ptr() -> int:
    """Address of ZERO_PAGE zero bytes the copy kernel reads slab gaps from:
    a pinned host block (device-mapped), zeroed by the CPU.  (A torch.zeros
    on the device was the first launch of torch's fill kernel in some
    processes: 15 ms of a cold async_take, spent loading its code object.)"""
    if not _zero_page:
        import ctypes

        pb = native.PinnedBuffer(ZERO_PAGE)
        ctypes.memset(pb.ptr, 0, ZERO_PAGE)
        _zero_page.append(pb)
    return _zero_page[0].ptr


def add_zero_fill(batch, dst: int, nbytes: int) -> None:
    """Zero ``nbytes`` at device address ``dst`` within ``batch``'s launch."""
    zero = zero_page_ptr()
    while nbytes > 0:
        n = min(nbytes, ZERO_PAGE)
        batch.add_bytes(zero, dst, n)
        dst += n
        nbytes -= n


def _layout(write_reqs: List[WriteReq]) -> Dict[int, list]:
    """device -> [(region bytes, member offsets, blob bytes, wr, stagers)]."""
    by_dev = defaultdict(list)
    for wr in write_reqs:
        if wr.buffer_stager.__dict__.get("captured") is not None:
            continue  # copied by the CPU (engine/uvm_capture.py)
        sts = _cuda_sources(wr)
        if not sts:
            continue
        t = sts[0].tensor
        dev = t.device.index if t.device.index is not None else torch.cuda.current_device()
        by_dev[dev].append((*_region(wr, sts), wr, sts))
    return by_dev


def _plan_layout(write_reqs: List[WriteReq], plan) -> Dict[int, list]:
    """The layout of a reused take plan's requests is the same every take
    (same tensors, same slabs): computed once and kept on the plan.  Requests
    outside the plan (host tensors, objects) are scanned as usual."""
    cache = getattr(plan, "freeze_layout", None)
    if cache is None:
        ids = {id(wr) for wr in plan.write_reqs}
        cache = plan.freeze_layout = {"ids": ids, "layout": _layout(plan.write_reqs),
                                      "launch": {}}
    ids = cache["ids"]
    extra = _layout([wr for wr in write_reqs if id(wr) not in ids])
    base = cache["layout"]
    if any(r[3].buffer_stager.__dict__.get("captured") is not None
           for v in base.values() for r in v):
        # tables the CPU captures this take (engine/uvm_capture.py) stay out
        base = {d: [r for r in v if r[3].buffer_stager.__dict__.get("captured") is None]
                for d, v in base.items()}
        base = {d: v for d, v in base.items() if v}
    if not extra:
        return base
    merged = defaultdict(list, {d: list(v) for d, v in base.items()})
    for d, v in extra.items():
        merged[d].extend(v)
    return merged


def freeze_device_state(write_reqs: List[WriteReq], plan=None,
                        keep: Optional[set] = None) -> Dict[int, int]:
    """Returns {device: arena_bytes} for the devices that were (partly) frozen.
    ``plan``: the reused take plan the requests come from (layout and the
    freeze launch's descriptor table are cached on it).  ``keep``: ids of
    stagers a reused plan must not reset (taken over by a UVM capture)."""
    if not native.gpu_available():
        return {}
    if plan is not None:
        plan.mutated = True  # its stagers are re-pointed at the arena below
    for wr in write_reqs:
        # a previous take's region (reused plan) never carries over
        wr.buffer_stager.__dict__.pop("frozen_region", None)
        wr.buffer_stager.__dict__.pop("frozen_event", None)
    with timeline.span("freeze_layout"):
        by_dev = _plan_layout(write_reqs, plan) if plan is not None else _layout(write_reqs)
    launch_cache = plan.freeze_layout["launch"] if plan is not None else None
    frozen = {}
    placed: set = set(keep or ())  # ids of the stagers re-pointed at an arena below
    try:
        _freeze_devices(by_dev, launch_cache, frozen, placed)
    finally:
        if plan is not None and plan.pending_reset:
            plan.reset_except(placed)
    return frozen


def _freeze_devices(by_dev, launch_cache, frozen: Dict[int, int], placed: set) -> None:
    cap = knobs.hbm_staging_max_bytes()
    for dev, reqs in by_dev.items():
        want = sum(r[0] for r in reqs)
        kept = _kept.get(dev)
        if kept is not None and not kept[1] and kept[0].numel() >= want and want <= cap:
            # the idle kept arena holds everything: no room estimate needed
            try:
                _freeze(dev, reqs, want, launch_cache, placed)
            except torch.cuda.OutOfMemoryError:
                logger.info(f"HBM staging on cuda:{dev}: arena of {want} B not allocatable")
                continue
            frozen[dev] = want
            continue
        with timeline.span("freeze_room"):
            free, _ = torch.cuda.mem_get_info(dev)
            # blocks torch's caching allocator holds but does not use are free
            # for the arena too (the allocator releases them and retries when
            # a fresh allocation does not fit) -- a trainer's cache is often
            # tens of GB
            cached = _cached_unused(dev)
        kept = _kept.get(dev)
        kept_bytes = kept[0].numel() if kept is not None and not kept[1] else 0
        room = min(free + max(cached, 0) + kept_bytes - knobs.hbm_staging_reserve_bytes(), cap)
        want = sum(r[0] for r in reqs)
        chosen, total = [], 0
        for r in reqs:
            if total + r[0] <= room:
                chosen.append(r)
                total += r[0]
        if not chosen:
            logger.info(f"HBM staging skipped on cuda:{dev}: need {want} B, room {room} B")
            continue
        if total < want:
            logger.info(f"HBM staging on cuda:{dev}: {total} of {want} B frozen, the rest "
                        "is staged to host before async_take returns")
        try:
            _freeze(dev, chosen, total, launch_cache if len(chosen) == len(reqs) else None,
                    placed)
        except torch.cuda.OutOfMemoryError:
            # fragmentation: the estimate above was optimistic -> host path
            logger.info(f"HBM staging on cuda:{dev}: arena of {total} B not allocatable")
            continue
        frozen[dev] = total


# Arena kept between async takes (knobs.TUNING.hbm_arena_keep): device ->
# [tensor, busy].  A training loop frees and re-allocates activations between
# checkpoints; a 48 GB arena handed back to torch's caching allocator gets
# split up by them, and the next take's torch.empty then goes through
# hipMalloc -- or frees cached blocks first -- right while a training step is
# queued (a ~200 ms step stall measured on Llama-3-8B + AdamW,
# profiles/r3/overlap/).  Kept, the next take reuses it as it is.
_kept: Dict[int, list] = {}


# device -> (event before, event after) the last freeze launch
_last_freeze: Dict[int, tuple] = {}


def last_freeze_ms(dev: int = 0) -> Optional[float]:
    """GPU time of the last async-take freeze launch on ``dev`` (waits for
    it): what the trainer's stream spends on the copy itself."""
    ev = _last_freeze.get(dev)
    if ev is None:
        return None
    ev[1].synchronize()
    return float(ev[0].elapsed_time(ev[1]))


# arena data_ptr -> the stagers whose frozen_at / frozen_region view it (a
# reused take plan keeps its stagers, and with them the arena, alive)
_holders: Dict[int, "weakref.WeakSet"] = {}


def _unpin(ptr: int) -> None:
    """Clear every stager reference into the arena at ``ptr`` (its drain is
    over): dropping the kept arena then really frees it."""
    for st in list(_holders.pop(ptr, ())):
        fa = st.__dict__.get("frozen_at")
        if fa is not None and fa[0].data_ptr() == ptr:
            st.frozen_at = None
            st.frozen = False
            st.wait_event = None
            st.__dict__.pop("arena_keepalive", None)
        fr = st.__dict__.get("frozen_region")
        if fr is not None and fr[0].data_ptr() == ptr:
            st.__dict__.pop("frozen_region", None)
            st.__dict__.pop("frozen_event", None)


def _drop_kept(t: torch.Tensor) -> None:
    _unpin(t.data_ptr())


def _arena(dev: int, total: int) -> torch.Tensor:
    k = _kept.get(dev)
    if k is not None and not k[1] and k[0].numel() >= total:
        k[1] = True
        return k[0][:max(total, 1)]
    if k is not None and not k[1]:
        _drop_kept(k[0])  # a smaller idle one is dropped
        del _kept[dev]
        k = None
    arena = torch.empty(max(total, 1), dtype=torch.uint8, device=f"cuda:{dev}")
    if knobs.hbm_arena_keep() and k is None:
        _kept[dev] = [arena, True]
    return arena


def is_kept(arena: torch.Tensor) -> bool:
    """Is ``arena`` (or a view at its start) the kept arena of its device?"""
    k = _kept.get(arena.device.index if arena.device.index is not None else 0)
    return k is not None and k[0].data_ptr() == arena.data_ptr()


def arena_done(arenas) -> None:
    """The drain of these arenas finished: a kept arena may be reused -- or
    is dropped when the trainer's headroom fell below the reserve
    (engine/memory.py)."""
    from . import memory

    for a in arenas:
        for dev, k in list(_kept.items()):
            if k[1] and a.data_ptr() == k[0].data_ptr():
                k[1] = False
                memory.settle_arena(dev)


def release_hbm_arena() -> int:
    """Drop the idle kept arenas (back to torch's caching allocator); returns
    the bytes released.  Busy ones (a drain still running) are kept."""
    freed = 0
    for dev in list(_kept):
        if not _kept[dev][1]:
            t = _kept.pop(dev)[0]
            _drop_kept(t)
            freed += t.numel()
    return freed


def _freeze(dev: int, chosen, total: int, launch_cache: Optional[dict] = None,
            placed_ids: Optional[set] = None) -> None:
    _retire_launches()
    stream = torch.cuda.current_stream(dev)
    with torch.cuda.device(dev):
        with timeline.span("freeze_alloc", bytes=total):
            arena = _arena(dev, total)
        base = arena.data_ptr()
        # a reused plan into the same arena launches the very same copies:
        # keep the packed descriptor table (sources = the plan's tensors,
        # unchanged by construction of plan reuse; destinations = this arena)
        key = (dev, base, total, len(chosen))
        hit = launch_cache.get(dev) if launch_cache is not None else None
        if hit is not None and hit[0] == key:
            arr, placed, regions = hit[1], hit[2], hit[3]
            for (wr, off, blob) in regions:
                wr.buffer_stager.frozen_region = (arena, off, blob)
        else:
            batch = native.CopyBatch()
            placed = []  # (stager, arena offset)
            regions = []  # (write request, arena offset, blob bytes)
            off = 0
            for region, moffs, blob, wr, sts in chosen:
                end = 0
                for st, mo in zip(sts, moffs):
                    if mo > end:  # slab gap: zeros, as the slab gather writes them
                        add_zero_fill(batch, base + off + end, mo - end)
                    t = st.tensor  # (only its pointer and layout are read: no detach)
                    if t.numel():
                        batch.add_tensor(t, base + off + mo)
                    placed.append((st, off + mo))
                    end = mo + t.numel() * t.element_size()
                wr.buffer_stager.frozen_region = (arena, off, blob)
                regions.append((wr, off, blob))
                off += region
            with timeline.span("copy_pack", n=len(batch)):
                arr = batch.pack()
            if launch_cache is not None:
                launch_cache[dev] = (key, arr, placed, regions)
        sts_all = [st for st, _ in placed]
        t_ev = time.perf_counter()
        # producers may differ from the current stream: order after them
        for p in {st.producer for st in sts_all if st.producer is not None}:
            if p != stream.cuda_stream:
                ev = torch.cuda.Event()
                ev.record(torch.cuda.default_stream(dev) if p == 0
                          else torch.cuda.ExternalStream(p))
                stream.wait_event(ev)
        t_start = torch.cuda.Event(enable_timing=True)
        t_start.record(stream)
        with timeline.span("freeze_launch", n=len(sts_all)):
            keep = native.launch_packed(arr, dev, int(stream.cuda_stream), sync=False)
        done = torch.cuda.Event(enable_timing=True)
        done.record(stream)
        _last_freeze[dev] = (t_start, done)
        timeline.add("freeze_events", "stage", t_ev, time.perf_counter())
    _live_launches.append((keep, done))
    done_keep = (keep, done)
    if is_kept(arena):
        holders = _holders.setdefault(base, weakref.WeakSet())
        holders.update(st for st, _ in placed)
        holders.update(r[0].buffer_stager for r in regions)
    if placed_ids is not None:
        placed_ids.update(id(st) for st, _ in placed)
    for st, o in placed:
        st.frozen_at = (arena, o)  # _source() views the arena from now on
        st.producer = None  # ordering is carried by wait_event
        st.frozen = True
        st.wait_event = done
        # keep the descriptor tables alive until the copy ran
        st.arena_keepalive = done_keep
    for _r, _m, _b, wr, _s in chosen:
        wr.buffer_stager.frozen_event = done


def is_deferrable(wr: WriteReq) -> bool:
    """A write whose bytes are already captured (frozen HBM copy or eagerly
    serialized object) can run entirely after ``async_take`` returns."""
    TensorBufferStager, GPUBatchedBufferStager, ObjectBufferStager = _types()
    st = wr.buffer_stager
    if isinstance(st, ObjectBufferStager):
        return True
    if isinstance(st, TensorBufferStager):
        return st.frozen
    if isinstance(st, GPUBatchedBufferStager):
        return all(m.frozen for _, m in st.members)
    return False
