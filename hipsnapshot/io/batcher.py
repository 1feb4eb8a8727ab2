"""Small-write coalescing into slabs, and read-side range merging.

Reference: `/root/reference/torchsnapshot/batcher.py:30-482`.  Same planning rules
(buffer-protocol tensors without a prepare func, smaller than the slab
threshold, packed into ~threshold-sized ``batched/<uuid4>`` slabs separately for
host and device tensors, entries relocated in place with ``byte_range``) but a
different data path:

* device slabs are filled by ONE ``hs_copy_nd`` gather launch into an HBM slab
  and leave with ONE SDMA transfer into pinned memory (reference: allocate,
  one DtoD per member, pageable ``.cpu()``);
* members are placed at ``slab_align()``-byte offsets (256 B default) so every
  member starts on a 16-B boundary and the gather kernel uses dwordx4 for all
  of them; readers only ever use ``byte_range`` so this is format-compatible;
* on read, all ranges of one file are merged into one read; CUDA members of
  the merged buffer are restored by one H2D + one scatter launch; the
  consuming cost counts the merged buffer (reference under-counted it,
  Appendix C #3).
"""

from __future__ import annotations

import os
import time
import uuid
from collections import defaultdict
from concurrent.futures import Executor
from typing import Dict, List, Optional, Tuple

import torch

from .. import knobs
from ..engine import staging
from ..utils.tracing import timeline
from ..format.manifest import Entry, iter_tensor_entries
from ..format.serialization import SER
from ..io_types import (BufferConsumer, BufferStager, CompressedSpan, ReadReq, StagedBuffer,
                        WriteReq)
from .tensor import TensorBufferStager, run_in_executor


def is_batchable(stager: BufferStager) -> bool:
    return (isinstance(stager, TensorBufferStager)
            and stager.entry.serializer == SER.BUFFER_PROTOCOL
            and stager._tensor_prepare_func is None)


def _align(n: int, a: int) -> int:
    return (n + a - 1) // a * a


class Slab:
    def __init__(self, device: Optional[torch.device], name: Optional[str] = None) -> None:
        self.device = device
        self.members: List[Tuple[Tuple[int, int], TensorBufferStager]] = []
        # Deterministic names (``batched/<prefix>_<device>_<k>``) when the
        # caller provides a prefix: re-taking a snapshot to the same path then
        # overwrites its slabs like every other blob instead of leaking
        # uuid-named files; uuid4 names otherwise (reference behaviour).
        self.location = os.path.join("batched", name or str(uuid.uuid4()))
        self.sz_bytes = 0

    def add(self, nbytes: int, stager: TensorBufferStager, align: int) -> Tuple[int, int]:
        lo = _align(self.sz_bytes, align) if self.members else 0
        rng = (lo, lo + nbytes)
        self.members.append((rng, stager))
        self.sz_bytes = rng[1]
        return rng

    def build(self) -> BufferStager:
        if self.device is not None and self.device.type == "cuda":
            return GPUBatchedBufferStager(self.members, self.sz_bytes)
        return BatchedBufferStager(self.members, self.sz_bytes)


class BatchedBufferStager(BufferStager):
    """Host slab: members copied into one (pinned when available) buffer."""

    def __init__(self, members, total: int) -> None:
        self.members = members
        self.total = total
        self.codec: Optional[dict] = None

    thread_staging = True  # stage_buffer_sync may run on a scheduler worker

    async def stage_buffer(self, executor: Optional[Executor] = None):
        return await run_in_executor(executor, self._stage_sync)

    def stage_buffer_sync(self) -> StagedBuffer:
        return self._stage_sync()

    def _stage_sync(self) -> StagedBuffer:
        raw = self._gather()
        if self.codec is None:
            return raw
        try:
            return staging.encode_host_buffer(raw, self.codec)
        finally:
            raw.release()

    def _gather(self) -> StagedBuffer:
        from ..ops import native

        if native.gpu_available() and native.hsgpu_loaded():
            pb = native.PinnedBuffer(self.total)
            out = StagedBuffer(pb.view, pb.ptr, release=pb.release, keepalive=pb)
        else:
            ba = bytearray(self.total)
            out = StagedBuffer(memoryview(ba), keepalive=ba)
        u8 = torch.frombuffer(out.view, dtype=torch.uint8) if self.total else None
        for (lo, hi), st in self.members:
            t = st._source()
            if hi > lo:
                u8[lo:hi].view(t.dtype).view(t.shape).copy_(t)
        return out

    def get_staging_cost_bytes(self) -> int:
        return self.total


class GPUBatchedBufferStager(BufferStager):
    """Device slab: one gather kernel into HBM + one DMA into pinned memory."""

    def __init__(self, members, total: int) -> None:
        self.members = members
        self.total = total
        self.codec: Optional[dict] = None  # HSZ1 info when the slab is compressed
        self._pack_cache: dict = {}  # the gather launch's descriptor table (plan reuse)

    thread_staging = True

    async def stage_buffer(self, executor: Optional[Executor] = None):
        return await run_in_executor(executor, self._stage_sync)

    def stage_buffer_sync(self) -> StagedBuffer:
        return self._stage_sync()

    def _stage_sync(self) -> StagedBuffer:
        t0 = time.perf_counter()
        for ev in {id(st.wait_event): st.wait_event for _, st in self.members
                   if st.wait_event is not None}.values():
            ev.synchronize()
        producers = sorted({st.producer for _, st in self.members if st.producer is not None})
        pairs = [(st._source_view(), lo) for (lo, _hi), st in self.members]
        timeline.add("slab_sources", "stage", t0, time.perf_counter(), n=len(pairs))
        return staging.gather_to_host(pairs, self.total, producers,
                                      via_device_slab=knobs.use_gpu_gather_for_slabs(),
                                      codec=self.codec, pack_cache=self._pack_cache)

    def get_staging_cost_bytes(self) -> int:
        return self.total


def batch_write_requests(entries: List[Entry], write_reqs: List[WriteReq],
                         slab_size_threshold_bytes: Optional[int] = None,
                         name_prefix: Optional[str] = None
                         ) -> Tuple[List[Entry], List[WriteReq]]:
    threshold = slab_size_threshold_bytes or knobs.get_slab_size_threshold_bytes()
    align = knobs.slab_align()
    out: List[WriteReq] = []
    # Tail taper: slabs are staged after the big blobs (largest first), and
    # one file is written by one thread at ~10-15 GB/s (buffered writes to a
    # file serialize on its inode lock), while the DMA feeding the writes runs
    # at ~56 GB/s.  A slab staged when R batchable bytes remain must be written
    # before those R bytes have crossed PCIe (writes are ~5x slower per file),
    # so once fewer than 8 full slabs remain on a device, slabs close at an
    # eighth of what remains (a geometric taper down to 8 MiB).  With
    # equal-sized slabs the last big writes outlived the staging by ~4 ms:
    # the taper takes 1/8 off one rank's take at 8 GPUs (profiles/rank_share/).
    floor = min(threshold, max(threshold // 16, 8 << 20))  # smaller slabs gain nothing
    # batchable bytes per CUDA device index (-1: host) not placed yet
    remaining: Dict[int, int] = {}
    small = []  # (write request, stager, bytes, device index), in plan order
    bp = SER.BUFFER_PROTOCOL
    for wr in write_reqs:
        st = wr.buffer_stager
        if isinstance(st, TensorBufferStager) and st.entry.serializer == bp \
                and st._tensor_prepare_func is None:
            t = st.tensor
            nb = t.numel() * t.element_size()
            if nb < threshold:
                di = t.get_device()  # -1 for host tensors
                remaining[di] = remaining.get(di, 0) + nb
                small.append((wr, st, nb, di))
                continue
        out.append(wr)

    def _new_slab(di: int, k: int) -> Slab:
        dev = torch.device("cuda", di) if di >= 0 else None
        if name_prefix is None:
            return Slab(dev)
        return Slab(dev, f"{name_prefix}_{f'cuda{di}' if di >= 0 else 'cpu'}_{k}")

    slabs: Dict[int, List[Slab]] = {}
    moved = []  # (write request, stager, slab location, lo, hi)
    for wr, st, nb, di in small:
        left = remaining[di]
        remaining[di] = left - nb
        cap = threshold if left > 8 * threshold else max(floor, min(threshold, left // 8))
        lst = slabs.get(di)
        if lst is None:
            lst = slabs[di] = [_new_slab(di, 0)]
        slab = lst[-1]
        if slab.members and _align(slab.sz_bytes, align) + nb >= cap:
            slab = _new_slab(di, len(lst))
            lst.append(slab)
        lo, hi = slab.add(nb, st, align)
        moved.append((wr, st, slab.location, lo, hi))
    for lst in slabs.values():
        for slab in lst:
            if slab.members:
                out.append(WriteReq(path=slab.location, buffer_stager=slab.build()))
    by_location = None
    for wr, st, new_loc, lo, hi in moved:
        te = st.entry  # the manifest's entry object (the preparers share it)
        if te.location != wr.path:
            if by_location is None:
                by_location = {te.location: te for e in entries for te in iter_tensor_entries(e)}
            te = by_location.get(wr.path)
            if te is None:
                raise RuntimeError(
                    f"The tensor entry with the location {wr.path} is not passed to batch_write.")
        te.location = new_loc
        te.byte_range = [lo, hi]
    return entries, out


class BatchedBufferConsumer(BufferConsumer):
    """Consumes one merged ranged read that covers several entries.

    Members that restore into HBM (plain tensors, DTensor/ShardedTensor
    shards) expose ``device_regions``; all of them are served by ONE H2D DMA
    of the merged pinned buffer and ONE scatter/cast kernel launch per device.
    """

    def __init__(self, members: List[Tuple[Tuple[int, int], BufferConsumer]],
                 buf_sz_bytes: int) -> None:
        self.members = members
        self.buf_sz_bytes = buf_sz_bytes
        self._gpu = []
        self._other = []
        for rng, c in members:
            fn = getattr(c, "device_regions", None)
            regions = fn(rng[0]) if fn is not None else None
            if regions:
                self._gpu.append((rng, c, regions))
            else:
                self._other.append((rng, c))

    # reference-compatible attribute
    @property
    def byte_range_to_buffer_consumer(self):
        return {rng: c for rng, c in self.members}

    def get_read_dest(self, nbytes: int) -> Optional[StagedBuffer]:
        if self._gpu:
            from ..ops import native

            pb = native.PinnedBuffer(nbytes)
            return StagedBuffer(pb.view, pb.ptr, release=pb.release, keepalive=pb)
        return None

    def get_compressed_read_dest(self, nbytes: int) -> Optional[StagedBuffer]:
        return self.get_read_dest(nbytes)

    async def consume_buffer(self, buf, executor: Optional[Executor] = None) -> None:
        if isinstance(buf, CompressedSpan):
            if self._gpu:
                await run_in_executor(executor, self._consume_gpu, buf)
            if self._other:
                mv = await run_in_executor(executor, buf.decode_host)
                await self._consume_other(mv, executor)
            return
        mv = memoryview(buf.view if isinstance(buf, StagedBuffer) else buf).cast("B")
        if self._gpu:
            await run_in_executor(executor, self._consume_gpu, buf)
        await self._consume_other(mv, executor)

    async def _consume_other(self, mv: memoryview, executor: Optional[Executor]) -> None:
        """Host members: tensor consumers run back to back in ONE executor job
        (one thread hop per member cost ~0.15 ms each: 45 ms for the 291
        members of a Llama FSDP slab); other consumers keep their own path."""
        sync = [(rng, c) for rng, c in self._other
                if callable(getattr(c, "_consume_sync", None)) and not getattr(c, "_direct", False)]
        if sync:
            def run() -> None:
                for (lo, hi), c in sync:
                    c._consume_sync(mv[lo:hi])

            await run_in_executor(executor, run)
        ids = {id(c) for _, c in sync}
        for (lo, hi), c in self._other:
            if id(c) not in ids:
                await c.consume_buffer(mv[lo:hi], executor=executor)

    def _consume_gpu(self, buf) -> None:
        by_dev: Dict[int, list] = defaultdict(list)
        producers = {}
        for _rng, c, regions in self._gpu:
            dev = staging.device_of(regions[0][4])
            by_dev[dev].extend(regions)
            producers.setdefault(dev, getattr(c, "producer", None))
        for dev, regions in by_dev.items():
            if isinstance(buf, CompressedSpan):
                staging.scatter_compressed(buf, regions, dev, producers[dev])
            else:
                staging.scatter_host_regions(staging.host_buffer_addr(buf), self.buf_sz_bytes,
                                             regions, dev, producers[dev])

    def get_consuming_cost_bytes(self) -> int:
        return self.buf_sz_bytes + sum(c.get_consuming_cost_bytes() for _, c in self.members)


def batch_read_requests(read_reqs: List[ReadReq]) -> List[ReadReq]:
    out: List[ReadReq] = []
    grouped: Dict[str, List[ReadReq]] = defaultdict(list)
    for rr in read_reqs:
        if rr.byte_range is None or not rr.mergeable:
            out.append(rr)
        else:
            grouped[rr.path].append(rr)
    for path, rrs in grouped.items():
        if len(rrs) == 1:
            out.append(rrs[0])
            continue
        lo = min(r.byte_range[0] for r in rrs)
        hi = max(r.byte_range[1] for r in rrs)
        members = [((r.byte_range[0] - lo, r.byte_range[1] - lo), r.buffer_consumer) for r in rrs]
        out.append(ReadReq(path=path, byte_range=(lo, hi),
                           buffer_consumer=BatchedBufferConsumer(members, hi - lo),
                           codec=rrs[0].codec))
    return out
