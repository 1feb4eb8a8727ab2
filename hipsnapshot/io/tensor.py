"""Plain-tensor write/read planning: ``TensorEntry`` + stager + consumer.

Behavioural reference: `/root/reference/torchsnapshot/io_preparers/tensor.py:47-403`
(serializer choice, in-place load when dtype+shape match, tiled reads under a
buffer limit, quantized-aware ``tensor_copy``).  What is different:

* staging of CUDA tensors goes through ``engine.staging`` (pinned pool + SDMA
  on a side stream, or the pack kernel for strided views), never pageable
  ``.cpu()``;
* async snapshots copy EVERY host tensor before returning (the reference's
  enum-vs-string comparison made that copy dead code);
* ``_tensor_prepare_func`` output is what gets staged (reference staged the
  original tensor, Appendix C #2);
* reads land directly in the destination: CPU targets are filled in place by
  the storage engine (no intermediate buffer), CUDA targets get a pinned
  buffer followed by DMA (+ cast kernel when the dtype/strides differ);
* opt-in ``hipsnapshot_fp8_block`` serializer (GPU fp8 quantized save).
"""

from __future__ import annotations

import asyncio
import math
from concurrent.futures import Executor
from typing import Any, Callable, List, Optional, Tuple, Union

import torch

from ..format.manifest import ChunkedTensorEntry, TensorEntry
from ..format.serialization import (
    SUPPORTED_QUANTIZED_DTYPES,
    SER,
    dtype_to_element_size,
    dtype_to_string,
    is_buffer_protocol_dtype,
    string_to_dtype,
    tensor_from_bytes,
    torch_load_from_bytes,
    torch_save_as_bytes,
)
from ..io_types import (BufferConsumer, BufferStager, CompressedSpan, Future, ReadReq,
                        StagedBuffer, WriteReq)
from ..engine import staging

PrepareFunc = Callable[[torch.Tensor, bool], torch.Tensor]

# reads above this size are split into AUTO_TILE_BYTES ranged reads that run
# concurrently on the I/O engine and overlap with the H2D DMA of earlier tiles
AUTO_TILE_THRESHOLD_BYTES = 256 << 20
AUTO_TILE_BYTES = 64 << 20


async def run_in_executor(executor: Optional[Executor], fn, *args):
    if executor is None:
        return fn(*args)
    return await asyncio.get_running_loop().run_in_executor(executor, fn, *args)


def tensor_nbytes_from_entry(entry: Union[TensorEntry, ChunkedTensorEntry]) -> int:
    n = 1
    for s in entry.shape:
        n *= int(s)
    return n * dtype_to_element_size(string_to_dtype(entry.dtype))


def is_uvm_like(t: torch.Tensor) -> bool:
    from ..ops.uvm import is_uvm_tensor

    return is_uvm_tensor(t)


class TensorIOPreparer:
    @staticmethod
    def prepare_write(storage_path: str, tensor: torch.Tensor, is_async_snapshot: bool = False,
                      _tensor_prepare_func: Optional[PrepareFunc] = None,
                      serializer: Optional[str] = None) -> Tuple[TensorEntry, List[WriteReq]]:
        proc = tensor if _tensor_prepare_func is None else _tensor_prepare_func(tensor, True)
        if proc.shape != tensor.shape:
            raise RuntimeError(
                "_tensor_prepare_func shouldn't change the tensor's shape "
                f"(changed from {tensor.shape} to {proc.shape}).")
        quant = None
        if serializer == SER.FP8_BLOCK:
            from ..ops.quant import fp8_entry_quant_info, fp8_supported

            if not fp8_supported(proc):
                serializer = None
            else:
                quant = fp8_entry_quant_info(proc)
        if serializer is None:
            serializer = (SER.BUFFER_PROTOCOL if is_buffer_protocol_dtype(proc.dtype)
                          else SER.TORCH_SAVE)
        entry = TensorEntry(location=storage_path, serializer=serializer,
                            dtype=dtype_to_string(proc.dtype), shape=list(proc.shape),
                            replicated=False, quant=quant)
        stager = TensorBufferStager(tensor=tensor, entry=entry,
                                    is_async_snapshot=is_async_snapshot,
                                    _tensor_prepare_func=_tensor_prepare_func)
        return entry, [WriteReq(path=storage_path, buffer_stager=stager)]

    @classmethod
    def prepare_read(cls, entry: TensorEntry, tensor_out: Optional[torch.Tensor] = None,
                     buffer_size_limit_bytes: Optional[int] = None
                     ) -> Tuple[List[ReadReq], Future]:
        if tensor_out is None or not cls.can_load_inplace(entry, tensor_out):
            if entry.serializer == SER.TORCH_SAVE:
                # the payload carries its own tensor (quantized params etc.):
                # hand the loaded object out instead of pre-allocating
                fut = Future()
                consumer = TensorBufferConsumer(tensor=None, entry=entry, future=fut)
                return [ReadReq(path=entry.location, byte_range=entry.byte_range_tuple,
                                buffer_consumer=consumer, codec=entry.codec)], fut
            tensor_out = cls.empty_tensor_from_entry(entry)
        if entry.serializer == SER.BUFFER_PROTOCOL and entry.codec is None:
            if buffer_size_limit_bytes is not None:
                return cls.prepare_read_tiled(entry, tensor_out, buffer_size_limit_bytes)
            if tensor_nbytes_from_entry(entry) > AUTO_TILE_THRESHOLD_BYTES:
                # large blobs: parallel ranged reads pipelined with H2D
                return cls.prepare_read_tiled(entry, tensor_out, AUTO_TILE_BYTES)
        consumer = TensorBufferConsumer(tensor=tensor_out, entry=entry)
        return [ReadReq(path=entry.location, byte_range=entry.byte_range_tuple,
                        buffer_consumer=consumer, codec=entry.codec)], Future(obj=tensor_out)

    @classmethod
    def prepare_read_tiled(cls, entry: TensorEntry, tensor_out: torch.Tensor,
                           buffer_size_limit_bytes: int) -> Tuple[List[ReadReq], Future]:
        """Split one blob into byte-ranged reads of <= limit bytes (dim-0 tiles
        of the flattened tensor when it is viewable as 1-D, else dim-0 chunks)."""
        total = tensor_nbytes_from_entry(entry)
        n_chunks = max(1, math.ceil(total / max(buffer_size_limit_bytes, 1)))
        target = tensor_out
        try:
            target = tensor_out.view(-1)
        except RuntimeError:
            pass
        es = dtype_to_element_size(string_to_dtype(entry.dtype))
        chunks = torch.chunk(target, chunks=n_chunks, dim=0) if target.numel() else [target]
        base = entry.byte_range[0] if entry.byte_range is not None else 0
        offset = 0
        reqs = []
        for ch in chunks:
            nb = ch.numel() * es
            sub = TensorEntry(location=entry.location, serializer=entry.serializer,
                              dtype=entry.dtype, shape=list(ch.shape),
                              replicated=entry.replicated)
            reqs.append(ReadReq(path=entry.location,
                                byte_range=(base + offset, base + offset + nb),
                                buffer_consumer=TensorBufferConsumer(tensor=ch, entry=sub),
                                mergeable=False))
            offset += nb
        return reqs, Future(obj=tensor_out)

    @staticmethod
    def get_tensor_size_from_entry(entry) -> int:
        return tensor_nbytes_from_entry(entry)

    @staticmethod
    def can_load_inplace(entry: Union[TensorEntry, ChunkedTensorEntry], obj: Any) -> bool:
        if not isinstance(obj, torch.Tensor) or _is_dtensor(obj):
            return False
        return string_to_dtype(entry.dtype) == obj.dtype and list(entry.shape) == list(obj.shape)

    @staticmethod
    def empty_tensor_from_entry(entry: Union[TensorEntry, ChunkedTensorEntry]) -> torch.Tensor:
        dtype = string_to_dtype(entry.dtype)
        if dtype in SUPPORTED_QUANTIZED_DTYPES:
            raise RuntimeError("Allocating an empty quantized tensor is not supported yet.")
        return torch.empty(list(entry.shape), dtype=dtype)


def _is_dtensor(t) -> bool:
    try:
        from torch.distributed.tensor import DTensor
    except Exception:  # pragma: no cover
        return False
    return isinstance(t, DTensor)


class TensorBufferStager(BufferStager):
    def __init__(self, tensor: torch.Tensor, entry: TensorEntry, is_async_snapshot: bool,
                 _tensor_prepare_func: Optional[PrepareFunc] = None) -> None:
        self.tensor = tensor
        self._plan_tensor = tensor  # what the plan saves (``tensor`` may be re-pointed)
        self.entry = entry
        self.is_async_snapshot = is_async_snapshot
        self._tensor_prepare_func = _tensor_prepare_func
        self.producer = staging.producer_stream_handle(tensor)
        # set by the async-take HBM snapshot: tensor already copied to an
        # arena that nobody else mutates -> no extra host copy needed
        self.frozen = False
        self.wait_event = None  # torch.cuda.Event guarding a frozen HBM copy
        # (arena, byte offset) of the frozen copy; the view is built lazily
        # in the drain so async_take does not pay ~4 us per tensor for it
        self.frozen_at: Optional[Tuple[torch.Tensor, int]] = None
        self.codec: Optional[dict] = None  # HSZ1 info when the blob is compressed

    def reset_for_reuse(self) -> None:
        """Back to the planned state for a later take (engine/plan_cache.py):
        undo an async HBM freeze or UVM capture and order after the caller's
        current stream."""
        cap = self.__dict__.pop("captured", None)
        if cap is not None:
            cap[0].drop(cap[1])
        self.tensor = self._plan_tensor
        self.frozen = False
        self.wait_event = None
        self.frozen_at = None
        self.__dict__.pop("arena_keepalive", None)
        self.producer = staging.producer_stream_handle(self.tensor)

    def _source_view(self) -> torch.Tensor:
        """The source for pointer-only consumers (the slab gather kernel):
        the tensor itself when no prepare func or frozen copy is involved
        (``_source``'s ``detach`` costs ~8 us per member under load)."""
        if self.frozen_at is None and self._tensor_prepare_func is None:
            return self.tensor
        return self._source()

    def _source(self) -> torch.Tensor:
        if self.frozen_at is not None:
            arena, off = self.frozen_at
            t = self.tensor
            return arena[off: off + t.numel() * t.element_size()].view(t.dtype).view(t.shape)
        t = self.tensor
        if self._tensor_prepare_func is not None:
            t = self._tensor_prepare_func(t, False)
        return t.detach()

    async def stage_buffer(self, executor: Optional[Executor] = None):
        if self._tensor_prepare_func is not None:
            # the user's prepare func runs on the event-loop thread, as in the
            # reference; only the copy goes to the executor
            t = self._source()
            return await run_in_executor(executor, self._stage_source, t)
        return await run_in_executor(executor, self.stage_buffer_sync)

    @property
    def thread_staging(self) -> bool:
        """``stage_buffer_sync`` may run on a scheduler worker thread."""
        return self._tensor_prepare_func is None

    def stage_buffer_sync(self):
        cap = self.__dict__.get("captured")
        if cap is not None:  # an async take's CPU copy of a host UVM table
            return cap[0].buffer(cap[1])
        return self._stage_source(self._source())

    def _stage_source(self, t: torch.Tensor):
        ser = self.entry.serializer
        if ser == SER.BUFFER_PROTOCOL:
            if t.is_cuda:
                return self._d2h(t)
            # async snapshots must not alias live host memory (Appendix C #1);
            # a prepare-func result that owns fresh storage needs no copy.
            fresh = (self._tensor_prepare_func is not None
                     and t.untyped_storage().data_ptr()
                     != self.tensor.untyped_storage().data_ptr())
            copy = self.is_async_snapshot and not self.frozen and not fresh
            if self.codec is not None:
                return self._encode_host(t)
            return staging.cpu_tensor_bytes(t, copy)
        if ser == SER.FP8_BLOCK:
            from ..ops.quant import stage_fp8

            return stage_fp8(t, self.entry, self.producer)
        if ser == SER.TORCH_SAVE:
            return _torch_save_tensor(t)
        raise ValueError(f"Unrecognized serializer: {ser}.")

    def _encode_host(self, t: torch.Tensor):
        raw = staging.cpu_tensor_bytes(t, copy=False)
        try:
            return staging.encode_host_buffer(raw, self.codec)
        finally:
            raw.release()

    def _d2h(self, t: torch.Tensor):
        if self.wait_event is not None:
            self.wait_event.synchronize()
        # a blocking take may write host-resident UVM pages in place
        return staging.d2h_tensor(t, self.producer, codec=self.codec,
                                  alias_ok=not self.is_async_snapshot)

    def get_staging_cost_bytes(self) -> int:
        n = tensor_nbytes_from_entry(self.entry)
        return 2 * n if self.entry.serializer == SER.TORCH_SAVE else n


def _torch_save_tensor(t: torch.Tensor) -> bytes:
    if t.is_cuda:
        t = t.cpu()
    elif t.numel() != t.untyped_storage().nbytes() // max(t.element_size(), 1):
        # a view of a larger storage: torch.save would write the whole storage
        t = t.clone()
    return torch_save_as_bytes(t)


def deserialize_tensor(buf, entry: TensorEntry) -> torch.Tensor:
    if entry.serializer == SER.TORCH_SAVE:
        # tensor payloads (complex / quantized dtypes) load weights-only
        return torch_load_from_bytes(buf, trusted=False)
    if entry.serializer == SER.BUFFER_PROTOCOL:
        return tensor_from_bytes(buf, string_to_dtype(entry.dtype), entry.shape)
    if entry.serializer == SER.FP8_BLOCK:
        from ..ops.quant import dequantize_host_fp8

        return dequantize_host_fp8(buf, entry)
    if entry.serializer == SER.PER_TENSOR_QTENSOR:
        from ..format.serialization import per_tensor_qtensor_from_bytes

        return per_tensor_qtensor_from_bytes(buf)
    if entry.serializer == SER.PER_CHANNEL_QTENSOR:
        from ..format.serialization import per_channel_qtensor_from_bytes

        return per_channel_qtensor_from_bytes(buf)
    raise ValueError(f"Unrecognized serializer: {entry.serializer}.")


class TensorBufferConsumer(BufferConsumer):
    def __init__(self, tensor: Optional[torch.Tensor], entry: TensorEntry,
                 future: Optional[Future] = None) -> None:
        self.tensor = tensor
        self.entry = entry
        self.future = future
        self.producer = staging.producer_stream_handle(tensor) if tensor is not None else None
        self._direct = False

    def _nbytes(self) -> int:
        return tensor_nbytes_from_entry(self.entry)

    def _fp8_on_device(self) -> bool:
        t = self.tensor
        return (t is not None and t.is_cuda and self.entry.serializer == SER.FP8_BLOCK
                and t.is_contiguous() and t.dtype == string_to_dtype(self.entry.dtype))

    def get_read_dest(self, nbytes: int) -> Optional[StagedBuffer]:
        if self._fp8_on_device():
            from ..ops import native

            pb = native.PinnedBuffer(nbytes)
            return StagedBuffer(pb.view, pb.ptr, release=pb.release, keepalive=pb)
        if self.entry.serializer != SER.BUFFER_PROTOCOL or self.tensor is None:
            return None
        t = self.tensor
        if (not t.is_cuda and t.dtype == string_to_dtype(self.entry.dtype)
                and nbytes == self._nbytes() and list(t.shape) == list(self.entry.shape)):
            dest = staging.staged_from_tensor_storage(t)
            if dest is not None:
                self._direct = True
                return dest
        if (t.is_cuda and t.is_contiguous() and t.dtype == string_to_dtype(self.entry.dtype)
                and nbytes == self._nbytes() and list(t.shape) == list(self.entry.shape)
                and nbytes and staging.host_resident_managed(t)):
            # UVM pages in host DRAM: read the file straight into them
            self._direct = True
            return staging.managed_host_view(t, self.producer)
        if t.is_cuda:
            from ..ops import native

            pb = native.PinnedBuffer(nbytes)
            return StagedBuffer(pb.view, pb.ptr, release=pb.release, keepalive=pb)
        return None

    def get_compressed_read_dest(self, nbytes: int) -> Optional[StagedBuffer]:
        t = self.tensor
        if t is not None and t.is_cuda and self.entry.serializer == SER.BUFFER_PROTOCOL:
            from ..ops import native

            pb = native.PinnedBuffer(nbytes)
            return StagedBuffer(pb.view, pb.ptr, release=pb.release, keepalive=pb)
        return None

    async def consume_buffer(self, buf, executor: Optional[Executor] = None) -> None:
        if self._direct:
            return  # bytes were read straight into the destination tensor
        await run_in_executor(executor, self._consume_sync, buf)

    def _consume_sync(self, buf) -> None:
        t = self.tensor
        if isinstance(buf, CompressedSpan):
            if (t is not None and t.is_cuda
                    and self.entry.serializer == SER.BUFFER_PROTOCOL):
                staging.scatter_compressed(
                    buf, [(string_to_dtype(self.entry.dtype), self.entry.shape, 0, None, t)],
                    staging.device_of(t), self.producer)
                return
            buf = buf.decode_host()
        if t is None:
            self.future.obj = deserialize_tensor(buf, self.entry)
            return
        if self._fp8_on_device() and isinstance(buf, StagedBuffer):
            # raw blob -> HBM by DMA, dequantized on the GPU into the target
            from ..ops import native
            from ..ops.quant import dequantize_device

            dev = staging.device_of(t)
            total = self.entry.quant["total_bytes"]
            blob = torch.empty(total, dtype=torch.uint8, device=t.device)
            # order after the allocator's stream (and the target's producer)
            native.memcpy(dev, staging.copy_slot(), blob.data_ptr(), buf.addr, total, native.H2D,
                          int(torch.cuda.current_stream(t.device).cuda_stream), sync=True)
            dequantize_device(blob, self.entry, t)
            torch.cuda.current_stream(t.device).synchronize()
            return
        if (t.is_cuda and self.entry.serializer == SER.BUFFER_PROTOCOL):
            staging.h2d_into(t, staging.host_buffer_addr(buf), self._nbytes(),
                             string_to_dtype(self.entry.dtype), self.entry.shape, self.producer)
            return
        loaded = deserialize_tensor(buf, self.entry)
        tensor_copy(t, loaded)

    def get_consuming_cost_bytes(self) -> int:
        n = self._nbytes()
        return 2 * n if self.entry.serializer == SER.TORCH_SAVE else n

    def device_regions(self, base: int):
        """Scatter regions for a merged (batched) GPU restore, or None."""
        t = self.tensor
        if (t is not None and t.is_cuda
                and self.entry.serializer == SER.BUFFER_PROTOCOL and t.dim() <= 8 and list(t.shape) == list(self.entry.shape)):
            return [(string_to_dtype(self.entry.dtype), self.entry.shape, base, None, t)]
        return None


def _q_params_equal(lhs: torch.Tensor, rhs: torch.Tensor) -> bool:
    if lhs.qscheme() != rhs.qscheme():
        return False
    if lhs.qscheme() == torch.per_tensor_affine:
        return lhs.q_scale() == rhs.q_scale() and lhs.q_zero_point() == rhs.q_zero_point()
    if lhs.qscheme() in (torch.per_channel_affine, torch.per_channel_affine_float_qparams):
        return (torch.equal(lhs.q_per_channel_scales(), rhs.q_per_channel_scales())
                and torch.equal(lhs.q_per_channel_zero_points(), rhs.q_per_channel_zero_points())
                and lhs.q_per_channel_axis() == rhs.q_per_channel_axis())
    raise RuntimeError(f"Unrecognized qscheme {lhs.qscheme()}")


def tensor_copy(dst: torch.Tensor, src: torch.Tensor) -> None:
    """``dst.copy_(src)`` that also handles quantized <-> float and qparam changes.

    Quantized sources are dequantized when the destination is not quantized,
    has another qscheme/dtype, or is a view whose qparams differ (copying then
    would silently re-label the view's data under the parent's qparams).
    """
    if src.is_quantized and (
            not dst.is_quantized or dst.qscheme() != src.qscheme() or dst.dtype != src.dtype
            or (dst._is_view() and not _q_params_equal(dst, src))):
        src = src.dequantize()
    with torch.no_grad():
        # quantized -> quantized copy_ also moves the qparams onto its
        # destination: that must be ``dst`` itself, not a detach()'d alias
        # (the alias took the new scale / zero point, ``dst`` kept its old
        # ones and read back wrong values)
        (dst if dst.is_quantized else dst.detach()).copy_(src)
