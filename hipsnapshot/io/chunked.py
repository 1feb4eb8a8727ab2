"""Large tensors split along dim 0 into <= ``max_chunk_size`` pieces.

Reference: `/root/reference/torchsnapshot/io_preparers/chunked_tensor.py:26-126`.
Chunk boundaries follow ``torch.chunk`` on dim 0 with
``ceil(nbytes / max_chunk)`` chunks; each chunk is a ``TensorEntry`` at
``<storage_path>_<off0>_<off1>...`` wrapped in a ``Shard``.  Replicated chunked
tensors are the unit the partitioner spreads across ranks chunk by chunk.
"""

from __future__ import annotations

import math
from dataclasses import dataclass
from typing import List, Optional, Tuple, Union

import torch

from ..format.manifest import ChunkedTensorEntry, Shard
from ..format.serialization import dtype_to_string
from ..io_types import Future, ReadReq, WriteReq
from ..knobs import get_max_chunk_size_bytes
from .tensor import PrepareFunc, TensorIOPreparer


@dataclass
class Chunk:
    offsets: List[int]
    sizes: List[int]
    dtype: str


def subtensor_view(tensor: torch.Tensor, chunk: Union[Shard, Chunk]) -> torch.Tensor:
    out = tensor.view(-1) if tensor.ndim == 0 else tensor
    for d, (o, z) in enumerate(zip(chunk.offsets, chunk.sizes)):
        out = out.narrow(d, o, z)
    return out


class ChunkedTensorIOPreparer:
    @staticmethod
    def chunk_tensor(tensor: torch.Tensor, chunking_dim: int = 0,
                     chunk_sz_bytes: Optional[int] = None) -> List[Chunk]:
        chunk_sz_bytes = chunk_sz_bytes or get_max_chunk_size_bytes()
        if tensor.ndim == 0:
            tensor = tensor.view(-1)
        nbytes = tensor.numel() * tensor.element_size()
        n_chunks = max(1, math.ceil(nbytes / chunk_sz_bytes))
        pieces = torch.chunk(tensor, chunks=n_chunks, dim=chunking_dim)
        offsets = [0] * tensor.ndim
        out = []
        for p in pieces:
            out.append(Chunk(offsets=list(offsets), sizes=list(p.shape), dtype=str(tensor.dtype)))
            offsets[chunking_dim] += p.shape[chunking_dim]
        return out

    @staticmethod
    def _get_subtensor_view(tensor: torch.Tensor, chunk) -> torch.Tensor:
        return subtensor_view(tensor, chunk)

    @classmethod
    def prepare_write(cls, storage_path: str, tensor: torch.Tensor,
                      chunking_instruction: List[Chunk], is_async_snapshot: bool = False,
                      _tensor_prepare_func: Optional[PrepareFunc] = None,
                      serializer: Optional[str] = None
                      ) -> Tuple[ChunkedTensorEntry, List[WriteReq]]:
        chunks, reqs = [], []
        for ch in chunking_instruction:
            suffix = "_".join(str(x) for x in ch.offsets)
            entry, wrs = TensorIOPreparer.prepare_write(
                storage_path=f"{storage_path}_{suffix}", tensor=subtensor_view(tensor, ch),
                is_async_snapshot=is_async_snapshot, _tensor_prepare_func=_tensor_prepare_func,
                serializer=serializer)
            chunks.append(Shard(offsets=list(ch.offsets), sizes=list(ch.sizes), tensor=entry))
            reqs += wrs
        dtype = chunks[0].tensor.dtype if chunks else dtype_to_string(tensor.dtype)
        return ChunkedTensorEntry(dtype=dtype, shape=list(tensor.shape), chunks=chunks,
                                  replicated=False), reqs

    @classmethod
    def prepare_read(cls, entry: ChunkedTensorEntry, tensor_out: Optional[torch.Tensor] = None,
                     buffer_size_limit_bytes: Optional[int] = None
                     ) -> Tuple[List[ReadReq], Future]:
        if _is_quantized_entry(entry) or (tensor_out is not None and tensor_out.is_quantized):
            return _read_quantized_chunks(entry, tensor_out, buffer_size_limit_bytes)
        if tensor_out is None or not TensorIOPreparer.can_load_inplace(entry, tensor_out):
            tensor_out = TensorIOPreparer.empty_tensor_from_entry(entry)
        reqs: List[ReadReq] = []
        for ch in entry.chunks:
            rrs, _ = TensorIOPreparer.prepare_read(ch.tensor, subtensor_view(tensor_out, ch),
                                                   buffer_size_limit_bytes)
            reqs += rrs
        return reqs, Future(obj=tensor_out)


def _is_quantized_entry(entry: ChunkedTensorEntry) -> bool:
    from ..format.serialization import SUPPORTED_QUANTIZED_DTYPES, string_to_dtype

    try:
        return string_to_dtype(entry.dtype) in SUPPORTED_QUANTIZED_DTYPES
    except Exception:  # noqa: BLE001 - an unknown dtype string: not quantized
        return False


class _JoinedQuantized(Future):
    """A chunked quantized tensor.  Its chunks load as tensors of their own: a
    chunk-sized view of the destination cannot take the saved scale / zero
    point (``copy_`` moves qparams onto the view only), so the chunks are
    joined on first access and copied into ``out`` whole."""

    def __init__(self, parts: List[Future], entry: ChunkedTensorEntry,
                 out: Optional[torch.Tensor]) -> None:
        self._parts, self._entry, self._out, self._done = parts, entry, out, False

    @property
    def obj(self):
        if not self._done:
            self._out = _join_quantized([f.obj for f in self._parts], self._entry, self._out)
            self._done = True
        return self._out

    @obj.setter
    def obj(self, value) -> None:
        self._out, self._done = value, True


def _join_quantized(parts: List[torch.Tensor], entry: ChunkedTensorEntry,
                    out: Optional[torch.Tensor]) -> torch.Tensor:
    from .tensor import tensor_copy

    shape = list(entry.shape)
    flat0 = len(shape) == 0  # a 0-d tensor was chunked as a 1-d view
    if parts[0].qscheme() in (torch.per_tensor_affine, torch.per_tensor_symmetric):
        full = torch.cat(parts, dim=0)
    else:
        axis = parts[0].q_per_channel_axis()
        # per-channel qparams along the chunked dim are cut with it; along
        # another dim every chunk carries the same ones
        if axis == 0:
            scales = torch.cat([p.q_per_channel_scales() for p in parts])
            zeros = torch.cat([p.q_per_channel_zero_points() for p in parts])
        else:
            scales, zeros = parts[0].q_per_channel_scales(), parts[0].q_per_channel_zero_points()
        full = torch._make_per_channel_quantized_tensor(
            torch.cat([p.int_repr() for p in parts], dim=0), scales, zeros, axis)
    full = full.reshape(shape) if not flat0 else full.reshape([])
    if out is None:
        return full
    tensor_copy(out, full)
    return out


def _read_quantized_chunks(entry: ChunkedTensorEntry, tensor_out: Optional[torch.Tensor],
                           limit: Optional[int]) -> Tuple[List[ReadReq], Future]:
    reqs: List[ReadReq] = []
    parts: List[Future] = []
    for ch in sorted(entry.chunks, key=lambda c: list(c.offsets)):
        rrs, fut = TensorIOPreparer.prepare_read(ch.tensor, None, limit)
        reqs += rrs
        parts.append(fut)
    return reqs, _JoinedQuantized(parts, entry, tensor_out)
