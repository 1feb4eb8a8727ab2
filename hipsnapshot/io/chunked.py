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
        if tensor_out is None or not TensorIOPreparer.can_load_inplace(entry, tensor_out):
            tensor_out = TensorIOPreparer.empty_tensor_from_entry(entry)
        reqs: List[ReadReq] = []
        for ch in entry.chunks:
            rrs, _ = TensorIOPreparer.prepare_read(ch.tensor, subtensor_view(tensor_out, ch),
                                                   buffer_size_limit_bytes)
            reqs += rrs
        return reqs, Future(obj=tensor_out)
