"""Per-object write/read dispatch and the blob-location policy.

Reference: `/root/reference/torchsnapshot/io_preparer.py:46-175`.

location policy (on-disk format):
  * sharded (ShardedTensor / DTensor)  -> ``sharded/<logical_path>``
  * replicated                         -> ``replicated/<logical_path>``
  * otherwise                          -> ``<rank>/<logical_path>``
dispatch:
  primitive (int/str/bool/bytes/float) -> inline ``PrimitiveEntry``
  ShardedTensor / DTensor              -> ``ShardedTensorIOPreparer``
  Tensor > max_chunk_size              -> ``ChunkedTensorIOPreparer``
  Tensor                               -> ``TensorIOPreparer``
  anything else                        -> ``ObjectIOPreparer`` (torch.save)
"""

from __future__ import annotations

import os
from typing import Any, List, Optional, Tuple

import torch

from ..format.manifest import (
    ChunkedTensorEntry,
    Entry,
    ObjectEntry,
    PRIMITIVE_TYPES,
    PrimitiveEntry,
    ShardedTensorEntry,
    TensorEntry,
)
from ..io_types import Future, ReadReq, WriteReq
from ..knobs import get_max_chunk_size_bytes
from .chunked import Chunk, ChunkedTensorIOPreparer
from .object import ObjectBufferConsumer, ObjectBufferStager, ObjectIOPreparer
from .sharded import ShardedTensorIOPreparer, is_sharded
from .tensor import PrepareFunc, TensorBufferConsumer, TensorBufferStager, TensorIOPreparer, tensor_copy

__all__ = [
    "Chunk", "ObjectBufferConsumer", "ObjectBufferStager", "TensorBufferConsumer",
    "TensorBufferStager", "tensor_copy", "prepare_write", "prepare_read", "get_storage_path",
    "PrimitivePreparer",
]


def get_storage_path(obj: Any, logical_path: str, rank: int, replicated: bool) -> str:
    if is_sharded(obj):
        return os.path.join("sharded", logical_path)
    if replicated:
        return os.path.join("replicated", logical_path)
    return os.path.join(str(rank), logical_path)


class PrimitivePreparer:
    @staticmethod
    def should_inline(obj: Any) -> bool:
        return type(obj).__name__ in PRIMITIVE_TYPES and type(obj) in (int, str, bool, bytes,
                                                                       float)

    @staticmethod
    def prepare_write(obj: Any) -> PrimitiveEntry:
        return PrimitiveEntry.from_object(obj)

    @staticmethod
    def prepare_read(entry: PrimitiveEntry) -> Tuple[List[ReadReq], Future]:
        return [], Future(obj=entry.get_value())


def prepare_write(obj: Any, logical_path: str, rank: int, replicated: bool,
                  is_async_snapshot: bool = False,
                  _tensor_prepare_func: Optional[PrepareFunc] = None,
                  serializer: Optional[str] = None,
                  max_chunk_size_bytes: Optional[int] = None,
                  max_shard_size_bytes: Optional[int] = None) -> Tuple[Entry, List[WriteReq]]:
    """The size knobs default to their current values; a take reads them once
    and passes them to every call (an env lookup per leaf adds up at ~300
    leaves per Llama-3-8B state dict)."""
    if PrimitivePreparer.should_inline(obj):
        entry = PrimitivePreparer.prepare_write(obj)
        entry.replicated = replicated
        return entry, []
    storage_path = get_storage_path(obj, logical_path, rank, replicated)
    if is_sharded(obj):
        return ShardedTensorIOPreparer.prepare_write(
            storage_path=storage_path, obj=obj, is_async_snapshot=is_async_snapshot,
            _tensor_prepare_func=_tensor_prepare_func, serializer=serializer,
            max_shard_size_bytes=max_shard_size_bytes)
    if isinstance(obj, torch.Tensor):
        if obj.numel() * obj.element_size() > (max_chunk_size_bytes or get_max_chunk_size_bytes()):
            entry, wrs = ChunkedTensorIOPreparer.prepare_write(
                storage_path=storage_path, tensor=obj,
                chunking_instruction=ChunkedTensorIOPreparer.chunk_tensor(obj),
                is_async_snapshot=is_async_snapshot, _tensor_prepare_func=_tensor_prepare_func,
                serializer=serializer)
        else:
            entry, wrs = TensorIOPreparer.prepare_write(
                storage_path=storage_path, tensor=obj, is_async_snapshot=is_async_snapshot,
                _tensor_prepare_func=_tensor_prepare_func, serializer=serializer)
    else:
        entry, wrs = ObjectIOPreparer.prepare_write(storage_path, obj)
    entry.replicated = replicated
    return entry, wrs


def prepare_read(entry: Entry, obj_out: Optional[Any] = None,
                 buffer_size_limit_bytes: Optional[int] = None,
                 trust_objects: Optional[bool] = None) -> Tuple[List[ReadReq], Future]:
    if isinstance(entry, ShardedTensorEntry):
        if obj_out is None:
            raise RuntimeError(
                "Reading a ShardedTensor without a runtime object is not supported.")
        return ShardedTensorIOPreparer.prepare_read(entry, obj_out)
    if isinstance(entry, ChunkedTensorEntry):
        return ChunkedTensorIOPreparer.prepare_read(entry, obj_out, buffer_size_limit_bytes)
    if isinstance(entry, TensorEntry):
        return TensorIOPreparer.prepare_read(entry, obj_out, buffer_size_limit_bytes)
    if isinstance(entry, ObjectEntry):
        return ObjectIOPreparer.prepare_read(entry, obj_out, trusted=trust_objects)
    if isinstance(entry, PrimitiveEntry):
        return PrimitivePreparer.prepare_read(entry)
    raise Exception(f"Unsupported entry type: {entry} ({entry.type}).")
