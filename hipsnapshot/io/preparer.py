"""Which preparer plans a state-dict leaf (write) or a manifest entry (read).

Behaviour of `/root/reference/torchsnapshot/io_preparer.py:46-175` (where a
blob lives, and which preparer handles which kind of value); the structure
here is table-driven instead of an if-chain:

* a leaf is classified ONCE per Python type (``_leaf_kind``, cached): a cold
  take of an FSDP2 Llama-3-8B plans ~300 DTensor leaves on the
  ``async_take`` unblock path, so the per-leaf dispatch is a dict lookup;
* a manifest entry is read by ``_READERS[type(entry)]``.

Blob locations (the on-disk format)::

    sharded leaf (ShardedTensor / DTensor)  sharded/<logical path>
    replicated leaf                         replicated/<logical path>
    anything else                           <rank>/<logical path>

Leaf kinds: ``primitive`` (int / str / bool / bytes / float, stored inline in
the manifest), ``sharded``, ``tensor`` (chunked along dim 0 when larger than
the max chunk size), ``object`` (``torch.save`` bytes).
"""

from __future__ import annotations

from typing import Any, Callable, Dict, List, Optional, Tuple

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

_INLINE_TYPES = (int, str, bool, bytes, float)


class PrimitivePreparer:
    """Values stored inline in the manifest (no blob)."""

    @staticmethod
    def should_inline(obj: Any) -> bool:
        t = type(obj)
        return t in _INLINE_TYPES and t.__name__ in PRIMITIVE_TYPES

    @staticmethod
    def prepare_write(obj: Any) -> PrimitiveEntry:
        return PrimitiveEntry.from_object(obj)

    @staticmethod
    def prepare_read(entry: PrimitiveEntry) -> Tuple[List[ReadReq], Future]:
        return [], Future(obj=entry.get_value())


# -- write side ----------------------------------------------------------------

_KIND_BY_TYPE: Dict[type, str] = {}


def _leaf_kind(obj: Any) -> str:
    t = type(obj)
    kind = _KIND_BY_TYPE.get(t)
    if kind is None:
        if PrimitivePreparer.should_inline(obj):
            kind = "primitive"
        elif is_sharded(obj):
            kind = "sharded"
        elif isinstance(obj, torch.Tensor):
            kind = "tensor"
        else:
            kind = "object"
        _KIND_BY_TYPE[t] = kind
    return kind


def _storage_dir(kind: str, rank: int, replicated: bool) -> str:
    if kind == "sharded":
        return "sharded"
    return "replicated" if replicated else str(rank)


def get_storage_path(obj: Any, logical_path: str, rank: int, replicated: bool) -> str:
    return f"{_storage_dir(_leaf_kind(obj), rank, replicated)}/{logical_path}"


def _write_sharded(obj, path, is_async, prepare_func, serializer, max_chunk, max_shard):
    return ShardedTensorIOPreparer.prepare_write(
        storage_path=path, obj=obj, is_async_snapshot=is_async,
        _tensor_prepare_func=prepare_func, serializer=serializer,
        max_shard_size_bytes=max_shard)


def _write_tensor(obj, path, is_async, prepare_func, serializer, max_chunk, max_shard):
    max_chunk = max_chunk or get_max_chunk_size_bytes()
    # quantized tensors stay whole (the reference chunks them too): a chunk
    # restored into a view of the destination could not carry its qparams
    if obj.numel() * obj.element_size() > max_chunk and not obj.is_quantized:
        return ChunkedTensorIOPreparer.prepare_write(
            storage_path=path, tensor=obj,
            chunking_instruction=ChunkedTensorIOPreparer.chunk_tensor(obj,
                                                                      chunk_sz_bytes=max_chunk),
            is_async_snapshot=is_async, _tensor_prepare_func=prepare_func,
            serializer=serializer)
    return TensorIOPreparer.prepare_write(
        storage_path=path, tensor=obj, is_async_snapshot=is_async,
        _tensor_prepare_func=prepare_func, serializer=serializer)


def _write_object(obj, path, is_async, prepare_func, serializer, max_chunk, max_shard):
    return ObjectIOPreparer.prepare_write(path, obj)


_WRITERS: Dict[str, Callable] = {"sharded": _write_sharded, "tensor": _write_tensor,
                                 "object": _write_object}


def prepare_write(obj: Any, logical_path: str, rank: int, replicated: bool,
                  is_async_snapshot: bool = False,
                  _tensor_prepare_func: Optional[PrepareFunc] = None,
                  serializer: Optional[str] = None,
                  max_chunk_size_bytes: Optional[int] = None,
                  max_shard_size_bytes: Optional[int] = None) -> Tuple[Entry, List[WriteReq]]:
    """The manifest entry of leaf ``obj`` and the write requests of its
    blob(s).  The size knobs default to their current values; a take reads
    them once and passes them to every call."""
    kind = _leaf_kind(obj)
    if kind == "primitive":
        entry = PrimitivePreparer.prepare_write(obj)
        entry.replicated = replicated
        return entry, []
    path = f"{_storage_dir(kind, rank, replicated)}/{logical_path}"
    entry, wrs = _WRITERS[kind](obj, path, is_async_snapshot, _tensor_prepare_func, serializer,
                                max_chunk_size_bytes, max_shard_size_bytes)
    entry.replicated = replicated
    return entry, wrs


# -- read side -----------------------------------------------------------------

def _read_sharded(entry, obj_out, limit, trust_objects):
    if obj_out is None:
        raise RuntimeError(f"the sharded entry {entry.type!r} can only be read into an obj_out "
                           "(DTensor, ShardedTensor or Tensor) that receives it")
    return ShardedTensorIOPreparer.prepare_read(entry, obj_out)


def _read_chunked(entry, obj_out, limit, trust_objects):
    return ChunkedTensorIOPreparer.prepare_read(entry, obj_out, limit)


def _read_tensor(entry, obj_out, limit, trust_objects):
    return TensorIOPreparer.prepare_read(entry, obj_out, limit)


def _read_object(entry, obj_out, limit, trust_objects):
    return ObjectIOPreparer.prepare_read(entry, obj_out, trusted=trust_objects)


def _read_primitive(entry, obj_out, limit, trust_objects):
    return PrimitivePreparer.prepare_read(entry)


_READERS: Dict[type, Callable] = {
    ShardedTensorEntry: _read_sharded, ChunkedTensorEntry: _read_chunked,
    TensorEntry: _read_tensor, ObjectEntry: _read_object, PrimitiveEntry: _read_primitive,
}


def prepare_read(entry: Entry, obj_out: Optional[Any] = None,
                 buffer_size_limit_bytes: Optional[int] = None,
                 trust_objects: Optional[bool] = None) -> Tuple[List[ReadReq], Future]:
    """Read requests that restore ``entry`` (into ``obj_out`` in place when
    it fits) and the future that will hold the value."""
    reader = _READERS.get(type(entry))
    if reader is None:  # a subclass of a known entry type
        reader = next((fn for cls, fn in _READERS.items() if isinstance(entry, cls)), None)
    if reader is None:
        raise TypeError(f"no reader for manifest entry {entry!r} of type {entry.type!r}")
    return reader(entry, obj_out, buffer_size_limit_bytes, trust_objects)
