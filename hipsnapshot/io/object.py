"""Arbitrary picklable objects -> ``torch.save`` blobs.

Reference: `/root/reference/torchsnapshot/io_preparers/object.py:35-92`.

Reading is SAFE by default: payloads are loaded with ``weights_only=True``
(tensors, containers, primitives and torch's allow-listed types -- enough for
model / optimizer / scheduler state).  Arbitrary pickled classes are only
unpickled when the caller opts in, either per snapshot
(``Snapshot(path, trust_objects=True)``) or process-wide
(``HIPSNAPSHOT_TRUST_OBJECTS=1``); otherwise the load error is raised with a
hint.  (torch >= 2.6 made weights-only the default, which broke the
reference's object path -- SURVEY Appendix C #8.)
"""

from __future__ import annotations

from concurrent.futures import Executor
from typing import Any, List, Optional, Tuple

from .. import knobs
from ..format.manifest import ObjectEntry
from ..format.serialization import SER, torch_load_from_bytes, torch_save_as_bytes
from ..io_types import BufferConsumer, BufferStager, Future, ReadReq, WriteReq


class ObjectBufferStager(BufferStager):
    def __init__(self, obj: Any) -> None:
        # serialize eagerly: the object is captured at take time (async-safe)
        self._buf = torch_save_as_bytes(obj)

    thread_staging = True

    async def stage_buffer(self, executor: Optional[Executor] = None):
        return self._buf

    def stage_buffer_sync(self):
        return self._buf

    def get_staging_cost_bytes(self) -> int:
        return len(self._buf)


class UntrustedObjectError(RuntimeError):
    pass


class ObjectBufferConsumer(BufferConsumer):
    def __init__(self, entry: ObjectEntry, trusted: Optional[bool] = None) -> None:
        self.entry = entry
        self.future: Future = Future()
        self.trusted = knobs.trust_object_payloads() if trusted is None else trusted
        self._cost = 0

    async def consume_buffer(self, buf, executor: Optional[Executor] = None) -> None:
        self._cost = len(memoryview(buf))
        if self.trusted:
            self.future.obj = torch_load_from_bytes(buf, trusted=True)
            return
        try:
            self.future.obj = torch_load_from_bytes(buf, trusted=False)
        except Exception as e:  # noqa: BLE001
            raise UntrustedObjectError(
                f"object entry {self.entry.location!r} (type {self.entry.obj_type}) cannot be "
                "loaded with weights_only=True. If this snapshot comes from a trusted source, "
                "pass trust_objects=True to Snapshot(...) or set HIPSNAPSHOT_TRUST_OBJECTS=1, "
                "or register the type with torch.serialization.add_safe_globals. "
                f"Loader error: {e}") from e

    def get_consuming_cost_bytes(self) -> int:
        return self._cost


class ObjectIOPreparer:
    @staticmethod
    def prepare_write(storage_path: str, obj: Any) -> Tuple[ObjectEntry, List[WriteReq]]:
        t = type(obj)
        entry = ObjectEntry(location=storage_path, serializer=SER.TORCH_SAVE,
                            obj_type=f"{t.__module__}.{t.__qualname__}", replicated=False)
        return entry, [WriteReq(path=storage_path, buffer_stager=ObjectBufferStager(obj))]

    @staticmethod
    def prepare_read(entry: ObjectEntry, obj_out: Optional[Any] = None,
                     trusted: Optional[bool] = None) -> Tuple[List[ReadReq], Future]:
        consumer = ObjectBufferConsumer(entry, trusted=trusted)
        return [ReadReq(path=entry.location, buffer_consumer=consumer)], consumer.future
