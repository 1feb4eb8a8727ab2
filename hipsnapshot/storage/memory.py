"""In-process object store (``memory://bucket/prefix``).

Not in the reference; used by tests and by benchmarks that want to take
storage out of the measurement.  Objects live in a process-global dict so a
snapshot written by one ``Snapshot`` object is readable by another.
"""

from __future__ import annotations

import threading
from typing import Any, Dict, Optional

from ..io_types import ReadIO, StoragePlugin, WriteIO

_STORE: Dict[str, bytes] = {}
_LOCK = threading.Lock()


def clear_memory_store(prefix: str = "") -> None:
    with _LOCK:
        for k in [k for k in _STORE if k.startswith(prefix)]:
            del _STORE[k]


class MemoryStoragePlugin(StoragePlugin):
    def __init__(self, root: str, storage_options: Optional[Dict[str, Any]] = None) -> None:
        self.root = root.rstrip("/")

    def _key(self, path: str) -> str:
        return f"{self.root}/{path}"

    async def write(self, write_io: WriteIO) -> None:
        data = bytes(memoryview(write_io.buf).cast("B"))
        with _LOCK:
            _STORE[self._key(write_io.path)] = data

    async def read(self, read_io: ReadIO) -> None:
        with _LOCK:
            try:
                data = _STORE[self._key(read_io.path)]
            except KeyError:
                raise FileNotFoundError(self._key(read_io.path)) from None
        if read_io.byte_range is not None:
            lo, hi = read_io.byte_range
            data = data[lo:hi]
        if read_io.dest is not None and read_io.dest.nbytes >= len(data):
            read_io.dest.view[: len(data)] = data
            read_io.buf = read_io.dest.view[: len(data)]
        else:
            read_io.buf = memoryview(data)

    async def size(self, path: str) -> Optional[int]:
        with _LOCK:
            data = _STORE.get(self._key(path))
        return None if data is None else len(data)

    async def delete(self, path: str) -> None:
        with _LOCK:
            _STORE.pop(self._key(path), None)

    async def delete_dir(self, path: str) -> None:
        clear_memory_store(self._key(path).rstrip("/") + "/")

    async def close(self) -> None:
        return None
