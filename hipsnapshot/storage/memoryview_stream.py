"""Zero-copy read-only file object over a ``memoryview``.

Reference: `/root/reference/torchsnapshot/memoryview_stream.py:12-81`.  Lets
HTTP clients stream staged (pinned) tensor bytes without materialising a
``bytes`` copy.
"""

from __future__ import annotations

import io
from typing import Optional


class MemoryviewStream(io.RawIOBase):
    def __init__(self, mv: memoryview) -> None:
        super().__init__()
        self._mv = memoryview(mv).cast("B")
        self._pos = 0

    def readable(self) -> bool:
        return True

    def seekable(self) -> bool:
        return True

    def read(self, size: Optional[int] = -1) -> bytes:
        if self.closed:
            raise ValueError("I/O operation on closed stream")
        if size is None or size < 0:
            end = len(self._mv)
        else:
            end = min(len(self._mv), self._pos + size)
        out = self._mv[self._pos:end]
        self._pos = end
        return out.tobytes()

    def read_view(self, size: int = -1) -> memoryview:
        """Like ``read`` but returns a zero-copy slice."""
        end = len(self._mv) if size < 0 else min(len(self._mv), self._pos + size)
        out = self._mv[self._pos:end]
        self._pos = end
        return out

    def readinto(self, b) -> int:
        data = self.read_view(len(memoryview(b)))
        n = len(data)
        memoryview(b).cast("B")[:n] = data
        return n

    def seek(self, offset: int, whence: int = io.SEEK_SET) -> int:
        if whence == io.SEEK_SET:
            pos = offset
        elif whence == io.SEEK_CUR:
            pos = self._pos + offset
        elif whence == io.SEEK_END:
            pos = len(self._mv) + offset
        else:
            raise ValueError(f"invalid whence ({whence})")
        if pos < 0:
            raise ValueError(f"negative seek position {pos}")
        self._pos = pos
        return self._pos

    def tell(self) -> int:
        return self._pos

    def __len__(self) -> int:
        return len(self._mv)
