"""Request / buffer types shared by the planners, the engine and storage plugins.

Mirrors the reference's contract (`/root/reference/torchsnapshot/io_types.py:16-111`):
a write is ``WriteReq(path, buffer_stager)`` whose stager produces the bytes,
a read is ``ReadReq(path, buffer_consumer, byte_range)`` whose consumer eats
them, and storage plugins only see ``WriteIO`` / ``ReadIO``.

Differences that matter for MI355X:

* ``StagedBuffer`` carries the host address of the bytes (a pinned pool block,
  a CPU tensor's storage, ...) plus a ``release`` hook, so the native I/O
  engine writes straight from pinned memory and the block returns to the pool
  the moment the write completes.
* a ``BufferConsumer`` may offer a destination (``get_read_dest``) so storage
  reads land directly in pinned memory or in the restore target's storage.
"""

from __future__ import annotations

import asyncio
import io
from abc import ABC, abstractmethod
from concurrent.futures import Executor
from dataclasses import dataclass, field
from typing import Any, Callable, Generic, Optional, Tuple, TypeVar, Union

import numpy as np

BufferType = Union[bytes, bytearray, memoryview]
T = TypeVar("T")


def buffer_address(buf) -> int:
    if len(memoryview(buf)) == 0:
        return 0
    return int(np.frombuffer(buf, dtype=np.uint8).ctypes.data)


class StagedBuffer:
    """Bytes ready for storage: ``view`` + raw ``addr`` + release hook."""

    __slots__ = ("view", "addr", "_release", "keepalive", "checksum", "ready", "numa_node")

    def __init__(self, view: BufferType, addr: Optional[int] = None,
                 release: Optional[Callable[[], None]] = None, keepalive: Any = None) -> None:
        mv = memoryview(view)
        if mv.format != "B" or mv.ndim != 1:
            mv = mv.cast("B")
        self.view = mv
        self.addr = buffer_address(mv) if addr is None else addr
        self._release = release
        self.keepalive = keepalive
        # hs64 of the bytes when the stager computed it (on the GPU); None =
        # the writer hashes them on the host (ops/checksum.py)
        self.checksum: Optional[int] = None
        # set when the bytes are still arriving (asynchronous SDMA copy):
        # call it (blocking, once) before reading the buffer
        self.ready: Optional[Callable[[], None]] = None
        # NUMA node of the host pages ``view`` points into, when the writer
        # should run there (host-resident UVM tables written in place)
        self.numa_node: Optional[int] = None

    @property
    def nbytes(self) -> int:
        return self.view.nbytes

    def release(self) -> None:
        rel, self._release = self._release, None
        self.keepalive = None
        if rel is not None:
            rel()


def as_staged(buf: Union[StagedBuffer, BufferType]) -> StagedBuffer:
    return buf if isinstance(buf, StagedBuffer) else StagedBuffer(buf)


class BufferStager(ABC):
    @abstractmethod
    async def stage_buffer(self, executor: Optional[Executor] = None) -> Union[StagedBuffer, BufferType]:
        ...

    @abstractmethod
    def get_staging_cost_bytes(self) -> int:
        ...


@dataclass
class WriteReq:
    path: str
    buffer_stager: BufferStager


class BufferConsumer(ABC):
    @abstractmethod
    async def consume_buffer(self, buf: BufferType, executor: Optional[Executor] = None) -> None:
        ...

    @abstractmethod
    def get_consuming_cost_bytes(self) -> int:
        ...

    def get_read_dest(self, nbytes: int) -> Optional[StagedBuffer]:
        """Optionally provide a writable destination for the raw bytes."""
        return None

    def get_compressed_read_dest(self, nbytes: int) -> Optional[StagedBuffer]:
        """Destination for the ENCODED bytes of an HSZ1 blob (pinned memory
        for consumers that decode on the GPU); None = plain host memory."""
        return None


class SpanTail:
    """The part of a compressed span's buffer that a second read is still
    filling: bytes from ``offset`` on.  The read's completion (on the event
    loop) calls ``arrived``; consumer threads call ``wait``."""

    def __init__(self, offset: int) -> None:
        import threading

        self.offset = offset
        self._event = threading.Event()
        self._error: Optional[BaseException] = None

    def arrived(self, error: Optional[BaseException] = None) -> None:
        self._error = error
        self._event.set()

    def wait(self) -> None:
        self._event.wait()
        if self._error is not None:
            raise self._error


class CompressedSpan:
    """Encoded frames [first, last) of an HSZ1 blob covering the logical byte
    range [lo, hi) a read asked for.  Consumers that restore into HBM move
    the encoded bytes with one H2D and decode on the GPU
    (``engine.staging.scatter_compressed``); others call ``decode_host``."""

    def __init__(self, buf: "StagedBuffer", header, first: int, last: int, lo: int,
                 hi: int, tail: Optional["SpanTail"] = None) -> None:
        self.buf = buf
        self.header = header
        self.first = first
        self.last = last
        self.lo = lo
        self.hi = hi
        # bytes of ``buf`` from ``tail.offset`` on may still be arriving
        self.tail = tail

    def wait_tail(self) -> None:
        """Block until every byte of ``buf`` has arrived (raises if the read
        of the rest failed)."""
        if self.tail is not None:
            self.tail.wait()

    @property
    def nbytes(self) -> int:
        return self.hi - self.lo

    @property
    def frames_logical_lo(self) -> int:
        return self.first * self.header.frame_bytes

    def decode_host(self) -> memoryview:
        """Logical bytes [lo, hi) decoded by the C++ codec into host memory."""
        from .ops import codec

        self.wait_tail()

        h = self.header
        n_log = min(self.last * h.frame_bytes, h.logical_size) - self.frames_logical_lo
        out = np.empty(max(n_log, 1), dtype=np.uint8)
        base = h.offsets[self.first]
        offs = np.asarray([o - base for o in h.offsets[self.first: self.last + 1]],
                          dtype=np.uint64)
        if self.last > self.first:
            from .ops import native

            native.hsz_decode_cpu(self.buf.addr, offs.ctypes.data, self.first,
                                  self.last - self.first, h.logical_size, h.elem_width,
                                  h.frame_bytes, out.ctypes.data)
        shift = self.lo - self.frames_logical_lo
        return memoryview(out)[shift: shift + self.nbytes]

    def release(self) -> None:
        self.buf.release()


@dataclass
class ReadReq:
    path: str
    buffer_consumer: BufferConsumer
    byte_range: Optional[Tuple[int, int]] = None
    # False for tiles of one large tensor: merging them back into one read
    # would defeat the memory budget / read-H2D pipelining they exist for
    mergeable: bool = True
    # HSZ1 info of the blob (entry.codec): byte_range is then in logical bytes
    codec: Optional[dict] = None


@dataclass
class Future(Generic[T]):
    obj: Optional[T] = None


@dataclass
class WriteIO:
    path: str
    buf: BufferType
    addr: Optional[int] = None
    # ``StagedBuffer.numa_node``: run the write on that node's CPUs
    numa_node: Optional[int] = None


@dataclass
class ReadIO:
    path: str
    byte_range: Optional[Tuple[int, int]] = None
    buf: Any = field(default_factory=io.BytesIO)
    dest: Optional[StagedBuffer] = None

    def data(self) -> BufferType:
        """The bytes read (memoryview/bytes), whatever the plugin produced."""
        b = self.buf
        if isinstance(b, io.BytesIO):
            return b.getbuffer()
        return b


class StoragePlugin(ABC):
    """Async storage backend; the ``sync_*`` helpers drive a given loop."""

    @abstractmethod
    async def write(self, write_io: WriteIO) -> None:
        ...

    @abstractmethod
    async def read(self, read_io: ReadIO) -> None:
        ...

    @abstractmethod
    async def delete(self, path: str) -> None:
        ...

    async def delete_dir(self, path: str) -> None:
        raise NotImplementedError(f"{type(self).__name__} does not implement delete_dir")

    async def rename(self, src: str, dst: str) -> None:
        """Atomically move blob ``src`` to ``dst`` (optional: a take that
        replaces a committed snapshot stashes its metadata this way, and
        otherwise keeps a copy of the bytes to put back)."""
        raise NotImplementedError(f"{type(self).__name__} does not implement rename")

    async def size(self, path: str) -> Optional[int]:
        """Stored size of a blob, or None when the backend cannot tell
        cheaply (then compressed blobs are read header-first)."""
        return None

    @abstractmethod
    async def close(self) -> None:
        ...

    def sync_write(self, write_io: WriteIO, event_loop: Optional[asyncio.AbstractEventLoop] = None) -> None:
        _run(self.write(write_io), event_loop)

    def sync_read(self, read_io: ReadIO, event_loop: Optional[asyncio.AbstractEventLoop] = None) -> None:
        _run(self.read(read_io), event_loop)

    def sync_delete(self, path: str, event_loop: Optional[asyncio.AbstractEventLoop] = None) -> None:
        _run(self.delete(path), event_loop)

    def sync_close(self, event_loop: Optional[asyncio.AbstractEventLoop] = None) -> None:
        _run(self.close(), event_loop)


async def _capture(coro):
    try:
        return await coro, None
    except BaseException as e:  # noqa: BLE001 - re-raised by run_sync
        return None, e


def run_sync(loop: asyncio.AbstractEventLoop, coro):
    """``loop.run_until_complete(coro)`` without a reference cycle on error.

    An exception raised through ``run_until_complete`` keeps its frame, whose
    ``future`` local is the task holding that same exception: a cycle that
    pins every caller frame's locals (a take's whole plan: entries, write
    requests, stagers) until the next full collection.  ``_uncommit``'s
    expected FileNotFoundError on a fresh path did exactly that.  Here the
    task ends normally and the exception is re-raised from this frame only."""
    res, err = loop.run_until_complete(_capture(coro))
    if err is None:
        return res
    try:
        raise err
    finally:
        del err


def _run(coro, loop: Optional[asyncio.AbstractEventLoop]):
    if loop is None:
        loop = asyncio.new_event_loop()
        try:
            return run_sync(loop, coro)
        finally:
            loop.close()
    return run_sync(loop, coro)
