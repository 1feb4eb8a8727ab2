"""Local / network file-system storage on the native C++ I/O engine.

Reference behaviour (`/root/reference/torchsnapshot/storage_plugins/fs.py:19-56`):
``wb+`` writes through aiofiles, mkdir with a dir cache, ranged reads by
seek+read, no fsync.  Here every blob write/read is one job on the C++ worker
pool of ``hipsnapshot/csrc/hsio.cpp``: the worker pwrite()s directly from the
staged buffer's address (pinned pool block or CPU tensor storage) and reports
completion through an eventfd watched by the asyncio loop, so no Python thread
and no intermediate ``bytes`` copy is involved.

storage_options:
  ``direct_io`` (bool)  O_DIRECT for the 4 KiB-aligned body (default: knob)
  ``fsync`` (bool)      fdatasync each blob (default: knob)
  ``io_threads`` (int)  engine workers (default: knob, 16)
"""

from __future__ import annotations

import asyncio
import ctypes
import errno
import os
import shutil
import time
from typing import Any, Dict, Optional

from .. import knobs
from ..io_types import ReadIO, StagedBuffer, StoragePlugin, WriteIO, buffer_address
from ..utils.tracing import timeline

try:
    from ..ops import native as _native
except Exception:  # pragma: no cover - numpy/ctypes always present
    _native = None


class FSStoragePlugin(StoragePlugin):
    def __init__(self, root: str, storage_options: Optional[Dict[str, Any]] = None) -> None:
        opts = dict(storage_options or {})
        self.root = root
        self.direct_io = bool(opts.get("direct_io", knobs.use_direct_io()))
        self.fsync = bool(opts.get("fsync", knobs.use_fsync()))
        # None: knobs.get_io_threads() when the engine starts (it depends on
        # how many ranks share this host, learnt by the take's first collective)
        self._io_threads_opt = opts.get("io_threads")
        self._engine = None
        self._loop: Optional[asyncio.AbstractEventLoop] = None
        self._pending: Dict[int, tuple] = {}
        self._native_ok = True
        self.bytes_written = 0
        self.bytes_read = 0

    @property
    def io_threads(self) -> int:
        if self._io_threads_opt is not None:
            return int(self._io_threads_opt)
        return knobs.get_io_threads()

    # -- engine plumbing ---------------------------------------------------

    def _get_engine(self):
        if not self._native_ok:
            return None
        if self._engine is None:
            try:
                self._engine = _native.acquire_io_engine(self.io_threads)
            except Exception:  # pragma: no cover - compiler missing
                self._native_ok = False
                return None
        loop = asyncio.get_running_loop()
        if self._loop is not loop:
            if self._loop is not None and not self._loop.is_closed():
                try:
                    self._loop.remove_reader(self._engine.efd)
                except Exception:
                    pass
            loop.add_reader(self._engine.efd, self._on_ready)
            self._loop = loop
        return self._engine

    def _on_ready(self) -> None:
        for job_id, result in self._engine.poll():
            fut, _keep = self._pending.pop(job_id, (None, None))
            if fut is not None and not fut.done():
                fut.set_result(result)

    async def _await_job(self, job_id: int, keepalive: Any) -> int:
        fut = asyncio.get_running_loop().create_future()
        self._pending[job_id] = (fut, keepalive)
        # the completion may already be queued
        self._on_ready()
        return await _uncancellable(fut)

    def _flags(self, mkdirs: bool = False) -> int:
        f = 0
        if self.direct_io:
            f |= _native.IO_DIRECT
        if self.fsync:
            f |= _native.IO_SYNC
        if mkdirs:
            f |= _native.IO_MKDIRS
        return f

    def _abs(self, path: str) -> str:
        return os.path.join(self.root, path)

    def native_drain_root(self):
        """(root, fsync, O_DIRECT) for the native drain of an async take's
        frozen blobs (engine/native_drain.py).  O_DIRECT when this plugin
        writes O_DIRECT (``direct_io`` storage option / ``HIPSNAPSHOT_FS_DIRECT_IO``)."""
        return self.root, self.fsync, self.direct_io

    def native_read_root(self) -> str:
        """Root of the blobs for the native restore (engine/native_restore.py)."""
        return self.root

    # -- StoragePlugin -------------------------------------------------------

    async def write(self, write_io: WriteIO) -> None:
        path = self._abs(write_io.path)
        mv = memoryview(write_io.buf).cast("B")
        n = mv.nbytes
        addr = write_io.addr if write_io.addr is not None else buffer_address(mv)
        eng = self._get_engine()
        if eng is None:
            await _uncancellable(asyncio.get_running_loop().run_in_executor(
                None, _py_write, path, mv))
        else:
            flags = self._flags(mkdirs=True)
            if write_io.numa_node is not None and 0 <= write_io.numa_node < 255:
                flags |= (write_io.numa_node + 1) << _native.IO_NODE_SHIFT  # csrc/hsio.cpp
            job = eng.submit_write(path, addr, n, 0, flags)
            res = await self._await_job(job, mv)
            if res < 0:
                raise OSError(-res, os.strerror(-res), path)
        self.bytes_written += n

    async def read(self, read_io: ReadIO) -> None:
        path = self._abs(read_io.path)
        if read_io.byte_range is None:
            size = os.path.getsize(path)
            offset, n = 0, size
        else:
            offset, end = read_io.byte_range
            n = end - offset
        if read_io.dest is not None and read_io.dest.nbytes >= n:
            dest_view, addr = read_io.dest.view[:n], read_io.dest.addr
        else:
            ba = bytearray(n)
            dest_view = memoryview(ba)
            addr = buffer_address(ba) if n else 0
        eng = self._get_engine()
        if n == 0:
            read_io.buf = dest_view
            return
        if eng is None:
            got = await _uncancellable(asyncio.get_running_loop().run_in_executor(
                None, _py_read, path, dest_view, offset))
        else:
            job = eng.submit_read(path, addr, n, offset, self._flags())
            got = await self._await_job(job, dest_view)
            if got < 0:
                raise OSError(-got, os.strerror(-got), path)
        if got != n:
            raise OSError(errno.EIO, f"short read ({got} of {n} bytes)", path)
        read_io.buf = dest_view
        self.bytes_read += n

    async def size(self, path: str) -> Optional[int]:
        return os.path.getsize(self._abs(path))

    async def commit_metadata(self, path: str, buf: bytes) -> None:
        """Atomic commit: write a temp file then rename it into place."""
        final = self._abs(path)
        tmp = f"{final}.tmp.{os.getpid()}"
        os.makedirs(os.path.dirname(final) or ".", exist_ok=True)
        with open(tmp, "wb") as f:
            f.write(buf)
            if self.fsync:
                f.flush()
                os.fsync(f.fileno())
        os.replace(tmp, final)

    async def delete(self, path: str) -> None:
        os.remove(self._abs(path))

    async def rename(self, src: str, dst: str) -> None:
        os.replace(self._abs(src), self._abs(dst))

    async def delete_dir(self, path: str) -> None:
        shutil.rmtree(self._abs(path))

    async def close(self) -> None:
        if self._engine is not None:
            if self._loop is not None and not self._loop.is_closed():
                try:
                    self._loop.remove_reader(self._engine.efd)
                except Exception:
                    pass
            _native.release_io_engine(self._engine, reusable=not self._pending)
            self._engine = None
            self._loop = None


async def _uncancellable(fut: "asyncio.Future[Any]") -> Any:
    """Await a job that reads or writes a caller-owned buffer.

    Cancelling the awaiting task does not stop the engine worker (or executor
    thread) behind ``fut``: it keeps pread()ing into / pwrite()ing from the
    buffer.  Callers release that buffer (back to the pinned pool, or to
    hipHostFree) as soon as this coroutine ends, so a cancellation must not
    end it early: wait for the job, then re-raise the cancellation."""
    cancelled = False
    while not fut.done():
        try:
            await asyncio.shield(fut)
        except asyncio.CancelledError:
            if fut.cancelled():
                raise
            cancelled = True
    if cancelled:
        raise asyncio.CancelledError()
    return fut.result()


def _py_write(path: str, mv: memoryview) -> None:
    os.makedirs(os.path.dirname(path), exist_ok=True)
    with open(path, "wb") as f:
        f.write(mv)


def _py_read(path: str, dest: memoryview, offset: int) -> int:
    with open(path, "rb") as f:
        f.seek(offset)
        return f.readinto(dest)
