"""Async-take drain in a helper process (``HIPSNAPSHOT_DRAIN_PROCESS=1``).

The native drain (``engine/native_drain.py``, ``csrc/hsdrain.hip``) keeps
Python out of an async take's background commit, but its threads still live
in the trainer's process: every SDMA submit, hash launch and pinned-slot
operation goes through the trainer's HIP runtime next to the training loop's
own launches, and the ``pwrite`` copies run in its address space.  A
launch-bound training step (Llama-3-8B at seq 512, ~200 ms) ran 3-8 % slower
while such a drain was in flight; the same bytes drained from another
process cost it ~1.6 % (``profiles/overlap_iso/``).

Here the drain runs in ``_hsdrain_helper`` (``csrc/hsdrain_helper.cpp``), a
small C++ child started once per trainer process:

* the frozen arena's allocation goes over as a HIP IPC handle (dmabuf) plus
  the blobs' offsets in it; the helper maps it once and keeps the mapping
  while the arena is kept between takes (``HIPSNAPSHOT_HBM_ARENA_KEEP``);
  dropping a kept arena queues an unmap that the helper runs before its next
  job;
* the helper runs the very same ``hsg_drain_start`` / ``hsg_drain_wait`` and
  replies with the hs64 partial sums, bytes written and per-phase seconds.

Any failure to start the helper or to map the arena falls back to the
in-process native drain (logged once); a helper that dies during a drain
fails that take's commit like any other I/O error, and the next drain starts
a new helper.

Reference counterpart: the async snapshot's background commit,
`/root/reference/torchsnapshot/snapshot.py:891-933`.
"""

from __future__ import annotations

import atexit
import errno
import logging
import os
import select
import struct
import subprocess
import threading
import time
from typing import Dict, List, Optional, Sequence, Tuple

from .. import _build

logger = logging.getLogger(__name__)

_MAGIC = 0x48534448  # "HSDH"
_OP_DRAIN, _OP_CLOSE, _OP_PING = 1, 2, 3


class DrainHelperError(RuntimeError):
    """The helper process could not run a drain (it died or refused the job)."""


class DrainHelperMapTimeout(DrainHelperError):
    """The helper did not report the arena mapping in time (nothing drained)."""


class DrainHelper:
    """One ``_hsdrain_helper`` child and its request pipe."""

    def __init__(self) -> None:
        from ..ops import native

        rt = native.hip_runtime_path()
        if rt is None:
            raise DrainHelperError("no libamdhip64 mapped in this process")
        if not os.path.exists(_build.DRAIN_HELPER):
            raise DrainHelperError(f"{_build.DRAIN_HELPER} is not built "
                                   "(python -m hipsnapshot._build)")
        self.pid_owner = os.getpid()
        self.proc = subprocess.Popen([_build.DRAIN_HELPER, rt, _build.HSGPU_SO],
                                     stdin=subprocess.PIPE, stdout=subprocess.PIPE,
                                     close_fds=True)
        self._w = self.proc.stdin.fileno()
        self._r = self.proc.stdout.fileno()
        self._send(struct.pack("=II", _MAGIC, _OP_PING))
        rc, pid = struct.unpack("=ii", self._recv(8, timeout=60.0))
        if rc != 0 or pid != self.proc.pid:
            raise DrainHelperError(f"drain helper handshake failed ({rc}, {pid})")

    # -- pipe ---------------------------------------------------------------
    def _send(self, data: bytes) -> None:
        mv = memoryview(data)
        try:
            while mv:
                n = os.write(self._w, mv)
                mv = mv[n:]
        except OSError as e:
            raise DrainHelperError(f"drain helper is gone ({e})") from e

    def _recv(self, n: int, timeout: Optional[float] = None, poke=None) -> bytes:
        """``n`` reply bytes.  The helper's liveness is checked every few
        seconds; ``timeout`` (s) bounds the whole wait (None = the drain
        timeout knob)."""
        from .. import knobs

        limit = knobs.drain_helper_timeout_s() if timeout is None else timeout
        t_end = time.monotonic() + limit if limit > 0 else None
        parts, left = [], n
        while left:
            while True:
                slot = 5.0 if poke is None else 0.05
                wait = slot if t_end is None else min(slot, t_end - time.monotonic())
                if wait <= 0:
                    self.proc.kill()
                    cls = DrainHelperMapTimeout if timeout is not None else DrainHelperError
                    raise cls(f"drain helper did not answer within {limit:.0f} s (killed)")
                ready, _, _ = select.select([self._r], [], [], wait)
                if ready:
                    break
                if poke is not None:
                    poke()
                if self.proc.poll() is not None:
                    raise DrainHelperError(
                        f"drain helper exited (status {self.proc.returncode})")
            b = os.read(self._r, left)  # the GIL is released while select waits
            if not b:
                code = self.proc.poll()
                raise DrainHelperError(f"drain helper exited (status {code})")
            parts.append(b)
            left -= len(b)
        return b"".join(parts)

    # -- requests -----------------------------------------------------------
    def close_handle(self, handle: bytes) -> None:
        self._send(struct.pack("=III", _MAGIC, _OP_CLOSE, len(handle)) + handle)
        (rc,) = struct.unpack("=i", self._recv(4))
        if rc != 0:
            logger.warning(f"drain helper: unmapping an arena failed ({rc})")

    def drain(self, dev: int, handle: bytes, blobs: Sequence[Tuple[int, int, str]],
              slot_bytes: int, nslots: int, nwriters: int, flags: int, max_hash_grid: int,
              close_after: bool) -> Tuple[int, int, List[int], List[float], float, str]:
        """blobs: (offset in the exported allocation, bytes, path).  Returns
        (rc, bytes written, hs64 partial sums, stats, map seconds, message)."""
        parts = [struct.pack("=IIiI", _MAGIC, _OP_DRAIN, dev, len(handle)), handle,
                 struct.pack("=QiiiiII", slot_bytes, nslots, nwriters, flags, max_hash_grid,
                             1 if close_after else 0, len(blobs))]
        for off, n, path in blobs:
            p = os.fsencode(path)
            parts.append(struct.pack("=QQI", off, n, len(p)))
            parts.append(p)
        self._send(b"".join(parts))
        from .. import knobs

        poke = None
        if knobs.drain_helper_poke():
            from ..ops import native

            lib = native.require_gpu_lib()
            poke = lambda: lib.hsg_runtime_poke(dev)  # noqa: E731
        (mapped,) = struct.unpack("=i", self._recv(4, timeout=knobs.drain_helper_map_timeout_s(),
                                                   poke=poke))
        rc, written, n = struct.unpack("=iQI", self._recv(16))
        sums = list(struct.unpack(f"={n}Q", self._recv(8 * n))) if n else []
        (nstats,) = struct.unpack("=I", self._recv(4))
        stats = list(struct.unpack(f"={nstats}d", self._recv(8 * nstats)))
        map_s, mlen = struct.unpack("=dI", self._recv(12))
        msg = self._recv(mlen).decode(errors="replace") if mlen else ""
        return rc, written, sums, stats, map_s, msg

    def shutdown(self) -> None:
        try:
            self.proc.stdin.close()  # EOF: the helper unmaps and exits
        except OSError:
            pass
        try:
            self.proc.wait(timeout=10)
        except subprocess.TimeoutExpired:
            self.proc.kill()
            self.proc.wait()


_lock = threading.Lock()
_helper: Optional[DrainHelper] = None
_start_failed: Optional[str] = None
_mapped: Dict[int, bytes] = {}  # kept arena data_ptr -> handle mapped in the helper
_to_close: List[bytes] = []     # unmaps to send before the next job


def _get() -> Optional[DrainHelper]:
    """The helper (started on first use); None if it cannot run here."""
    global _helper, _start_failed
    if _helper is not None and _helper.pid_owner != os.getpid():
        _helper = None  # forked child: the pipe belongs to the parent
        _mapped.clear()
        _to_close.clear()
    if _helper is None and _start_failed is None:
        try:
            _helper = DrainHelper()
        except (DrainHelperError, OSError) as e:
            _start_failed = str(e)
            logger.warning(f"drain helper unavailable, draining in process: {e}")
    return _helper


def available() -> bool:
    with _lock:
        return _get() is not None


def forget_arena(ptr: int) -> None:
    """A kept arena is being dropped: unmap it in the helper now when the
    helper is idle (its mapping would otherwise pin the memory), else before
    its next job (never blocks: a drain may hold the pipe for seconds)."""
    h = _mapped.pop(ptr, None)
    if h is None:
        return
    _to_close.append(h)
    if _lock.acquire(blocking=False):
        try:
            helper = _helper
            if helper is not None and helper.pid_owner == os.getpid():
                while _to_close:
                    helper.close_handle(_to_close.pop())
        except DrainHelperError as e:
            logger.warning(f"drain helper: unmapping a released arena failed: {e}")
        finally:
            _lock.release()


def drain(dev: int, arena_ptr: int, kept: bool, blobs: Sequence[Tuple[int, int, str]],
          slot_bytes: int, nslots: int, nwriters: int, flags: int,
          max_hash_grid: int) -> Optional[Tuple[List[int], int, Dict[str, float]]]:
    """Drain ``blobs`` ((offset in the arena, bytes, path)) of the arena at
    ``arena_ptr`` in the helper.  Returns (hs64 partial sums, bytes written,
    stats) or None when the helper cannot take the job (run it in process)."""
    from ..ops import native

    global _helper, _start_failed
    with _lock:
        helper = _get()
        if helper is None:
            return None
        try:
            handle, base_off, _size = native.ipc_export(arena_ptr)
        except native.HipError as e:
            logger.warning(f"drain helper: cannot export the arena, draining in process: {e}")
            return None
        try:
            while _to_close:
                helper.close_handle(_to_close.pop())
            rc, written, sums, stats, map_s, msg = helper.drain(
                dev, handle, [(base_off + off, n, p) for off, n, p in blobs], slot_bytes,
                nslots, nwriters, flags, max_hash_grid, close_after=not kept)
        except DrainHelperMapTimeout as e:
            # the arena could not be mapped in time: drain in process, now and
            # for the rest of this process
            logger.warning(f"{e}; draining in process from now on")
            _start_failed = str(e)
            dead, _helper = _helper, None
            _mapped.clear()
            _to_close.clear()
            dead.shutdown()
            return None
        except DrainHelperError:
            dead, _helper = _helper, None
            _mapped.clear()
            _to_close.clear()
            dead.shutdown()
            raise
        if rc == -10000:
            # mapping refused (IPC unsupported here): in process from now on
            logger.warning(f"drain helper: {msg}; draining in process")
            _helper = None
            _start_failed = msg
            helper.shutdown()
            return None
        if kept:
            _mapped[arena_ptr] = handle
    from ..ops.native import NativeDrain

    st = {k: round(v, 4) for k, v in zip(NativeDrain.STATS, stats)}
    st["ipc_map"] = round(map_s, 4)
    if rc != 0:
        if rc < 0 and -rc in errno.errorcode:
            raise OSError(-rc, msg)
        raise native.HipError(f"native drain (helper process) failed ({rc}): {msg}")
    return sums, written, st


def shutdown() -> None:
    global _helper
    with _lock:
        if _helper is not None and _helper.pid_owner == os.getpid():
            _helper.shutdown()
        _helper = None
        _mapped.clear()
        _to_close.clear()


atexit.register(shutdown)
