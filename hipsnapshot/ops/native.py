"""ctypes bindings for the native libraries (``_hsio.so`` and ``_hsgpu.so``).

Loading policy:

* ``_hsio.so`` (file I/O engine) is built on demand if missing -- it only needs
  a C++ compiler -- and is used on every machine.
* ``_hsgpu.so`` (HIP data plane) is REQUIRED whenever a GPU is visible: GPU
  tensors never silently fall back to ATen copies.  ``require_gpu_lib()`` raises
  with the build command if the library is missing or fails to load.

``torch`` is always imported before ``_hsgpu.so`` is dlopen'ed so the HIP
runtime resolved for our library is the one torch already loaded (same SONAME
``libamdhip64.so.7``) -- one HIP runtime, shared streams and contexts.
"""

from __future__ import annotations

import ctypes
import errno
import logging
import os
import threading
from typing import Dict, List, Optional, Sequence, Tuple

import numpy as np
import torch

from .. import _build

logger = logging.getLogger(__name__)

_lock = threading.Lock()
_hsio_lib: Optional[ctypes.CDLL] = None
_hsgpu_lib: Optional[ctypes.CDLL] = None
_hsgpu_error: Optional[str] = None

c_void_p = ctypes.c_void_p
c_int = ctypes.c_int
c_int64 = ctypes.c_int64
c_uint64 = ctypes.c_uint64
c_char_p = ctypes.c_char_p


def _declare(lib: ctypes.CDLL, name: str, restype, argtypes) -> None:
    fn = getattr(lib, name)
    fn.restype = restype
    fn.argtypes = argtypes


# ---------------------------------------------------------------------------
# _hsio.so
# ---------------------------------------------------------------------------

def hsio() -> ctypes.CDLL:
    global _hsio_lib
    if _hsio_lib is not None:
        return _hsio_lib
    with _lock:
        if _hsio_lib is None:
            path = _build.HSIO_SO
            if not os.path.exists(path):
                _build.build_hsio()
            lib = ctypes.CDLL(path)
            _declare(lib, "hsio_create", c_void_p, [c_int])
            _declare(lib, "hsio_destroy", None, [c_void_p])
            _declare(lib, "hsio_eventfd", c_int, [c_void_p])
            _declare(lib, "hsio_set_read_split", None, [c_void_p, c_uint64])
            _declare(lib, "hsio_submit_write", c_int64,
                     [c_void_p, c_char_p, c_void_p, c_uint64, c_uint64, c_int])
            _declare(lib, "hsio_submit_read", c_int64,
                     [c_void_p, c_char_p, c_void_p, c_uint64, c_uint64, c_int])
            _declare(lib, "hsio_submit_delete", c_int64, [c_void_p, c_char_p])
            _declare(lib, "hsio_poll", c_int,
                     [c_void_p, ctypes.POINTER(c_int64), ctypes.POINTER(c_int64), c_int])
            _declare(lib, "hsio_write_sync", c_int64,
                     [c_void_p, c_char_p, c_void_p, c_uint64, c_uint64, c_int])
            _declare(lib, "hsio_read_sync", c_int64,
                     [c_void_p, c_char_p, c_void_p, c_uint64, c_uint64, c_int])
            _declare(lib, "hsio_file_size", c_int64, [c_char_p])
            _declare(lib, "hsio_alloc_aligned", c_void_p, [c_uint64])
            _declare(lib, "hsio_free_aligned", None, [c_void_p])
            _declare(lib, "hsio_parallel_memcpy", None, [c_void_p, c_void_p, c_uint64, c_int])
            _declare(lib, "hs64_partial", c_uint64, [c_void_p, c_uint64, c_uint64, c_int])
            _declare(lib, "hs64_finish", c_uint64, [c_uint64, c_uint64])
            _declare(lib, "hsz_max_encoded_bytes", c_uint64, [c_uint64, ctypes.c_uint32])
            _declare(lib, "hsz_encode_cpu", c_int64,
                     [c_void_p, c_uint64, c_int, ctypes.c_uint32, c_void_p, c_int])
            _declare(lib, "hsz_decode_cpu", c_int,
                     [c_void_p, c_void_p, ctypes.c_uint32, ctypes.c_uint32, c_uint64, c_int,
                      ctypes.c_uint32, c_void_p, c_int])
            _hsio_lib = lib
    return _hsio_lib


IO_DIRECT = 1
IO_SYNC = 2
IO_MKDIRS = 4
IO_APPEND = 8
IO_NODE_SHIFT = 16  # flags bits 16..23: NUMA node + 1 whose CPUs run the job


class IOEngine:
    """A C++ worker pool bound to one process (re-created after fork)."""

    def __init__(self, nthreads: int) -> None:
        self.lib = hsio()
        self.nthreads = nthreads
        self.pid = os.getpid()
        self.handle = self.lib.hsio_create(nthreads)
        self.efd = self.lib.hsio_eventfd(self.handle)
        from .. import knobs

        self.lib.hsio_set_read_split(self.handle, knobs.get_io_read_split_bytes())
        self._ids = (c_int64 * 256)()
        self._res = (c_int64 * 256)()

    def submit_write(self, path: str, addr: int, nbytes: int, offset: int, flags: int) -> int:
        return self.lib.hsio_submit_write(self.handle, path.encode(), addr, nbytes, offset, flags)

    def submit_read(self, path: str, addr: int, nbytes: int, offset: int, flags: int) -> int:
        return self.lib.hsio_submit_read(self.handle, path.encode(), addr, nbytes, offset, flags)

    def submit_delete(self, path: str) -> int:
        return self.lib.hsio_submit_delete(self.handle, path.encode())

    def poll(self) -> List[tuple]:
        out = []
        while True:
            k = self.lib.hsio_poll(self.handle, self._ids, self._res, 256)
            for i in range(k):
                out.append((self._ids[i], self._res[i]))
            if k < 256:
                return out

    def write_sync(self, path: str, addr: int, nbytes: int, offset: int, flags: int) -> int:
        return self.lib.hsio_write_sync(self.handle, path.encode(), addr, nbytes, offset, flags)

    def read_sync(self, path: str, addr: int, nbytes: int, offset: int, flags: int) -> int:
        return self.lib.hsio_read_sync(self.handle, path.encode(), addr, nbytes, offset, flags)

    def close(self) -> None:
        if self.handle and os.getpid() == self.pid:
            self.lib.hsio_destroy(self.handle)
        self.handle = None


_engines = {}


def io_engine(nthreads: int = 16) -> IOEngine:
    """Process-wide shared engine (per thread count)."""
    key = (os.getpid(), nthreads)
    eng = _engines.get(key)
    if eng is None:
        with _lock:
            eng = _engines.get(key)
            if eng is None:
                eng = IOEngine(nthreads)
                _engines[key] = eng
    return eng


_idle_engines: Dict[Tuple[int, int], List[IOEngine]] = {}
_MAX_IDLE_ENGINES = 4


def acquire_io_engine(nthreads: int) -> IOEngine:
    """An engine for one storage plugin's exclusive use: an idle one left by a
    closed plugin, else a new one.  A take opens one plugin, so reusing the
    engine saves starting and joining ``nthreads`` threads per take."""
    with _lock:
        lst = _idle_engines.get((os.getpid(), nthreads))
        if lst:
            return lst.pop()
    return IOEngine(nthreads)


def release_io_engine(eng: IOEngine, reusable: bool) -> None:
    """Return an engine from ``acquire_io_engine``.  Only an engine with no
    job in flight may be reused (``reusable``): a later owner must never see a
    completion it did not submit."""
    if reusable and eng.handle and os.getpid() == eng.pid:
        with _lock:
            lst = _idle_engines.setdefault((eng.pid, eng.nthreads), [])
            if len(lst) < _MAX_IDLE_ENGINES:
                lst.append(eng)
                return
    eng.close()


def file_size(path: str) -> int:
    r = hsio().hsio_file_size(path.encode())
    if r < 0:
        raise OSError(-r, os.strerror(-r), path)
    return r


def parallel_memcpy(dst: int, src: int, nbytes: int, nthreads: int = 8) -> None:
    hsio().hsio_parallel_memcpy(dst, src, nbytes, nthreads)


def address_of(buf) -> int:
    """Address of a writable/readable contiguous buffer (memoryview/bytearray/ndarray)."""
    if isinstance(buf, torch.Tensor):
        return buf.data_ptr()
    arr = np.frombuffer(buf, dtype=np.uint8)
    return arr.ctypes.data


# ---------------------------------------------------------------------------
# _hsgpu.so
# ---------------------------------------------------------------------------

_gpu_seen = False


def gpu_available() -> bool:
    """torch.cuda.is_available(), remembered once true (it is asked per
    destination while a restore is planned)."""
    global _gpu_seen
    if not _gpu_seen:
        _gpu_seen = torch.cuda.is_available()
    return _gpu_seen


def _load_hsgpu() -> Optional[ctypes.CDLL]:
    global _hsgpu_lib, _hsgpu_error
    if _hsgpu_lib is not None or _hsgpu_error is not None:
        return _hsgpu_lib
    with _lock:
        if _hsgpu_lib is not None or _hsgpu_error is not None:
            return _hsgpu_lib
        path = _build.HSGPU_SO
        try:
            if not os.path.exists(path):
                _build.build_hsgpu()
            lib = ctypes.CDLL(path)
        except Exception as e:  # noqa: BLE001
            _hsgpu_error = f"{type(e).__name__}: {e}"
            return None
        _declare(lib, "hsg_last_error", c_char_p, [])
        _declare(lib, "hsg_device_count", c_int, [])
        _declare(lib, "hsg_pci_location", c_int,
                 [c_int, ctypes.POINTER(c_int), ctypes.POINTER(c_int), ctypes.POINTER(c_int)])
        _declare(lib, "hsg_pinned_acquire", c_void_p, [c_uint64])
        _declare(lib, "hsg_pinned_release", c_int, [c_void_p])
        _declare(lib, "hsg_pinned_acquire_on", c_void_p, [c_uint64, c_int])
        _declare(lib, "hsg_pinned_stats", None, [ctypes.POINTER(c_uint64), ctypes.POINTER(c_uint64)])
        _declare(lib, "hsg_pinned_trim", c_uint64, [])
        _declare(lib, "hsg_pinned_set_limit", None, [c_uint64])
        from .. import knobs

        lib.hsg_pinned_set_limit(knobs.pinned_pool_max_bytes())
        _declare(lib, "hsg_memcpy", c_int,
                 [c_int, c_int, c_void_p, c_void_p, c_uint64, c_int, c_void_p, c_int, c_int])
        _declare(lib, "hsg_stream_join", c_int, [c_int, c_int, c_void_p])
        _declare(lib, "hsg_stream_sync", c_int, [c_int, c_int])
        _declare(lib, "hsg_copy_stream", c_void_p, [c_int, c_int])
        _declare(lib, "hsg_sync_stream_handle", c_int, [c_void_p])
        _declare(lib, "hsg_desc_size", c_uint64, [])
        _declare(lib, "hsg_prewarm_module", c_int, [c_int])
        _declare(lib, "hsg_copy_workspace_bytes", c_uint64, [c_void_p, c_int])
        _declare(lib, "hsg_copy_nd", c_int,
                 [c_int, c_void_p, c_int, c_void_p, c_uint64, c_void_p, c_void_p, c_int])
        _declare(lib, "hsg_fp8_quantize", c_int,
                 [c_int, c_void_p, c_int, c_int64, c_void_p, c_void_p, c_int, c_void_p])
        _declare(lib, "hsg_fp8_dequantize", c_int,
                 [c_int, c_void_p, c_void_p, c_int64, c_void_p, c_int, c_int, c_void_p])
        _declare(lib, "hsg_fp8_hadamard_quantize", c_int,
                 [c_int, c_void_p, c_int, c_int64, c_void_p, c_void_p, c_void_p])
        _declare(lib, "hsg_fp8_hadamard_dequantize", c_int,
                 [c_int, c_void_p, c_void_p, c_int64, c_void_p, c_int, c_void_p])
        _declare(lib, "hsg_mx8_quantize", c_int,
                 [c_int, c_void_p, c_int, c_int64, c_void_p, c_void_p, c_void_p])
        _declare(lib, "hsg_mx8_dequantize", c_int,
                 [c_int, c_void_p, c_void_p, c_int64, c_void_p, c_int, c_void_p])
        _declare(lib, "hsg_drain_start", c_void_p,
                 [c_int, c_int, ctypes.POINTER(c_uint64), ctypes.POINTER(c_uint64),
                  ctypes.POINTER(c_char_p), c_uint64, c_int, c_int, c_int, c_int,
                  ctypes.POINTER(c_int)])
        _declare(lib, "hsg_drain_wait", c_int,
                 [c_void_p, ctypes.POINTER(c_uint64), ctypes.POINTER(c_uint64), c_char_p,
                  ctypes.POINTER(ctypes.c_double)])
        _declare(lib, "hsg_drain_pending", c_int, [c_void_p])
        _declare(lib, "hsg_drain_boost", None, [c_void_p])
        P = ctypes.POINTER
        _declare(lib, "hsg_restore_start", c_void_p,
                 [c_int, c_int, P(c_char_p), P(c_uint64), P(c_uint64), P(c_int), P(c_uint64),
                  P(c_uint64), P(c_uint64), P(c_int64), P(c_int), c_void_p, c_int64,
                  P(c_uint64), c_int, c_void_p, c_uint64, c_uint64, c_uint64, c_int, c_int,
                  c_uint64, c_int, P(c_int), c_int, P(c_int)])
        _declare(lib, "hsg_restore_wait", c_int,
                 [c_void_p, P(c_int), c_char_p, P(ctypes.c_double), P(c_uint64), P(c_uint64)])
        _declare(lib, "hsg_restore_trim", c_uint64, [c_int, c_uint64])
        _declare(lib, "hsg_restore_trim_pools", c_uint64, [c_int, c_uint64, c_uint64])
        _declare(lib, "hsg_restore_pool_bytes", None, [c_int, P(c_uint64)])
        _declare(lib, "hsg_uncached_bytes", c_uint64, [])
        _declare(lib, "hsg_poison_idle_pools", c_int, [c_int, c_int])
        _declare(lib, "hsg_restore_prewarm", c_int,
                 [c_int, c_uint64, c_uint64, c_uint64, c_int, c_uint64])
        _declare(lib, "hsg_sdma_h2d_submit", c_int,
                 [c_int, c_void_p, c_void_p, c_uint64, P(c_uint64)])
        _declare(lib, "hsg_is_managed", c_int, [c_void_p])
        _declare(lib, "hsg_managed_location", c_int,
                 [c_void_p, c_uint64, ctypes.POINTER(c_int), ctypes.POINTER(c_int)])
        _declare(lib, "hsg_managed_place", c_int, [c_int, c_void_p, c_uint64, c_int, c_void_p])
        _declare(lib, "hsg_managed_alloc", c_void_p, [c_int, c_uint64])
        _declare(lib, "hsg_managed_free", c_int, [c_void_p])
        _declare(lib, "hsg_gate_supported", c_int, [c_int])
        _declare(lib, "hsg_gate_arm", c_int, [c_int, c_void_p, ctypes.POINTER(ctypes.c_uint32)])
        _declare(lib, "hsg_gate_release", c_int, [c_int, ctypes.c_uint32])
        _declare(lib, "hsg_gate_value", ctypes.c_uint32, [c_int])
        _declare(lib, "hsg_hsz_last_error", c_char_p, [])
        _declare(lib, "hsg_set_thread_grid_cap", c_int, [c_int])
        _declare(lib, "hsg_hash64", c_int, [c_int, c_int, c_int, c_void_p, c_uint64, c_uint64,
                                             c_int, ctypes.POINTER(c_int)])
        _declare(lib, "hsg_hash64_result", c_int, [c_int, c_int, c_int, ctypes.POINTER(c_uint64)])
        _declare(lib, "hsg_sdma_last_error", c_char_p, [])
        _declare(lib, "hsg_sdma_engines", c_int, [c_int])
        _declare(lib, "hsg_sdma_h2d", c_int, [c_int, c_void_p, c_void_p, c_uint64])
        _declare(lib, "hsg_uncached_acquire", c_void_p, [c_int, c_uint64])
        _declare(lib, "hsg_uncached_release", c_int, [c_void_p])
        _declare(lib, "hsg_uncached_trim", c_uint64, [])
        _declare(lib, "hsg_rt_dev_alloc", c_void_p, [c_int, c_uint64, c_int])
        _declare(lib, "hsg_rt_dev_free", None, [c_void_p])
        _declare(lib, "hsg_rt_memcpy_d2h", c_int, [c_void_p, c_void_p, c_uint64])
        _declare(lib, "hsg_rt_last_error", c_char_p, [])
        _declare(lib, "hsg_rt_set_trace", None, [c_int])
        _declare(lib, "hsg_rt_vmm_alloc", c_void_p, [c_int, c_uint64, c_int])
        _declare(lib, "hsg_rt_vmm_free", c_int, [c_void_p])
        _declare(lib, "hsg_rt_vmm_retired_bytes", c_uint64, [])
        _declare(lib, "hsg_sdma_d2h", c_int,
                 [c_int, c_void_p, c_void_p, c_uint64, c_int, c_void_p])
        _declare(lib, "hsg_sdma_d2h_submit", c_int,
                 [c_int, c_void_p, c_void_p, c_uint64, c_void_p, ctypes.POINTER(c_uint64)])
        _declare(lib, "hsg_sdma_wait", c_int, [c_uint64])
        _declare(lib, "hsg_hsz_meta_bytes", c_uint64, [ctypes.c_uint32])
        _declare(lib, "hsg_hsz_encode", c_int,
                 [c_int, c_void_p, c_uint64, c_int, ctypes.c_uint32, c_void_p, c_void_p,
                  c_void_p, c_void_p])
        _declare(lib, "hsg_hsz_decode", c_int,
                 [c_int, c_void_p, c_void_p, ctypes.c_uint32, ctypes.c_uint32, c_uint64, c_int,
                  ctypes.c_uint32, c_void_p, c_void_p, c_void_p])
        if lib.hsg_desc_size() != COPY_DESC_DTYPE.itemsize:
            _hsgpu_error = (f"CopyDesc layout mismatch: native {lib.hsg_desc_size()} "
                            f"vs python {COPY_DESC_DTYPE.itemsize}")
            return None
        _hsgpu_lib = lib
    return _hsgpu_lib


def hsgpu_loaded() -> bool:
    return _load_hsgpu() is not None


def require_gpu_lib() -> ctypes.CDLL:
    lib = _load_hsgpu()
    if lib is None:
        raise RuntimeError(
            "hipsnapshot's HIP data plane (_hsgpu.so) is unavailable: "
            f"{_hsgpu_error}. Build it with `python -m hipsnapshot._build` "
            "(hipcc --offload-arch=gfx950).")
    return lib


class HipError(RuntimeError):
    pass


def _check(rc: int, what: str) -> None:
    if rc != 0:
        lib = _load_hsgpu()
        msg = lib.hsg_last_error().decode() if lib is not None else "?"
        raise HipError(f"{what} failed ({rc}): {msg}")


_prewarmed: set = set()


def prewarm_module(dev: int, pool) -> None:
    """Load the HIP code object of ``_hsgpu.so`` on ``dev`` on a thread of
    ``pool`` while the caller goes on planning.  The library is opened here
    (Python work under the GIL), the load itself runs in the ctypes call,
    which releases the GIL."""
    if dev in _prewarmed:
        return
    _prewarmed.add(dev)
    lib = _load_hsgpu()
    if lib is not None:
        pool.submit(lib.hsg_prewarm_module, dev)


class PinnedBuffer:
    """A page-locked host block from the native caching pool.

    ``view`` is a writable memoryview over the first ``nbytes`` bytes; the
    block goes back to the pool on :meth:`release` (idempotent) or GC.
    """

    __slots__ = ("ptr", "nbytes", "_released", "_cbuf", "__weakref__")

    def __init__(self, nbytes: int, node: Optional[int] = None) -> None:
        lib = require_gpu_lib()
        ptr = None
        if node is not None and node >= 0:  # pages bound to that NUMA node
            ptr = lib.hsg_pinned_acquire_on(max(int(nbytes), 1), int(node))
        if not ptr:
            ptr = lib.hsg_pinned_acquire(max(int(nbytes), 1))
        if not ptr:
            raise MemoryError(f"pinned allocation of {nbytes} bytes failed: "
                              f"{lib.hsg_last_error().decode()}")
        self.ptr = ptr
        self.nbytes = int(nbytes)
        self._released = False
        self._cbuf = (ctypes.c_char * max(self.nbytes, 1)).from_address(ptr)

    @property
    def view(self) -> memoryview:
        return memoryview(self._cbuf).cast("B")[: self.nbytes]

    def as_tensor(self, nbytes: Optional[int] = None) -> torch.Tensor:
        n = self.nbytes if nbytes is None else nbytes
        if n == 0:
            return torch.empty(0, dtype=torch.uint8)
        return torch.frombuffer(self._cbuf, dtype=torch.uint8, count=n)

    def release(self) -> None:
        if not self._released:
            self._released = True
            lib = _load_hsgpu()
            if lib is not None:
                lib.hsg_pinned_release(self.ptr)

    def __del__(self) -> None:  # pragma: no cover - GC path
        try:
            self.release()
        except Exception:
            pass


def pci_location(dev: int) -> Optional[Tuple[int, int, int]]:
    """(domain, bus, device) of HIP device ``dev``, or None."""
    lib = require_gpu_lib()
    d, b, v = c_int(0), c_int(0), c_int(0)
    if lib.hsg_pci_location(dev, ctypes.byref(d), ctypes.byref(b), ctypes.byref(v)) != 0:
        return None
    return int(d.value), int(b.value), int(v.value)


def pinned_stats() -> tuple:
    lib = require_gpu_lib()
    a, b = c_uint64(), c_uint64()
    lib.hsg_pinned_stats(ctypes.byref(a), ctypes.byref(b))
    return a.value, b.value


def pinned_trim() -> int:
    return int(require_gpu_lib().hsg_pinned_trim())


# ---- DMA ------------------------------------------------------------------

D2H, H2D, D2D = 0, 1, 2


def _stream_handle(stream) -> int:
    if stream is None:
        return 0
    if isinstance(stream, int):
        return stream
    return int(stream.cuda_stream)


def memcpy(dev: int, slot: int, dst: int, src: int, nbytes: int, kind: int,
           producer=None, sync: bool = True) -> None:
    """DMA on copy stream (dev, slot).  ``producer``: stream (or raw handle;
    0 = torch's default/null stream) whose queued work must finish first;
    None = no ordering."""
    lib = require_gpu_lib()
    _check(lib.hsg_memcpy(dev, slot, dst, src, nbytes, kind, _stream_handle(producer),
                          int(producer is not None),
                          1 if sync else 0), "hsg_memcpy")


def set_thread_grid_cap(cap: int) -> int:
    """Cap the grid of this thread's data-plane launches (copy gathers, HSZ1
    encode) at ``cap`` workgroups, i.e. about that many CUs; 0 = no cap.
    Returns the previous cap."""
    return int(require_gpu_lib().hsg_set_thread_grid_cap(int(cap)))


def sdma_engines(dev: int) -> int:
    """SDMA engines usable for device -> host copies of ``dev`` (0 = none:
    the SDMA path is unavailable and hipMemcpyAsync is used)."""
    return int(require_gpu_lib().hsg_sdma_engines(dev))


def sdma_d2h(dev: int, dst: int, src: int, nbytes: int, stream=None,
             max_engines: int = 0) -> None:
    """Blocking device -> pinned-host copy on the SDMA engines, ordered after
    the work queued on ``stream`` (handle or torch stream; None/0 = the null
    stream).  ``max_engines`` 0 = every free engine."""
    lib = require_gpu_lib()
    r = lib.hsg_sdma_d2h(dev, dst, src, nbytes, max_engines, _stream_handle(stream) or None)
    if r != 0:
        msg = lib.hsg_sdma_last_error()
        raise HipError(f"hsg_sdma_d2h failed ({r}): {msg.decode() if msg else ''}")


def sdma_h2d(dev: int, dst: int, src: int, nbytes: int) -> None:
    """Blocking pinned-host -> device copy on an SDMA engine.  ``dst`` must be
    an ``UncachedBlock`` (the GPU reads it without an L2, so the copy needs no
    acquire before kernels read it)."""
    lib = require_gpu_lib()
    r = lib.hsg_sdma_h2d(dev, dst, src, nbytes)
    if r != 0:
        msg = lib.hsg_sdma_last_error()
        raise HipError(f"hsg_sdma_h2d failed ({r}): {msg.decode() if msg else ''}")


class UncachedBlock:
    """Device memory the GPU never caches (hipDeviceMallocUncached), from a
    per-device caching pool: the target of SDMA uploads."""

    __slots__ = ("ptr", "dev", "nbytes", "_released", "__weakref__")

    def __init__(self, dev: int, nbytes: int) -> None:
        lib = require_gpu_lib()
        ptr = lib.hsg_uncached_acquire(dev, max(int(nbytes), 1))
        if not ptr:
            raise torch.cuda.OutOfMemoryError(
                f"uncached device allocation of {nbytes} bytes failed: "
                f"{lib.hsg_last_error().decode()}")
        self.ptr, self.dev, self.nbytes, self._released = ptr, dev, int(nbytes), False

    def release(self) -> None:
        if not self._released:
            self._released = True
            lib = _load_hsgpu()
            if lib is not None:
                lib.hsg_uncached_release(self.ptr)

    def __del__(self) -> None:  # pragma: no cover - GC path
        try:
            self.release()
        except Exception:
            pass


def uncached_trim() -> int:
    return int(require_gpu_lib().hsg_uncached_trim())


def sdma_d2h_submit(dev: int, dst: int, src: int, nbytes: int, stream=None) -> int:
    """Submit one device -> pinned-host SDMA copy ordered after ``stream``;
    returns the handle ``sdma_wait`` takes (exactly once)."""
    lib = require_gpu_lib()
    h = c_uint64(0)
    r = lib.hsg_sdma_d2h_submit(dev, dst, src, nbytes, _stream_handle(stream) or None,
                                ctypes.byref(h))
    if r != 0:
        msg = lib.hsg_sdma_last_error()
        raise HipError(f"hsg_sdma_d2h_submit failed ({r}): {msg.decode() if msg else ''}")
    return h.value


def sdma_wait(handle: int) -> None:
    lib = require_gpu_lib()
    r = lib.hsg_sdma_wait(handle)
    if r != 0:
        msg = lib.hsg_sdma_last_error()
        raise HipError(f"hsg_sdma_wait failed ({r}): {msg.decode() if msg else ''}")


def copy_stream(dev: int, slot: int) -> int:
    h = require_gpu_lib().hsg_copy_stream(dev, slot)
    if not h:
        raise HipError("hsg_copy_stream failed")
    return h


def stream_join(dev: int, slot: int, consumer) -> None:
    _check(require_gpu_lib().hsg_stream_join(dev, slot, _stream_handle(consumer)),
           "hsg_stream_join")


def stream_sync(dev: int, slot: int) -> None:
    _check(require_gpu_lib().hsg_stream_sync(dev, slot), "hsg_stream_sync")


def sync_stream_handle(handle: int) -> None:
    _check(require_gpu_lib().hsg_sync_stream_handle(handle), "hsg_sync_stream_handle")


# ---- batched strided copy / cast --------------------------------------------

MAX_DIMS = 8
COPY_DESC_DTYPE = np.dtype([
    ("src", np.uint64), ("dst", np.uint64), ("numel", np.int64),
    ("ndim", np.int32), ("src_dtype", np.int32), ("dst_dtype", np.int32),
    ("flags", np.int32),
    ("sizes", np.int64, (MAX_DIMS,)), ("src_strides", np.int64, (MAX_DIMS,)),
    ("dst_strides", np.int64, (MAX_DIMS,)),
])

_RAW_CODE = {1: 0, 2: 1, 4: 2, 8: 3, 16: 4}
_FLOAT_CODE = {torch.float16: 10, torch.bfloat16: 11, torch.float32: 12, torch.float64: 13}


def dtype_code(dtype: torch.dtype) -> int:
    return _FLOAT_CODE.get(dtype, -1)


def can_cast_on_device(src: torch.dtype, dst: torch.dtype) -> bool:
    if src == dst:
        return True
    return src in _FLOAT_CODE and dst in _FLOAT_CODE


def collapse_dims(sizes: Sequence[int], s_strides: Sequence[int],
                  d_strides: Sequence[int]) -> tuple:
    """Drop size-1 dims and merge adjacent dims that are jointly contiguous."""
    dims = [(int(z), int(a), int(b)) for z, a, b in zip(sizes, s_strides, d_strides) if z != 1]
    if not dims:
        return [1], [1], [1]
    out = [dims[0]]
    for z, a, b in dims[1:]:
        pz, pa, pb = out[-1]
        if pa == a * z and pb == b * z:
            out[-1] = (pz * z, a, b)
        else:
            out.append((z, a, b))
    return [d[0] for d in out], [d[1] for d in out], [d[2] for d in out]


def _fast_mode(src_ptr: int, dst_ptr: int, z, a, b, es: int):
    """Pick a specialised kernel path for a same-dtype strided copy.

    * rows (flags 2): 2-D, inner dim contiguous on both sides -> vectorised
      row copies (column shards, narrowed views); vector width in flags >> 8.
    * transpose (flags 4): src contiguous along one dim, dst along another ->
      LDS-tiled 64x64 transpose; canonical dims [B, I, J].
    """
    if len(z) == 2 and a[1] == 1 and b[1] == 1:
        row_bytes = z[1] * es
        vw = 16
        while vw > 1 and (row_bytes % vw or src_ptr % vw or dst_ptr % vw
                          or (a[0] * es) % vw or (b[0] * es) % vw):
            vw //= 2
        return 2 | (vw << 8), z, a, b
    if len(z) in (2, 3):
        i = next((k for k in range(len(z)) if a[k] == 1), None)
        j = next((k for k in range(len(z)) if b[k] == 1), None)
        if i is None or j is None or i == j:
            return None
        rest = [k for k in range(len(z)) if k not in (i, j)]
        order = rest + [i, j]
        zz, aa, bb = [z[k] for k in order], [a[k] for k in order], [b[k] for k in order]
        if len(zz) == 2:
            zz, aa, bb = [1] + zz, [0] + aa, [0] + bb
        return 4, zz, aa, bb
    return None


_ZPAD = [(0,) * (MAX_DIMS - k) for k in range(MAX_DIMS + 1)]


class CopyBatch:
    """Accumulates strided copy/cast descriptors executed by ONE kernel launch."""

    def __init__(self) -> None:
        self.rows: List[tuple] = []

    def __len__(self) -> int:
        return len(self.rows)

    def add(self, src_ptr: int, src_dtype: torch.dtype, src_strides: Sequence[int],
            dst_ptr: int, dst_dtype: torch.dtype, dst_strides: Sequence[int],
            sizes: Sequence[int], elem_size: int) -> None:
        numel = 1
        for z in sizes:
            numel *= int(z)
        if numel == 0:
            return
        z, a, b = collapse_dims(sizes, src_strides, dst_strides)
        if len(z) > MAX_DIMS:
            raise ValueError(f"too many non-mergeable dims ({len(z)}) for the copy kernel")
        if src_dtype == dst_dtype or elem_size == 16:
            sc = dc = _RAW_CODE[elem_size]
        else:
            sc, dc = dtype_code(src_dtype), dtype_code(dst_dtype)
            if sc < 0 or dc < 0:
                raise ValueError(f"device cast {src_dtype}->{dst_dtype} unsupported")
        flags = 1 if (sc == dc and len(z) == 1 and a[0] == 1 and b[0] == 1) else 0
        if not flags and sc == dc and elem_size <= 8:
            mode = _fast_mode(src_ptr, dst_ptr, z, a, b, elem_size)
            if mode is not None:
                flags, z, a, b = mode
        self.rows.append((src_ptr, dst_ptr, numel, len(z), sc, dc, flags, z, a, b))

    def add_bytes(self, src_ptr: int, dst_ptr: int, nbytes: int) -> None:
        """Contiguous byte copy (the common case: no stride analysis needed)."""
        if nbytes > 0:
            self.rows.append((src_ptr, dst_ptr, nbytes, 1, 0, 0, 1, (nbytes,), (1,), (1,)))

    def add_tensor(self, t: torch.Tensor, dst_ptr: int) -> None:
        """Copy ``t`` (any strides) into C-order bytes at ``dst_ptr``."""
        if t.is_contiguous():
            self.add_bytes(t.data_ptr(), dst_ptr, t.numel() * t.element_size())
            return
        st = [1] * t.dim()
        for i in range(t.dim() - 2, -1, -1):
            st[i] = st[i + 1] * max(int(t.shape[i + 1]), 1)
        self.add(t.data_ptr(), t.dtype, t.stride(), dst_ptr, t.dtype, st, list(t.shape),
                 t.element_size())

    def pack(self) -> np.ndarray:
        """Descriptor table, filled column-wise (per-row structured-array
        assignment costs ~10 us a row: milliseconds for a model's state)."""
        n = len(self.rows)
        arr = np.zeros(n, dtype=COPY_DESC_DTYPE)
        if not n:
            return arr
        cols = list(zip(*self.rows))
        if all(d == 1 for d in cols[3]):
            # every row one run (contiguous copies: a freeze of a model's
            # tensors): fill column 0 of the shape/stride tables directly
            for field, v in (("src", cols[0]), ("dst", cols[1])):
                arr[field] = np.asarray(v, dtype=np.uint64)
            arr["numel"] = cols[2]
            arr["ndim"] = 1
            arr["src_dtype"] = cols[4]
            arr["dst_dtype"] = cols[5]
            arr["flags"] = cols[6]
            arr["sizes"][:, 0] = [z[0] for z in cols[7]]
            arr["src_strides"][:, 0] = [a[0] for a in cols[8]]
            arr["dst_strides"][:, 0] = [b[0] for b in cols[9]]
            return arr
        arr["src"] = np.asarray(cols[0], dtype=np.uint64)
        arr["dst"] = np.asarray(cols[1], dtype=np.uint64)
        arr["numel"] = cols[2]
        arr["ndim"] = cols[3]
        arr["src_dtype"] = cols[4]
        arr["dst_dtype"] = cols[5]
        arr["flags"] = cols[6]
        for field, col in (("sizes", cols[7]), ("src_strides", cols[8]),
                           ("dst_strides", cols[9])):
            # rows padded in Python, converted once (a slice assignment per
            # row cost ~2 ms per 300-row table)
            pad = [tuple(v) + _ZPAD[len(v)] for v in col]
            arr[field] = np.array(pad, dtype=np.int64).reshape(n, MAX_DIMS)
        return arr

    def launch(self, dev: int, stream_handle: int, sync: bool = True) -> None:
        """Run all descriptors in one launch on ``stream_handle``.

        The descriptor/tile tables go through a pinned staging block and a
        device workspace that are kept alive until the stream has passed them
        (``sync=True``) -- callers that pass ``sync=False`` must keep the
        returned objects alive until they synchronize the stream.
        """
        if not self.rows:
            return None
        from ..utils.tracing import timeline

        with timeline.span("copy_pack", n=len(self.rows)):
            arr = self.pack()
        return launch_packed(arr, dev, stream_handle, sync)


def launch_packed(arr: np.ndarray, dev: int, stream_handle: int, sync: bool = True):
    """``CopyBatch.launch`` of an already packed descriptor table (a caller
    that launches the same copies again -- the async-take freeze of a reused
    take plan -- keeps the table instead of rebuilding it)."""
    if not len(arr):
        return None
    from ..utils.tracing import timeline

    lib = require_gpu_lib()
    ws_bytes = int(lib.hsg_copy_workspace_bytes(arr.ctypes.data, len(arr)))
    with timeline.span("copy_stage_alloc", bytes=ws_bytes):
        stage = PinnedBuffer(ws_bytes)
    ws = torch.empty(ws_bytes, dtype=torch.uint8, device=f"cuda:{dev}")
    cur = torch.cuda.current_stream(dev)
    if int(cur.cuda_stream) != int(stream_handle):
        # ``ws`` comes from torch's caching allocator in the CURRENT
        # stream's order: its block may have been freed a moment ago by
        # another thread (the trainer) with kernels still queued on that
        # stream.  The launch stream must not write it before they ran.
        ev = torch.cuda.Event()
        ev.record(cur)
        torch.cuda.ExternalStream(int(stream_handle), device=f"cuda:{dev}").wait_event(ev)
    rc = lib.hsg_copy_nd(dev, arr.ctypes.data, len(arr), ws.data_ptr(), ws_bytes,
                         stage.ptr, stream_handle, 1 if sync else 0)
    _check(rc, "hsg_copy_nd")
    if sync:
        stage.release()
        return None
    return (stage, ws)


def tensor_copy_descriptor(batch: CopyBatch, src: torch.Tensor, dst: torch.Tensor) -> None:
    """Queue ``dst.copy_(src)`` (same shape; any strides; float casts allowed)."""
    if list(src.shape) != list(dst.shape):
        raise ValueError(f"shape mismatch {src.shape} vs {dst.shape}")
    es = src.element_size()
    batch.add(src.data_ptr(), src.dtype, src.stride(), dst.data_ptr(), dst.dtype,
              dst.stride(), list(src.shape), es if src.dtype == dst.dtype else es)


# ---- fp8 ----------------------------------------------------------------------

def fp8_quantize(dev: int, src: torch.Tensor, out: torch.Tensor, scales: torch.Tensor,
                 vpt: int, stream_handle: int) -> None:
    lib = require_gpu_lib()
    _check(lib.hsg_fp8_quantize(dev, src.data_ptr(), dtype_code(src.dtype), src.numel(),
                                out.data_ptr(), scales.data_ptr(), vpt, stream_handle),
           "hsg_fp8_quantize")


def fp8_dequantize(dev: int, q: torch.Tensor, scales: torch.Tensor, dst: torch.Tensor,
                   vpt: int, stream_handle: int) -> None:
    lib = require_gpu_lib()
    _check(lib.hsg_fp8_dequantize(dev, q.data_ptr(), scales.data_ptr(), q.numel(),
                                  dst.data_ptr(), dtype_code(dst.dtype), vpt, stream_handle),
           "hsg_fp8_dequantize")


def fp8_hadamard_quantize(dev: int, src: torch.Tensor, out: torch.Tensor, scales: torch.Tensor,
                          stream_handle: int) -> None:
    """MFMA Hadamard-32 rotation + blockwise e4m3 quantization (see hsgpu.hip)."""
    lib = require_gpu_lib()
    n = src.numel()
    n_pad = (n + 31) // 32 * 32
    assert out.numel() >= n_pad and scales.numel() >= (n_pad + 127) // 128
    assert src.is_contiguous() and dtype_code(src.dtype) in (10, 11, 12)
    _check(lib.hsg_fp8_hadamard_quantize(dev, src.data_ptr(), dtype_code(src.dtype), n,
                                         out.data_ptr(), scales.data_ptr(), stream_handle),
           "hsg_fp8_hadamard_quantize")


def fp8_hadamard_dequantize(dev: int, q: torch.Tensor, scales: torch.Tensor, dst: torch.Tensor,
                            stream_handle: int) -> None:
    lib = require_gpu_lib()
    n = dst.numel()
    assert q.numel() >= (n + 31) // 32 * 32 and dst.is_contiguous()
    _check(lib.hsg_fp8_hadamard_dequantize(dev, q.data_ptr(), scales.data_ptr(), n,
                                           dst.data_ptr(), dtype_code(dst.dtype), stream_handle),
           "hsg_fp8_hadamard_dequantize")


def mx8_quantize(dev: int, src: torch.Tensor, out: torch.Tensor, scales: torch.Tensor,
                 stream_handle: int) -> None:
    """MX fp8 (e4m3fn + E8M0 scale per 32 elements, hs_mx8_quant): ``out``
    gets round_up(n, 16) bytes (padding zeroed), ``scales`` ceil(n / 32)."""
    lib = require_gpu_lib()
    n = src.numel()
    assert src.is_contiguous() and dtype_code(src.dtype) in (10, 11, 12)
    assert out.numel() >= (n + 15) // 16 * 16 and scales.numel() >= (n + 31) // 32
    assert out.dtype == torch.uint8 and scales.dtype == torch.uint8
    _check(lib.hsg_mx8_quantize(dev, src.data_ptr(), dtype_code(src.dtype), n, out.data_ptr(),
                                scales.data_ptr(), stream_handle), "hsg_mx8_quantize")


def mx8_dequantize(dev: int, q: torch.Tensor, scales: torch.Tensor, dst: torch.Tensor,
                   stream_handle: int) -> None:
    lib = require_gpu_lib()
    n = dst.numel()
    assert dst.is_contiguous() and dtype_code(dst.dtype) in (10, 11, 12, 13)
    assert q.numel() >= n and scales.numel() >= (n + 31) // 32
    _check(lib.hsg_mx8_dequantize(dev, q.data_ptr(), scales.data_ptr(), n, dst.data_ptr(),
                                  dtype_code(dst.dtype), stream_handle), "hsg_mx8_dequantize")


class NativeDrain:
    """``hsg_drain_start`` / ``hsg_drain_wait`` (csrc/hsdrain.cpp): device
    byte ranges -> files, entirely in native threads (SDMA copies through
    pinned slots, pwrite, optional fdatasync and GPU hs64 hashing)."""

    def __init__(self, dev: int, blobs: Sequence[Tuple[int, int, str]], slot_bytes: int,
                 nslots: int, nwriters: int, fsync: bool, hash_blobs: bool,
                 max_hash_grid: int, nice: int = 0, direct: bool = False,
                 hash_high_priority: bool = True, parked_writers: int = 0) -> None:
        lib = require_gpu_lib()
        n = len(blobs)
        self.n = n
        self._srcs = (c_uint64 * max(n, 1))(*[b[0] for b in blobs])
        self._sizes = (c_uint64 * max(n, 1))(*[b[1] for b in blobs])
        self._paths = (c_char_p * max(n, 1))(*[os.fsencode(b[2]) for b in blobs])
        err = c_int(0)
        flags = self.flags(fsync, hash_blobs, direct, hash_high_priority, nice) | \
            (max(0, min(parked_writers, 255)) << 16)
        # boost() (any thread) and wait() (the drain's thread) both use the
        # handle: hsg_drain_wait frees the job, so a boost must never run
        # concurrently with or after it
        self._lock = threading.Lock()
        self._h = lib.hsg_drain_start(dev, n, self._srcs, self._sizes, self._paths,
                                      slot_bytes, nslots, nwriters, flags, max_hash_grid,
                                      ctypes.byref(err))
        if not self._h:
            raise HipError(f"hsg_drain_start failed ({err.value})")

    @staticmethod
    def flags(fsync: bool, hash_blobs: bool, direct: bool, hash_high_priority: bool,
              nice: int) -> int:
        return (1 if fsync else 0) | (2 if hash_blobs else 0) | (4 if direct else 0) | \
            (0 if hash_high_priority else 8) | (max(0, min(nice, 19)) << 8)

    def pending(self) -> int:
        return require_gpu_lib().hsg_drain_pending(self._h) if self._h else 0

    def boost(self) -> None:
        """Start the parked writers (call while the job runs)."""
        with self._lock:
            if self._h:
                require_gpu_lib().hsg_drain_boost(self._h)

    STATS = ("slot_wait", "hash_collect", "hash_launch", "sdma_submit", "sdma_wait", "pwrite",
             "close", "open", "wall")

    def wait(self) -> Tuple[List[int], int]:
        """Blocks (GIL released); returns (hs64 partial sums, bytes written).
        ``self.stats``: seconds per phase (summed over the threads in it)."""
        lib = require_gpu_lib()
        sums = (c_uint64 * max(self.n, 1))()
        written = c_uint64(0)
        msg = ctypes.create_string_buffer(256)
        st = (ctypes.c_double * len(self.STATS))()
        with self._lock:
            h, self._h = self._h, None
        r = lib.hsg_drain_wait(h, sums, ctypes.byref(written), msg, st)
        self.stats = {k: round(v, 4) for k, v in zip(self.STATS, st)}
        if r != 0:
            text = msg.value.decode(errors="replace")
            if r < 0 and -r in errno.errorcode:
                raise OSError(-r, text)
            raise HipError(f"native drain failed ({r}): {text}")
        return list(sums[: self.n]), int(written.value)


class NativeRestore:
    """``hsg_restore_start`` / ``hsg_restore_wait`` (csrc/hsrestore.cpp):
    file byte ranges (raw, or whole HSZ1 blobs) -> HBM destinations in
    native threads: pread into pinned slots, SDMA uploads into uncached
    blocks, GPU decode and ONE region-copy launch per item.

    ``items``: (path, file_lo, nbytes, codec (0 raw / 1 hsz1), logical,
    direct device address or 0, base_off, descriptor rows (packed
    COPY_DESC_DTYPE array whose ``src`` are offsets)).  ``producers``:
    stream handles the device work is ordered after.  ``hash_items``: per
    item, hs64 its stored bytes in HBM before they are decoded / copied
    (``restore(verify=True)``); ``wait`` then fills ``self.sums`` (partial
    sums, ``checksum.finish`` them with the item's byte count)."""

    STATS = ("read", "slot_wait", "budget_wait", "alloc", "submit", "upload_wait", "launch",
             "retire_wait", "first_upload", "upload_busy", "wall")

    def __init__(self, dev: int, items: Sequence[tuple], producers: Sequence[int],
                 slot_bytes: int, piece_bytes: int, nslots: int, nreaders: int,
                 budget: int, engine: int = -1, first_bytes: int = 16 << 20,
                 hash_items: Optional[Sequence[bool]] = None, hash_grid: int = 64) -> None:
        import torch

        lib = require_gpu_lib()
        n = len(items)
        self.n = n
        m = max(n, 1)
        self._paths = (c_char_p * m)(*[os.fsencode(it[0]) for it in items])
        self._lo = (c_uint64 * m)(*[it[1] for it in items])
        self._nb = (c_uint64 * m)(*[it[2] for it in items])
        self._codec = (c_int * m)(*[it[3] for it in items])
        self._logical = (c_uint64 * m)(*[it[4] for it in items])
        self._direct = (c_uint64 * m)(*[it[5] for it in items])
        self._base = (c_uint64 * m)(*[it[6] for it in items])
        offs, counts, tables = [], [], []
        k = 0
        for it in items:
            offs.append(k)
            counts.append(len(it[7]))
            k += len(it[7])
            if len(it[7]):
                tables.append(it[7])
        self._doff = (c_int64 * m)(*offs)
        self._dn = (c_int * m)(*counts)
        self._descs = np.concatenate(tables) if tables else np.zeros(1, dtype=COPY_DESC_DTYPE)
        self._prod = (c_uint64 * max(len(producers), 1))(*producers)
        # one host-mapped word per item: the decoder flags corrupt frames there
        # (pinned arrays are reused: a hipHostMalloc per restore costs ~1 ms)
        self.err_words = _take_err_words(m)
        self._hash = (c_int * m)(*[int(bool(h)) for h in hash_items]) if hash_items else None
        self.sums: List[int] = []
        err = c_int(0)
        self._h = lib.hsg_restore_start(
            dev, n, self._paths, self._lo, self._nb, self._codec, self._logical, self._direct,
            self._base, self._doff, self._dn, self._descs.ctypes.data, k, self._prod,
            len(producers), self.err_words.data_ptr(), slot_bytes, first_bytes, piece_bytes,
            nslots, nreaders, budget, engine, self._hash, hash_grid, ctypes.byref(err))
        if not self._h:
            raise HipError(f"hsg_restore_start failed ({err.value})")

    def wait(self) -> Tuple[int, Optional[int], str]:
        """Blocks (GIL released) until every item is in place.  Returns (0 or
        the first error (negative errno), the item it concerns, its text);
        ``self.stats``: seconds per phase; ``self.bytes_read``."""
        lib = require_gpu_lib()
        item = c_int(-1)
        msg = ctypes.create_string_buffer(320)
        st = (ctypes.c_double * len(self.STATS))()
        nread = c_uint64(0)
        sums = (c_uint64 * max(self.n, 1))() if self._hash is not None else None
        h, self._h = self._h, None
        r = lib.hsg_restore_wait(h, ctypes.byref(item), msg, st, ctypes.byref(nread), sums)
        if sums is not None:
            self.sums = list(sums[: self.n])
        self.stats = {k: round(v, 5) for k, v in zip(self.STATS, st)}
        self.bytes_read = int(nread.value)
        return int(r), (int(item.value) if item.value >= 0 else None), \
            msg.value.decode(errors="replace")

    def corrupt_items(self) -> List[int]:
        """Items whose frames the GPU decoder rejected (after ``wait``); gives
        the error words back."""
        w = self.err_words
        if w is None:
            return []
        bad = torch.nonzero(w[: self.n]).flatten().tolist() if self.n else []
        self.err_words = None
        _give_err_words(w)
        return bad


_err_words_lock = threading.Lock()
_err_words_free: List[torch.Tensor] = []


def _take_err_words(n: int) -> torch.Tensor:
    with _err_words_lock:
        for i, t in enumerate(_err_words_free):
            if t.numel() >= n:
                _err_words_free.pop(i)
                t.zero_()
                return t
    return torch.zeros(max(n, 1024), dtype=torch.int32, pin_memory=True)


def _give_err_words(t: torch.Tensor) -> None:
    with _err_words_lock:
        if len(_err_words_free) < 8:
            _err_words_free.append(t)


def poison_idle_pools(dev: int, byte: int) -> int:
    """Test hook: fill every idle restore device block on ``dev`` and every
    idle pinned host block with ``byte``; returns the blocks written."""
    r = int(require_gpu_lib().hsg_poison_idle_pools(dev, byte))
    _check(min(r, 0), "hsg_poison_idle_pools")
    return r


def restore_pool_bytes(dev: int = -1) -> Dict[str, int]:
    """Device bytes the native restore's pools hold (``dev`` -1: all)."""
    out = (c_uint64 * 4)()
    require_gpu_lib().hsg_restore_pool_bytes(dev, out)
    return {"upload_idle": int(out[0]), "upload_live": int(out[1]),
            "scratch_idle": int(out[2]), "scratch_live": int(out[3])}


def set_pool_trace(on: bool) -> None:
    """Log every engine pool allocation / free / restore upload to stderr
    (csrc/hshost.hip ``hsg_rt_trace``): a debugging aid for multi-process
    restores (scripts/probes/trim_probe_diag.py --trace)."""
    require_gpu_lib().hsg_rt_set_trace(1 if on else 0)


def uncached_pool_bytes() -> int:
    return int(require_gpu_lib().hsg_uncached_bytes())


def restore_trim(dev: int, keep_bytes: int) -> int:
    """Free idle restore device blocks beyond ``keep_bytes`` per pool."""
    return int(require_gpu_lib().hsg_restore_trim(dev, keep_bytes))


def restore_prewarm(dev: int, up_bytes: int, sc_bytes: int, slot_bytes: int, nslots: int,
                    table_bytes: int) -> int:
    """Fill the restore pools with what a job is about to take (blocking;
    ctypes drops the GIL): 0, or -1 when an allocation failed."""
    return int(require_gpu_lib().hsg_restore_prewarm(dev, up_bytes, sc_bytes, slot_bytes,
                                                     nslots, table_bytes))


def gate_supported(dev: int) -> bool:
    return bool(require_gpu_lib().hsg_gate_supported(dev))


def gate_arm(dev: int, stream_handle: int) -> int:
    """Make work queued on ``stream_handle`` from now on wait for
    ``gate_release(dev, value)``; returns that value (csrc/hsgpu.hip).  The
    caller MUST release it on every path."""
    v = ctypes.c_uint32(0)
    _check(require_gpu_lib().hsg_gate_arm(dev, stream_handle or None, ctypes.byref(v)),
           "hsg_gate_arm")
    return int(v.value)


def gate_release(dev: int, value: int) -> None:
    require_gpu_lib().hsg_gate_release(dev, value)


def gate_value(dev: int) -> int:
    return int(require_gpu_lib().hsg_gate_value(dev))


def managed_location(ptr: int, nbytes: int) -> Tuple[int, int]:
    """(preferred, last prefetch) location of a managed range: device index,
    -1 = host DRAM, -2 = never advised / prefetched."""
    lib = require_gpu_lib()
    a, b = c_int(-2), c_int(-2)
    lib.hsg_managed_location(ptr, nbytes, ctypes.byref(a), ctypes.byref(b))
    return int(a.value), int(b.value)


def managed_place(dev: int, ptr: int, nbytes: int, loc: int, stream_handle: int) -> None:
    """Advise ``loc`` (device index or -1 = host) as the preferred location of
    a managed range and prefetch it there on ``stream_handle``."""
    _check(require_gpu_lib().hsg_managed_place(dev, ptr, nbytes, loc, stream_handle or None),
           "hsg_managed_place")


def hip_runtime_path() -> Optional[str]:
    """Path of the libamdhip64 this process has loaded (torch's)."""
    try:
        with open("/proc/self/maps") as f:
            for line in f:
                parts = line.split()
                if len(parts) >= 6 and os.path.basename(parts[5]).startswith("libamdhip64.so"):
                    return parts[5]
    except OSError:
        pass
    return None


# ---- managed memory -------------------------------------------------------------

def is_managed_ptr(ptr: int) -> bool:
    lib = _load_hsgpu()
    if lib is None or not gpu_available():
        return False
    return bool(lib.hsg_is_managed(ptr))


# ---- HSZ1 lossless codec (format: ops/codec.py) ---------------------------------

def hsz_encode_cpu(src_addr: int, logical: int, w: int, frame_bytes: int, out_addr: int,
                   nthreads: int = 8) -> int:
    r = hsio().hsz_encode_cpu(src_addr, logical, w, frame_bytes, out_addr, nthreads)
    if r < 0:
        raise RuntimeError(f"hsz_encode_cpu failed ({r})")
    return int(r)


def hsz_decode_cpu(frames_addr: int, offsets_addr: int, first: int, count: int, logical: int,
                   w: int, frame_bytes: int, out_addr: int, nthreads: int = 8) -> None:
    r = hsio().hsz_decode_cpu(frames_addr, offsets_addr, first, count, logical, w, frame_bytes,
                              out_addr, nthreads)
    if r == -74:  # EBADMSG: a frame failed validation
        raise CorruptBlobError("corrupt HSZ1 blob: the host decoder rejected a frame")
    if r != 0:
        raise RuntimeError(f"hsz_decode_cpu failed ({r})")


def hsz_max_encoded_bytes(logical: int, frame_bytes: int) -> int:
    return int(hsio().hsz_max_encoded_bytes(logical, frame_bytes))


def _hsz_check(rc: int, what: str) -> None:
    if rc != 0:
        msg = require_gpu_lib().hsg_hsz_last_error().decode()
        raise HipError(f"{what} failed ({rc}): {msg}")


def hsz_meta_bytes(n_frames: int) -> int:
    return int(require_gpu_lib().hsg_hsz_meta_bytes(n_frames))


def hsz_encode_gpu(dev: int, src_addr: int, logical: int, w: int, frame_bytes: int,
                   out_addr: int, meta_addr: int, total_addr: int, stream_handle: int) -> None:
    """Enqueue the 3 encode kernels on ``stream_handle`` (no synchronisation)."""
    assert src_addr % 16 == 0 and out_addr % 16 == 0, "HSZ1 buffers must be 16-B aligned"
    _hsz_check(require_gpu_lib().hsg_hsz_encode(dev, src_addr, logical, w, frame_bytes,
                                                out_addr, meta_addr, total_addr, stream_handle),
               "hsg_hsz_encode")


def hsz_decode_gpu(dev: int, frames_addr: int, offsets_addr: int, first: int, count: int,
                   logical: int, w: int, frame_bytes: int, out_addr: int,
                   stream_handle: int, err_addr: int = 0) -> None:
    """Enqueue the decode of frames [first, first+count) on ``stream_handle``.
    ``err_addr``: a zeroed host-mapped pinned uint32 (``DecodeErrorWord``) the
    kernels set to 1 for a rejected frame; check it after the stream sync."""
    _hsz_check(require_gpu_lib().hsg_hsz_decode(dev, frames_addr, offsets_addr, first, count,
                                                logical, w, frame_bytes, out_addr,
                                                stream_handle, err_addr or None),
               "hsg_hsz_decode")


class CorruptBlobError(ValueError, RuntimeError):
    """An HSZ1 blob failed validation in the host or GPU decoder."""


class DecodeErrorWord:
    """Pinned host word the GPU decoders flag corrupt HSZ1 frames in (the
    device writes it through the host mapping; no extra copy or sync).

    Words come from pinned slabs of 1024 (one hipHostMalloc each, reused):
    a restore creates one per blob, and a pinned allocation per blob cost
    ~0.1 ms of HIP runtime time each (profiles/r4/restore_trace/)."""

    _lock = threading.Lock()
    _free: List[tuple] = []  # (slab tensor, index)
    _SLAB = 1024

    def __init__(self) -> None:
        import torch

        with DecodeErrorWord._lock:
            if not DecodeErrorWord._free:
                slab = torch.zeros(DecodeErrorWord._SLAB, dtype=torch.int32, pin_memory=True)
                DecodeErrorWord._free.extend((slab, i) for i in range(DecodeErrorWord._SLAB))
            self._slab, self._i = DecodeErrorWord._free.pop()
        self._slab[self._i] = 0
        self.addr = self._slab.data_ptr() + 4 * self._i
        self._held = True

    def check(self, what: str) -> None:
        """Call after the decode's stream was synchronised."""
        bad = int(self._slab[self._i]) != 0
        self.release()
        if bad:
            raise CorruptBlobError(
                f"corrupt HSZ1 blob: the GPU decoder rejected a frame of {what}")

    def release(self) -> None:
        if self._held:
            self._held = False
            with DecodeErrorWord._lock:
                DecodeErrorWord._free.append((self._slab, self._i))

    def __del__(self) -> None:  # pragma: no cover - GC path
        try:
            self.release()
        except Exception:
            pass
