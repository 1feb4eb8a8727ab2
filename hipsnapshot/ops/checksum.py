"""hs64: per-blob checksums of a snapshot (opt-out integrity layer).

Not in the reference.  Every blob a take writes gets an hs64 checksum
(definition in ``csrc/hschk.cpp``): GPU-staged blobs are hashed in HBM by the
``hs_hash64`` kernel right before their DMA to the host (the DMA is
PCIe-bound, the hash runs at HBM speed), host-staged blobs by the C++ hasher.
Each rank records its blobs in ``.snapshot_checksums/<rank>`` (JSON, next to
``.snapshot_metadata``; the reference's reader ignores it, so snapshots stay
reference-readable), and ``Snapshot.verify()`` / ``python -m hipsnapshot
verify PATH`` re-reads every blob and checks it.

``hs64_reference`` is a NumPy implementation of the definition for tests.
"""

from __future__ import annotations

from typing import Optional

import numpy as np

ALGO = "hs64"
CHECKSUM_DIR = ".snapshot_checksums"
_MASK = (1 << 64) - 1
_M1 = 0x9E3779B97F4A7C15


def mix64(x: int) -> int:
    x &= _MASK
    x ^= x >> 30
    x = (x * 0xBF58476D1CE4E5B9) & _MASK
    x ^= x >> 27
    x = (x * 0x94D049BB133111EB) & _MASK
    x ^= x >> 31
    return x


def finish(partial_sum: int, n_bytes: int) -> int:
    return mix64((partial_sum & _MASK) ^ n_bytes)


def hs64_reference(data) -> int:
    """Slow, obviously-correct NumPy version of the definition."""
    b = np.frombuffer(memoryview(data).cast("B"), dtype=np.uint8)
    n = b.size
    pad = (-n) % 8
    w = np.concatenate([b, np.zeros(pad, np.uint8)]).view("<u8").astype(np.uint64)
    idx = np.arange(1, w.size + 1, dtype=np.uint64)
    with np.errstate(over="ignore"):
        x = w ^ (idx * np.uint64(_M1))
        x ^= x >> np.uint64(30)
        x *= np.uint64(0xBF58476D1CE4E5B9)
        x ^= x >> np.uint64(27)
        x *= np.uint64(0x94D049BB133111EB)
        x ^= x >> np.uint64(31)
        s = int(x.sum(dtype=np.uint64))
    return finish(s, n)


def hs64_host(addr: int, nbytes: int, nthreads: int = 8) -> int:
    """hs64 of host bytes at ``addr`` (C++, multi-threaded for large blobs)."""
    from . import native

    lib = native.hsio()
    return int(lib.hs64_finish(lib.hs64_partial(addr if nbytes else None, nbytes, 0, nthreads),
                               nbytes))


def hs64_of(buf) -> int:
    from ..io_types import buffer_address

    mv = memoryview(buf).cast("B")
    return hs64_host(buffer_address(mv) if mv.nbytes else 0, mv.nbytes)


def to_hex(h: int) -> str:
    return f"{h & _MASK:016x}"


def device_hash_start(dev: int, slot: int, ptr: int, nbytes: int,
                      after_slot: int = -1, max_grid: Optional[int] = None) -> int:
    """Enqueue the hs64 partial sum of device bytes on stream (dev, slot),
    after the work queued on stream (dev, after_slot) if that is >= 0, on at
    most ``max_grid`` workgroups (default ``knobs.TUNING.hash_grid``; 0 = the
    whole chip).  Returns the handle ``device_hash_result`` takes."""
    import ctypes

    from .. import knobs
    from . import native

    if max_grid is None:
        max_grid = knobs.get_hash_grid()
    h = ctypes.c_int(-1)
    native._check(native.require_gpu_lib().hsg_hash64(dev, slot, after_slot, ptr, nbytes, 0,
                                                      max_grid, ctypes.byref(h)), "hsg_hash64")
    return h.value


def device_hash_result(dev: int, slot: int, handle: int, nbytes: int) -> int:
    """Wait for the hash ``handle`` started on stream (dev, slot) and finish it."""
    import ctypes

    from . import native

    out = ctypes.c_uint64(0)
    native._check(native.require_gpu_lib().hsg_hash64_result(dev, slot, handle,
                                                             ctypes.byref(out)),
                  "hsg_hash64_result")
    return finish(out.value, nbytes)


def rank_file(rank: int) -> str:
    return f"{CHECKSUM_DIR}/{rank}"


def parse_hex(s: Optional[str]) -> Optional[int]:
    return None if s is None else int(s, 16)
