"""Opt-in verification of restored blobs: ``Snapshot.restore(..., verify=True)``.

Every take records an hs64 checksum of every blob it writes
(``.snapshot_checksums/<rank>``, ops/checksum.py), but the reference has no
integrity check on restore at all (`/root/reference/torchsnapshot/
snapshot.py:650-729` reads and copies whatever the files hold), and
``Snapshot.verify()`` is an offline pass.  With ``verify=True`` the restore
itself checks each blob it reads against the recorded checksum and raises
``CorruptBlobError`` naming the blob:

* native jobs (reads landing in HBM, engine/native_restore.py) hash each
  whole blob's stored bytes in HBM right after its upload, on the stream that
  then decodes / copies it (``hsg_hash64_into`` in csrc/hsrestore.cpp): the
  hash reads HBM at a few TB/s beside a PCIe-bound upload;
* the Python pipeline hashes whole-blob host reads with the C++ hasher
  (``checksum.hs64_host``, multi-threaded) before they are consumed;
* blobs only PART of which a restore reads (byte-range reads of one rank's
  piece, budgeted tiles) are read once more and hashed at the end, in pieces
  that keep the read within the caller's memory budget (hs64 is a sum over
  8-byte words with their index: pieces at word boundaries add up).

A flipped byte in a raw blob -- or in an HSZ1 blob's low-byte plane, which
the HSZ1 frame checks cannot see -- then fails the restore instead of landing
in the model silently.
"""

from __future__ import annotations

import asyncio
import threading
from typing import Dict, Optional, Set

from ..io_types import ReadIO, StoragePlugin
from ..ops import checksum


def corrupt_blob_error_class():
    from ..ops import native

    return native.CorruptBlobError


class RestoreVerifier:
    """The take's checksums of one snapshot and what a restore checked."""

    def __init__(self, expected: Dict[str, int]) -> None:
        self.expected = expected
        self.verified: Set[str] = set()
        self.partial: Set[str] = set()
        self.bytes_hashed = 0
        self._lock = threading.Lock()

    @classmethod
    async def load(cls, storage: StoragePlugin, world_size: int) -> "RestoreVerifier":
        from ..verify import _read_checksums

        sums = await _read_checksums(storage, world_size)
        if sums is None:
            raise RuntimeError("restore(verify=True): this snapshot has no blob checksums "
                               "(it was taken with HIPSNAPSHOT_CHECKSUM=0)")
        return cls(sums)

    def _fail(self, path: str, what: str) -> None:
        raise corrupt_blob_error_class()(f"blob {path!r} {what}")

    def check_sum(self, path: str, h: int, nbytes: int) -> None:
        """A whole blob of ``nbytes`` bytes hashed to ``h``."""
        want = self.expected.get(path)
        if want is None:
            self._fail(path, "has no recorded checksum")
        if h != want:
            self._fail(path, f"does not match its checksum ({checksum.to_hex(h)} != "
                             f"{checksum.to_hex(want)})")
        with self._lock:
            self.verified.add(path)
            self.partial.discard(path)
            self.bytes_hashed += nbytes

    def check_host(self, path: str, addr: int, nbytes: int) -> None:
        self.check_sum(path, checksum.hs64_host(addr, nbytes), nbytes)

    def note_partial(self, path: str) -> None:
        with self._lock:
            if path not in self.verified:
                self.partial.add(path)

    async def finish(self, storage: StoragePlugin, memory_budget_bytes: Optional[int] = None,
                     concurrency: int = 4) -> None:
        """Read and hash every blob only part of which was read.  At most
        ``concurrency`` pieces of ``memory_budget_bytes / concurrency`` bytes
        (capped at 64 MiB, at least 1 MiB) are in memory at once; a plugin
        that cannot tell a blob's size is read whole."""
        with self._lock:
            todo = sorted(self.partial - self.verified)
        piece = PIECE_MAX
        if memory_budget_bytes:
            # a small budget: fewer pieces at once rather than tiny pieces
            concurrency = max(1, min(concurrency, int(memory_budget_bytes) // PIECE_MIN))
            piece = max(PIECE_MIN, min(PIECE_MAX, int(memory_budget_bytes) // concurrency))
        piece = piece // 8 * 8
        sem = asyncio.Semaphore(concurrency)
        loop = asyncio.get_running_loop()

        async def read_piece(path: str, lo: int, hi: Optional[int]) -> tuple:
            async with sem:
                rio = ReadIO(path=path, byte_range=None if hi is None else (lo, hi))
                await storage.read(rio)
                mv = memoryview(rio.data()).cast("B")
                s = await loop.run_in_executor(None, _partial, mv, lo // 8)
                return s, mv.nbytes

        async def one(path: str) -> None:
            size = await storage.size(path)
            if size is None:
                s, n = await read_piece(path, 0, None)
            else:
                parts = await asyncio.gather(*(read_piece(path, lo, min(size, lo + piece))
                                               for lo in range(0, max(size, 1), piece)))
                s, n = sum(p[0] for p in parts), sum(p[1] for p in parts)
            self.check_sum(path, checksum.finish(s, n), n)

        await asyncio.gather(*(one(p) for p in todo))


PIECE_MIN = 1 << 20
PIECE_MAX = 64 << 20


def _partial(mv: memoryview, first_word: int) -> int:
    """hs64's partial sum of ``mv`` as the bytes starting at word
    ``first_word`` of their blob (added over pieces, then ``finish``ed)."""
    from ..io_types import buffer_address
    from ..ops import native

    n = mv.nbytes
    if n == 0:
        return 0
    return int(native.hsio().hs64_partial(buffer_address(mv), n, first_word, 4))


def whole_read(rr, stored_size: Optional[int]) -> bool:
    """Does read request ``rr`` cover its whole blob of ``stored_size`` bytes?"""
    if rr.byte_range is None:
        return True
    lo, hi = rr.byte_range
    return lo == 0 and stored_size is not None and hi == stored_size
