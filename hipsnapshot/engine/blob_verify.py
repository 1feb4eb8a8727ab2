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
  piece, budgeted tiles) are read once more in full and hashed at the end.

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

    async def finish(self, storage: StoragePlugin, concurrency: int = 4) -> None:
        """Read and hash, in full, every blob only part of which was read."""
        with self._lock:
            todo = sorted(self.partial - self.verified)
        sem = asyncio.Semaphore(concurrency)
        loop = asyncio.get_running_loop()

        async def one(path: str) -> None:
            async with sem:
                rio = ReadIO(path=path)
                await storage.read(rio)
                mv = memoryview(rio.data()).cast("B")
                h = await loop.run_in_executor(None, checksum.hs64_of, mv)
                self.check_sum(path, h, mv.nbytes)

        await asyncio.gather(*(one(p) for p in todo))


def whole_read(rr, stored_size: Optional[int]) -> bool:
    """Does read request ``rr`` cover its whole blob of ``stored_size`` bytes?"""
    if rr.byte_range is None:
        return True
    lo, hi = rr.byte_range
    return lo == 0 and stored_size is not None and hi == stored_size
