"""Snapshot integrity check: re-read every blob and compare its hs64 checksum.

Not in the reference (its snapshots carry no checksums).  A take records the
hs64 of every blob it writes in ``.snapshot_checksums/<rank>`` (see
``ops/checksum.py``); ``verify_snapshot`` walks the committed manifest,
collects every blob location (tensors, chunks, shards, objects, slabs that
several entries share), reads each blob once and hashes it with the
multi-threaded C++ hasher, a bounded number of blobs in flight.

    python -m hipsnapshot verify /path/to/snapshot [--json]
"""

from __future__ import annotations

import asyncio
import json
import time
from dataclasses import asdict, dataclass, field
from typing import Any, Dict, List, Optional, Set

from .format.manifest import ChunkedTensorEntry, Entry, ObjectEntry, ShardedTensorEntry, TensorEntry
from .io_types import ReadIO, StoragePlugin
from .ops import checksum


@dataclass
class VerifyReport:
    path: str
    blobs: int = 0                  # blobs the manifest references
    checked: int = 0                # blobs read and hashed
    bytes: int = 0
    seconds: float = 0.0
    mismatched: List[str] = field(default_factory=list)
    missing_blobs: List[str] = field(default_factory=list)      # unreadable
    missing_checksums: List[str] = field(default_factory=list)  # no recorded hs64
    has_checksums: bool = True      # False: the snapshot was taken without them

    @property
    def ok(self) -> bool:
        return self.has_checksums and not (self.mismatched or self.missing_blobs
                                           or self.missing_checksums)

    def as_dict(self) -> Dict[str, Any]:
        d = asdict(self)
        d["ok"] = self.ok
        return d


def blob_locations(manifest: Dict[str, Entry]) -> Set[str]:
    """Every storage location the manifest's entries read from."""
    locs: Set[str] = set()
    for e in manifest.values():
        if isinstance(e, (TensorEntry, ObjectEntry)):
            locs.add(e.location)
        elif isinstance(e, ChunkedTensorEntry):
            locs.update(c.tensor.location for c in e.chunks)
        elif isinstance(e, ShardedTensorEntry):
            locs.update(s.tensor.location for s in e.shards)
    return locs


async def _read_checksums(storage: StoragePlugin, world_size: int) -> Optional[Dict[str, int]]:
    sums: Dict[str, int] = {}
    found = False
    for rank in range(world_size):
        rio = ReadIO(path=checksum.rank_file(rank))
        try:
            await storage.read(rio)
        except (FileNotFoundError, KeyError):
            continue
        doc = json.loads(bytes(rio.data()).decode("utf-8"))
        if doc.get("algo") != checksum.ALGO:
            raise ValueError(f"unknown checksum algorithm {doc.get('algo')!r}")
        found = True
        for p, h in doc["blobs"].items():
            sums[p] = int(h, 16)
    return sums if found else None


async def _verify(storage: StoragePlugin, manifest: Dict[str, Entry], world_size: int,
                  report: VerifyReport, concurrency: int, part: int = 0, parts: int = 1) -> None:
    sums = await _read_checksums(storage, world_size)
    locs = sorted(blob_locations(manifest))[part::parts]
    report.blobs = len(locs)
    if sums is None:
        report.has_checksums = False
        return
    sem = asyncio.Semaphore(concurrency)
    loop = asyncio.get_running_loop()

    async def one(loc: str) -> None:
        want = sums.get(loc)
        if want is None:
            report.missing_checksums.append(loc)
            return
        async with sem:
            rio = ReadIO(path=loc)
            try:
                await storage.read(rio)
            except (FileNotFoundError, KeyError):
                report.missing_blobs.append(loc)
                return
            buf = rio.data()
            got = await loop.run_in_executor(None, checksum.hs64_of, buf)
            report.checked += 1
            report.bytes += memoryview(buf).nbytes
            if got != want:
                report.mismatched.append(loc)

    await asyncio.gather(*(one(loc) for loc in locs))
    for lst in (report.mismatched, report.missing_blobs, report.missing_checksums):
        lst.sort()


def verify_snapshot(path: str, storage_options: Optional[Dict[str, Any]] = None,
                    concurrency: int = 4, distributed: bool = False, pg=None) -> VerifyReport:
    """Check every blob of the committed snapshot at ``path`` (see module doc).

    ``distributed``: a collective over ``pg`` (default: the world group);
    every rank checks 1/world_size of the blobs and all ranks return the
    merged report (one object all-gather)."""
    from .parallel.comm import Comm
    from .snapshot import Snapshot
    from .storage.registry import url_to_storage_plugin_in_event_loop

    t0 = time.monotonic()
    comm = Comm(pg) if distributed else None
    rank, ws = (comm.get_rank(), comm.get_world_size()) if comm is not None else (0, 1)
    report = VerifyReport(path=path)
    loop = asyncio.new_event_loop()
    storage = url_to_storage_plugin_in_event_loop(path, loop, storage_options)
    try:
        md = Snapshot._read_snapshot_metadata(storage, loop)
        loop.run_until_complete(_verify(storage, md.manifest, md.world_size, report,
                                        concurrency, rank, ws))
    finally:
        storage.sync_close(loop)
        loop.close()
    report.seconds = time.monotonic() - t0
    if comm is not None and not comm.solo():
        parts: List[Any] = [None] * ws
        comm.all_gather_object(parts, report)
        merged = VerifyReport(path=path, has_checksums=all(p.has_checksums for p in parts))
        for p in parts:
            merged.blobs += p.blobs
            merged.checked += p.checked
            merged.bytes += p.bytes
            merged.seconds = max(merged.seconds, p.seconds)
            merged.mismatched += p.mismatched
            merged.missing_blobs += p.missing_blobs
            merged.missing_checksums += p.missing_checksums
        for lst in (merged.mismatched, merged.missing_blobs, merged.missing_checksums):
            lst.sort()
        return merged
    return report
