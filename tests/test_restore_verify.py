"""restore(verify=True) / read_object(verify=True): every blob a restore reads
is checked against the take's hs64 checksums (engine/blob_verify.py)."""

import os

import pytest
import torch

from hipsnapshot import Snapshot, StateDict
from hipsnapshot.knobs import override_is_batching_disabled, override_slab_size_threshold_bytes
from hipsnapshot.ops.native import CorruptBlobError


def _flip(path: str, offset: int) -> None:
    with open(path, "r+b") as f:
        f.seek(offset)
        b = f.read(1)
        f.seek(offset)
        f.write(bytes([b[0] ^ 0x10]))


def _state(seed=0):
    g = torch.Generator().manual_seed(seed)
    return StateDict(w=torch.randn(300, 200, generator=g), b=torch.randn(77, generator=g),
                     step=3)


@pytest.mark.parametrize("batching", [True, False])
def test_flipped_raw_byte_fails_verified_restore_only(tmp_path, batching):
    p = str(tmp_path / "s")
    src = _state()
    with override_is_batching_disabled(not batching):
        Snapshot.take(p, {"sd": src})
        snap = Snapshot(p)
        entry = snap.get_manifest()["0/sd/w"]
        blob = os.path.join(p, entry.location)
        lo = entry.byte_range[0] if entry.byte_range else 0
        out = _state(1)
        snap.restore({"sd": out}, verify=True)  # intact: passes
        assert torch.equal(out["w"], src["w"])
        _flip(blob, lo + 1234)
        out = _state(1)
        Snapshot(p).restore({"sd": out})  # default path: unchanged (no check)
        assert not torch.equal(out["w"], src["w"])
        with pytest.raises(CorruptBlobError, match=entry.location):
            Snapshot(p).restore({"sd": _state(1)}, verify=True)


def test_partial_reads_verify_the_whole_blob(tmp_path):
    """read_object with a memory budget reads byte ranges of the blob: the
    blob is hashed in full at the end, so a flip outside the ranges read is
    still found."""
    p = str(tmp_path / "s")
    src = _state()
    with override_slab_size_threshold_bytes(1):
        Snapshot.take(p, {"sd": src})
    entry = Snapshot(p).get_manifest()["0/sd/w"]
    out = torch.zeros_like(src["w"])
    Snapshot(p).read_object("0/sd/w", obj_out=out, memory_budget_bytes=4096, verify=True)
    assert torch.equal(out, src["w"])
    _flip(os.path.join(p, entry.location), 17)
    with pytest.raises(CorruptBlobError):
        Snapshot(p).read_object("0/sd/w", obj_out=torch.zeros_like(src["w"]),
                                memory_budget_bytes=4096, verify=True)


def test_flipped_low_byte_plane_of_hsz1_blob(tmp_path):
    """HSZ1 frame checks validate the container, not the stored low bytes: a
    flip there restores silently unless the checksum is checked."""
    from hipsnapshot.ops import codec

    p = str(tmp_path / "s")
    g = torch.Generator().manual_seed(4)
    w = (torch.randn(700, 1000, generator=g) * 0.02).to(torch.bfloat16)
    with override_slab_size_threshold_bytes(1):
        Snapshot.take(p, {"sd": StateDict(w=w)}, compression="hsz1+host")
    entry = Snapshot(p).get_manifest()["0/sd/w"]
    assert entry.codec
    blob = os.path.join(p, entry.location)
    from hipsnapshot.utils.test_utils import low_byte_offset

    with open(blob, "rb") as f:
        _flip(blob, low_byte_offset(f.read()))
    out = torch.zeros_like(w)
    Snapshot(p).restore({"sd": StateDict(w=out)})
    assert not torch.equal(out, w)  # decodes "fine", wrong values
    with pytest.raises(CorruptBlobError, match=entry.location):
        Snapshot(p).restore({"sd": StateDict(w=torch.zeros_like(w))}, verify=True)


def test_verify_needs_checksums(tmp_path, monkeypatch):
    p = str(tmp_path / "s")
    monkeypatch.setenv("HIPSNAPSHOT_CHECKSUM", "0")
    Snapshot.take(p, {"sd": _state()})
    monkeypatch.delenv("HIPSNAPSHOT_CHECKSUM")
    with pytest.raises(RuntimeError, match="no blob checksums"):
        Snapshot(p).restore({"sd": _state(1)}, verify=True)


def test_read_object_of_a_sharded_entry_without_obj_out(tmp_path):
    """A sharded entry comes back whole (global shape, host tensor) when no
    tensor obj_out is given."""
    import torch.distributed as dist
    from torch.distributed.device_mesh import init_device_mesh
    from torch.distributed.tensor import Shard, distribute_tensor

    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ.setdefault("MASTER_PORT", "29591")
    own = not dist.is_initialized()
    if own:
        dist.init_process_group("gloo", rank=0, world_size=1)
    try:
        mesh = init_device_mesh("cpu", (1,))
        full = torch.randn(37, 11)
        dt = distribute_tensor(full, mesh, [Shard(0)])
        p = str(tmp_path / "s")
        Snapshot.take(p, {"sd": StateDict(w=dt)})
        got = Snapshot(p).read_object("0/sd/w", verify=True)
        assert isinstance(got, torch.Tensor) and torch.equal(got, full)
        got = Snapshot(p).read_object("0/sd/w", memory_budget_bytes=512)
        assert torch.equal(got, full)
    finally:
        if own:
            dist.destroy_process_group()


def test_partial_blob_verification_stays_within_the_budget(tmp_path):
    """the end-of-read check of partially read blobs read each blob
    whole, ignoring the caller's budget.  It now reads budget-sized pieces
    and adds their hs64 partial sums: a 5 MiB blob checked under a 2 MiB
    budget never has more than the budget in flight, and the sum of the
    pieces equals the whole-blob hash (and still finds a flipped byte)."""
    import asyncio

    from hipsnapshot.engine.blob_verify import RestoreVerifier
    from hipsnapshot.ops import checksum
    from hipsnapshot.storage.fs import FSStoragePlugin

    data = torch.randint(0, 255, (5 << 20,), dtype=torch.uint8).numpy().tobytes() + b"xyz"
    (tmp_path / "blob").write_bytes(data)
    storage = FSStoragePlugin(str(tmp_path))
    reads, live, peak = [], [0], [0]
    orig = storage.read

    async def spy(rio):
        lo, hi = rio.byte_range if rio.byte_range else (0, len(data))
        reads.append(hi - lo)
        live[0] += hi - lo
        peak[0] = max(peak[0], live[0])
        await orig(rio)
        await asyncio.sleep(0.01)  # the piece stays in memory while it is hashed
        live[0] -= hi - lo

    storage.read = spy
    v = RestoreVerifier({"blob": checksum.hs64_of(data)})
    v.note_partial("blob")
    loop = asyncio.new_event_loop()
    try:
        loop.run_until_complete(v.finish(storage, memory_budget_bytes=2 << 20))
        assert "blob" in v.verified
        assert sum(reads) == len(data) and len(reads) > 1
        assert peak[0] <= 2 << 20, peak
        bad = bytearray(data)
        bad[(3 << 20) + 5] ^= 1
        (tmp_path / "blob").write_bytes(bytes(bad))
        v2 = RestoreVerifier({"blob": checksum.hs64_of(data)})
        v2.note_partial("blob")
        with pytest.raises(CorruptBlobError):
            loop.run_until_complete(v2.finish(storage, memory_budget_bytes=2 << 20))
        loop.run_until_complete(storage.close())
    finally:
        loop.close()
