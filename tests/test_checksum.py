"""hs64 blob checksums: the C++ hasher against the NumPy definition, takes
recording them, ``Snapshot.verify`` / ``python -m hipsnapshot verify``
catching corrupted and missing blobs."""

import json
import os

import numpy as np
import pytest
import torch

from hipsnapshot import Snapshot, StateDict
from hipsnapshot.__main__ import main as cli
from hipsnapshot.ops import checksum, native


@pytest.mark.parametrize("n", [0, 1, 7, 8, 9, 63, 64, 1000, 1 << 20, (40 << 20) + 5])
def test_host_hash_matches_definition(n):
    b = np.random.default_rng(n).integers(0, 256, n, dtype=np.uint8).tobytes()
    assert checksum.hs64_of(b) == checksum.hs64_reference(b)


@pytest.mark.parametrize("off", [1, 3, 5])
def test_host_hash_unaligned_start(off):
    b = np.random.default_rng(off).integers(0, 256, 4096 + off, dtype=np.uint8)
    v = memoryview(b)[off:]
    assert checksum.hs64_of(v) == checksum.hs64_reference(bytes(v))


def test_partial_sums_compose_over_aligned_ranges():
    b = np.random.default_rng(0).integers(0, 256, 1 << 16, dtype=np.uint8)
    lib = native.hsio()
    addr = b.ctypes.data
    whole = lib.hs64_partial(addr, b.size, 0, 1)
    cut = 8 * 1000
    parts = (lib.hs64_partial(addr, cut, 0, 1)
             + lib.hs64_partial(addr + cut, b.size - cut, cut // 8, 1)) & ((1 << 64) - 1)
    assert parts == whole


def test_hash_sensitive_to_position_and_length():
    a = bytes(range(16))
    assert checksum.hs64_of(a) != checksum.hs64_of(a[8:] + a[:8])
    assert checksum.hs64_of(b"\0" * 8) != checksum.hs64_of(b"\0" * 9)
    assert checksum.hs64_of(b"") != checksum.hs64_of(b"\0")


def _state():
    torch.manual_seed(0)
    return {"m": StateDict(w=torch.randn(257, 33), b=torch.randn(5, dtype=torch.bfloat16),
                           step=7, name="x", big=torch.randn(300_000))}


def _blob_files(root):
    out = []
    for d, _, fs in os.walk(root):
        for f in fs:
            p = os.path.join(d, f)
            rel = os.path.relpath(p, root)
            if not rel.startswith(".snapshot"):
                out.append(p)
    return sorted(out)


def test_take_records_checksums_and_verify_passes(tmp_path):
    p = str(tmp_path / "s")
    snap = Snapshot.take(p, _state())
    doc = json.load(open(os.path.join(p, checksum.CHECKSUM_DIR, "0")))
    assert doc["algo"] == "hs64" and doc["world_size"] == 1
    # every blob file is recorded, with the hash of its bytes
    for f in _blob_files(p):
        rel = os.path.relpath(f, p)
        assert int(doc["blobs"][rel], 16) == checksum.hs64_of(open(f, "rb").read())
    rep = snap.verify()
    assert rep.ok and rep.checked == rep.blobs > 0, rep
    assert cli(["verify", p]) == 0


def test_verify_detects_a_flipped_byte_and_a_missing_blob(tmp_path):
    p = str(tmp_path / "s")
    snap = Snapshot.take(p, _state())
    files = _blob_files(p)
    victim = max(files, key=os.path.getsize)
    with open(victim, "r+b") as f:
        f.seek(os.path.getsize(victim) // 2)
        c = f.read(1)
        f.seek(-1, 1)
        f.write(bytes([c[0] ^ 0x10]))
    rep = snap.verify()
    assert not rep.ok and rep.mismatched == [os.path.relpath(victim, p)]
    assert cli(["verify", p, "--json"]) == 1
    os.remove(victim)
    rep = snap.verify()
    assert rep.missing_blobs == [os.path.relpath(victim, p)] and not rep.ok


def test_checksums_off_and_stale_files_removed(tmp_path, monkeypatch):
    p = str(tmp_path / "s")
    Snapshot.take(p, _state())
    assert os.path.isdir(os.path.join(p, checksum.CHECKSUM_DIR))
    monkeypatch.setenv("HIPSNAPSHOT_CHECKSUM", "0")
    snap = Snapshot.take(p, _state())  # retake: the old checksums must not survive
    assert not os.path.exists(os.path.join(p, checksum.CHECKSUM_DIR))
    rep = snap.verify()
    assert not rep.has_checksums and not rep.ok


@pytest.mark.parametrize("compression", [None, "hsz1"])
def test_async_take_and_compressed_blobs_verify(tmp_path, compression):
    p = str(tmp_path / "a")
    st = _state()
    snap = Snapshot.async_take(p, st, compression=compression).wait()
    assert snap.verify().ok
    out = {"m": StateDict(w=torch.zeros(257, 33), b=torch.zeros(5, dtype=torch.bfloat16),
                          step=0, name="", big=torch.zeros(300_000))}
    snap.restore(out)
    assert torch.equal(out["m"]["big"], st["m"]["big"])


def test_memory_plugin_verify():
    p = "memory://cksum/snap"
    snap = Snapshot.take(p, _state())
    rep = snap.verify()
    assert rep.ok and rep.checked > 0
