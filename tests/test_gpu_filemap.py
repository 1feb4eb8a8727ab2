"""Blocking takes that rewrite existing blob files DMA straight into the
files' page-cache pages (csrc/hsfmap.cpp, ``FSStoragePlugin.mapped_dest``).

Each test compares the mapped take's files with a take of the same state
through the pinned + pwrite path (``knobs.TUNING.file_map`` off), and
restores them bitwise (with ``verify=True``: the blob checksums match)."""

import os

import pytest
import torch

from hipsnapshot import Snapshot, StateDict
from hipsnapshot.knobs import override_slab_size_threshold_bytes, override_tuning
from hipsnapshot.ops import native

pytestmark = pytest.mark.gpu


@pytest.fixture(autouse=True)
def _fresh_mappings():
    native.fmap_release(all_mappings=True)
    with override_tuning(file_map=True):  # off by default (knobs.TUNING.file_map)
        yield
    native.fmap_release(all_mappings=True)


def _state(gpu, seed):
    g = torch.Generator(device=gpu).manual_seed(seed)
    return StateDict(
        w=(torch.randn(2048, 2048, device=gpu, generator=g) * 0.02).bfloat16(),  # own blob
        v=torch.randn(3, 5000, device=gpu, generator=g),  # slab member
        s=torch.randn(70000, device=gpu, generator=g)[::2],  # non-contiguous
        h=torch.randn(1000, 33, generator=torch.Generator().manual_seed(seed)),  # host
        step=seed)


def _blobs(root):
    out = {}
    for d, _, files in os.walk(root):
        for f in files:
            if f.startswith(".snapshot_metadata"):
                continue
            p = os.path.join(d, f)
            with open(p, "rb") as fh:
                out[os.path.relpath(p, root)] = fh.read()
    return out


def _restored(path, like):
    out = StateDict({k: (torch.zeros_like(v) if isinstance(v, torch.Tensor) else 0)
                     for k, v in like.items()})
    Snapshot(path).restore({"sd": out}, verify=True)
    torch.cuda.synchronize()
    return out


def _assert_same(a, b):
    for k, v in a.items():
        if isinstance(v, torch.Tensor):
            assert torch.equal(v.cpu(), b[k].cpu()), k
        else:
            assert v == b[k], k


@pytest.mark.parametrize("comp", ["none", "hsz1"])
def test_rewrite_dmas_into_the_files_and_matches_the_pwrite_take(gpu, tmp_path, comp):
    p, ref = str(tmp_path / "s"), str(tmp_path / "ref")
    with override_slab_size_threshold_bytes(1 << 20):
        Snapshot.take(p, {"sd": _state(gpu, 1)}, compression=comp)  # new files: pwrite
        st0 = native.fmap_stats()
        # the same values twice (same HSZ1 sizes: mapped, then the mapping
        # reused), then new values (raw blobs keep their sizes)
        for seed in (1, 1, 2):
            sd = _state(gpu, seed)
            Snapshot.take(p, {"sd": sd}, compression=comp)
            with override_tuning(file_map=False):
                Snapshot.take(ref, {"sd": sd}, compression=comp)
            assert _blobs(p) == _blobs(ref)
            _assert_same(_restored(p, sd), sd)
    st = native.fmap_stats()
    assert st["maps"] > st0["maps"], (st0, st)  # the first rewrite mapped the files
    assert st["hits"] > st0["hits"], (st0, st)  # the second one reused the mappings


def test_replaced_or_resized_file_is_remapped(gpu, tmp_path):
    p = str(tmp_path / "s")
    with override_slab_size_threshold_bytes(1 << 20):
        Snapshot.take(p, {"sd": _state(gpu, 1)})
        Snapshot.take(p, {"sd": _state(gpu, 2)})
        entry = Snapshot(p).get_manifest()["0/sd/w"]
        blob = os.path.join(p, entry.location)
        # replaced by another file of the same size (new inode)
        with open(blob, "rb") as f:
            data = f.read()
        os.remove(blob)
        with open(blob, "wb") as f:
            f.write(bytes(len(data)))
        st0 = native.fmap_stats()
        sd = _state(gpu, 3)
        Snapshot.take(p, {"sd": sd})
        st = native.fmap_stats()
        assert st["maps"] > st0["maps"] and st["drops"] > st0["drops"], (st0, st)
        _assert_same(_restored(p, sd), sd)
        # rewritten in place by someone else (ctime changes): remapped again
        with open(blob, "r+b") as f:
            f.write(b"\0" * 4096)
        st0 = native.fmap_stats()
        sd = _state(gpu, 4)
        Snapshot.take(p, {"sd": sd})
        st = native.fmap_stats()
        assert st["maps"] > st0["maps"], (st0, st)
        _assert_same(_restored(p, sd), sd)
        # a different shape: other sizes, nothing mapped for those blobs
        sd = StateDict(w=torch.randn(100, device=gpu), v=torch.randn(3, device=gpu), step=5)
        Snapshot.take(p, {"sd": sd})
        _assert_same(_restored(p, sd), sd)


def test_fsync_and_direct_io_options(gpu, tmp_path):
    p = str(tmp_path / "s")
    with override_slab_size_threshold_bytes(1 << 20):
        for seed in (1, 2):
            sd = _state(gpu, seed)
            Snapshot.take(p, {"sd": sd}, storage_options={"fsync": True})
        _assert_same(_restored(p, sd), sd)
        st0 = native.fmap_stats()
        sd = _state(gpu, 3)
        Snapshot.take(p, {"sd": sd}, storage_options={"direct_io": True})
        st = native.fmap_stats()
        assert (st["hits"], st["maps"]) == (st0["hits"], st0["maps"])  # O_DIRECT: never mapped
        _assert_same(_restored(p, sd), sd)


def test_async_take_rewrite(gpu, tmp_path):
    p = str(tmp_path / "s")
    with override_slab_size_threshold_bytes(1 << 20):
        Snapshot.take(p, {"sd": _state(gpu, 1)})
        sd = _state(gpu, 2)
        expect = StateDict({k: (v.clone() if isinstance(v, torch.Tensor) else v)
                            for k, v in sd.items()})
        pending = Snapshot.async_take(p, {"sd": sd})
        for v in sd.values():
            if isinstance(v, torch.Tensor):
                v.add_(1)  # training goes on
        pending.wait()
        _assert_same(_restored(p, expect), expect)


def test_release_unregisters_everything(gpu, tmp_path):
    p = str(tmp_path / "s")
    with override_slab_size_threshold_bytes(1 << 20):
        Snapshot.take(p, {"sd": _state(gpu, 1)})
        Snapshot.take(p, {"sd": _state(gpu, 2)})
    assert native.fmap_stats()["mappings"] >= 1
    freed = native.fmap_release(all_mappings=True)
    assert freed > 0
    st = native.fmap_stats()
    assert st["mappings"] == 0 and st["bytes"] == 0
