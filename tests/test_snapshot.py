"""Single-process end-to-end take/restore (reference: tests/test_snapshot.py,
test_rng_state.py, test_read_object.py, test_fs_storage_plugin.py)."""

import json
import os
from collections import OrderedDict

import pytest
import torch

from hipsnapshot import RNGState, Snapshot, StateDict
from hipsnapshot.knobs import override_max_chunk_size_bytes, override_slab_size_threshold_bytes
from hipsnapshot.utils.test_utils import assert_state_dict_eq, rand_tensor


def _model():
    return torch.nn.Sequential(torch.nn.Linear(32, 64), torch.nn.ReLU(), torch.nn.Linear(64, 8))


def test_state_dict_odd_keys(tmp_path, toggle_batching):
    sd = StateDict({"a/b": torch.randn(3), "%2F": 1, "": {"": [torch.ones(2)]}, 7: "seven",
                    "nested": OrderedDict(x=1.5, y=[b"raw", True, None])})
    Snapshot.take(str(tmp_path / "s"), {"sd": sd})
    out = StateDict()
    Snapshot(str(tmp_path / "s")).restore({"sd": out})
    assert_state_dict_eq(dict(out), dict(sd))


@pytest.mark.parametrize("opt_cls", [torch.optim.Adagrad, torch.optim.Adam, torch.optim.SGD])
def test_model_and_optimizer(tmp_path, toggle_batching, opt_cls):
    torch.manual_seed(0)
    m = _model()
    kw = {"momentum": 0.9} if opt_cls is torch.optim.SGD else {}
    o = opt_cls(m.parameters(), lr=0.1, **kw)
    for _ in range(2):
        m(torch.randn(4, 32)).sum().backward()
        o.step()
    Snapshot.take(str(tmp_path / "s"), {"m": m, "o": o})
    m2 = _model()
    o2 = opt_cls(m2.parameters(), lr=0.5, **kw)
    m2(torch.randn(4, 32)).sum().backward()
    o2.step()
    Snapshot(str(tmp_path / "s")).restore({"m": m2, "o": o2})
    assert_state_dict_eq(m.state_dict(), m2.state_dict())
    assert_state_dict_eq(o.state_dict(), o2.state_dict())


def test_differing_structure_restore(tmp_path):
    """Restore only fills what the target asks for, adds what the snapshot has."""
    Snapshot.take(str(tmp_path / "s"), {"sd": StateDict(a=torch.ones(2), b=2)})
    out = StateDict(c=3)
    Snapshot(str(tmp_path / "s")).restore({"sd": out})
    assert set(out.keys()) == {"a", "b", "c"}


def test_inplace_restore_keeps_storage(tmp_path):
    t = torch.randn(64, 64)
    Snapshot.take(str(tmp_path / "s"), {"sd": StateDict(t=t)})
    target = torch.zeros(64, 64)
    ptr = target.data_ptr()
    sd = StateDict(t=target)
    Snapshot(str(tmp_path / "s")).restore({"sd": sd})
    assert sd["t"].data_ptr() == ptr and torch.equal(target, t)


def test_chunked_and_slabbed(tmp_path, toggle_batching):
    ts = {f"t{i}": rand_tensor([50 + i, 17], dt) for i, dt in
          enumerate([torch.float32, torch.bfloat16, torch.int64, torch.bool, torch.float16])}
    with override_max_chunk_size_bytes(1000), override_slab_size_threshold_bytes(3000):
        Snapshot.take(str(tmp_path / "s"), {"sd": StateDict(ts)})
    man = Snapshot(str(tmp_path / "s")).get_manifest()
    assert man["0/sd/t0"].type == "ChunkedTensor"
    out = StateDict({k: torch.zeros_like(v) for k, v in ts.items()})
    Snapshot(str(tmp_path / "s")).restore({"sd": out})
    assert_state_dict_eq(dict(out), ts)


def test_rng_state_invariant(tmp_path):
    torch.manual_seed(42)

    class Mutator:
        def state_dict(self):
            torch.rand(10)  # side effect on the RNG
            return {"x": 1}

        def load_state_dict(self, sd):
            torch.rand(10)

    app = {"rng": RNGState(), "mut": Mutator()}
    Snapshot.take(str(tmp_path / "s"), app)
    after_take = torch.rand(5)
    torch.rand(100)
    Snapshot(str(tmp_path / "s")).restore(app)
    assert torch.equal(torch.rand(5), after_take)


def test_multiple_rng_states_rejected(tmp_path):
    with pytest.raises(RuntimeError):
        Snapshot.take(str(tmp_path / "s"), {"a": RNGState(), "b": RNGState()})


def test_non_stateful_rejected(tmp_path):
    with pytest.raises(TypeError):
        Snapshot.take(str(tmp_path / "s"), {"a": {"not": "stateful"}})


def test_read_object(tmp_path):
    sd = StateDict(t=torch.randn(100, 10), p=3.5, s="hi", big=torch.arange(10000))
    Snapshot.take(str(tmp_path / "s"), {"sd": sd})
    snap = Snapshot(str(tmp_path / "s"))
    assert snap.read_object("0/sd/p") == 3.5
    assert snap.read_object("0/sd/s") == "hi"
    assert torch.equal(snap.read_object("0/sd/t"), sd["t"])
    out = torch.zeros(100, 10)
    assert snap.read_object("0/sd/t", obj_out=out) is out and torch.equal(out, sd["t"])
    assert torch.equal(snap.read_object("0/sd/big", memory_budget_bytes=1000), sd["big"])
    with pytest.raises(RuntimeError):
        snap.read_object("0/sd/missing")


def test_object_entries_weights_only_and_trust(tmp_path):
    class Custom:
        def __init__(self):
            self.v = 5

    import builtins

    builtins._HsTestCustom = Custom  # make it picklable by reference
    Custom.__module__, Custom.__qualname__ = "builtins", "_HsTestCustom"
    try:
        sd = StateDict(obj={1, 2, 3}, custom=Custom())
        Snapshot.take(str(tmp_path / "s"), {"sd": sd})
        snap = Snapshot(str(tmp_path / "s"))
        # sets are allow-listed in weights_only loading
        assert snap.read_object("0/sd/obj") == {1, 2, 3}
        with pytest.raises(Exception):
            snap.read_object("0/sd/custom")
        trusted = Snapshot(str(tmp_path / "s"), trust_objects=True)
        assert trusted.read_object("0/sd/custom").v == 5
    finally:
        del builtins._HsTestCustom


def test_metadata_format_on_disk(tmp_path):
    Snapshot.take(str(tmp_path / "s"), {"sd": StateDict(a=torch.ones(3), b=1)})
    md = json.loads((tmp_path / "s" / ".snapshot_metadata").read_text())
    assert md["version"] == "0.1.0" and md["world_size"] == 1
    assert md["manifest"]["0/sd"] == {"type": "dict", "keys": ["a", "b"]}
    assert md["manifest"]["0/sd/b"]["type"] == "int"
    assert md["manifest"]["0/sd/a"]["serializer"] == "buffer_protocol"


def test_retake_same_path_overwrites(tmp_path):
    p = str(tmp_path / "s")
    Snapshot.take(p, {"sd": StateDict(a=torch.ones(1000), b=torch.zeros(10))})
    Snapshot.take(p, {"sd": StateDict(a=torch.full((10,), 2.0))})
    out = StateDict()
    Snapshot(p).restore({"sd": out})
    assert torch.equal(out["a"], torch.full((10,), 2.0)) and "b" not in out
    # deterministic slab names: no stale blobs accumulate
    assert len(os.listdir(tmp_path / "s" / "batched")) == 1


def test_memory_storage_plugin():
    from hipsnapshot.storage.memory import clear_memory_store

    sd = StateDict(a=torch.randn(10), b="x")
    Snapshot.take("memory://bucket/snap", {"sd": sd})
    out = StateDict()
    Snapshot("memory://bucket/snap").restore({"sd": out})
    assert torch.equal(out["a"], sd["a"]) and out["b"] == "x"
    clear_memory_store("bucket")


def test_quantize_fp8_cpu(tmp_path):
    w = torch.randn(300, 70)
    Snapshot.take(str(tmp_path / "s"), {"sd": StateDict(w=w, i=torch.arange(5))},
                  quantize=["sd/w"])
    man = Snapshot(str(tmp_path / "s")).get_manifest()
    assert man["0/sd/w"].serializer == "hipsnapshot_fp8_block"
    assert man["0/sd/w"].quant["block"] == 32  # MX layout (E8M0 scale per 32)
    assert man["0/sd/w"].quant["format"] == "fp8_e4m3fn_mx"
    out = StateDict(w=torch.zeros(300, 70), i=torch.zeros(5, dtype=torch.int64))
    Snapshot(str(tmp_path / "s")).restore({"sd": out})
    rel = (out["w"] - w).abs().max() / w.abs().max()
    assert rel < 0.08 and torch.equal(out["i"], torch.arange(5))


def _cyclic_garbage(fn):
    import gc

    gc.collect()
    gc.set_debug(gc.DEBUG_SAVEALL)
    try:
        fn()
        gc.collect()
        found = list(gc.garbage)
    finally:
        gc.garbage.clear()
        gc.set_debug(0)
    return found


def test_take_leaves_no_reference_cycles(tmp_path):
    """A take to a fresh path hits the expected FileNotFoundError when it
    removes an older commit; that error must not leave a cycle (task <->
    traceback frame) pinning the take's plan until a full GC."""
    from hipsnapshot.io_types import WriteReq

    st = StateDict({f"w{i}": torch.randn(32, 8) for i in range(20)})
    for name, fn in [
        ("take", lambda: Snapshot.take(str(tmp_path / "s"), {"m": st})),
        ("async_take", lambda: Snapshot.async_take(str(tmp_path / "a"), {"m": st}).wait()),
        ("restore", lambda: Snapshot(str(tmp_path / "s")).restore({"m": st})),
    ]:
        found = _cyclic_garbage(fn)
        assert not [o for o in found if isinstance(o, (WriteReq, BaseException))], name


def test_run_sync_reraises_without_cycle():
    import asyncio

    from hipsnapshot.io_types import run_sync

    async def boom():
        raise FileNotFoundError("x")

    async def ok():
        return 7

    loop = asyncio.new_event_loop()
    try:
        assert run_sync(loop, ok()) == 7

        def fail():
            with pytest.raises(FileNotFoundError):
                run_sync(loop, boom())

        assert not [o for o in _cyclic_garbage(fail) if isinstance(o, BaseException)]
    finally:
        loop.close()


def test_in_place_module_restore_skips_self_copy(tmp_path, monkeypatch):
    """Every leaf read into the module's own tensor: load_state_dict would
    copy each tensor onto itself, so it is skipped; a module that customises
    loading (its own _load_from_state_dict, or a load hook) still gets it."""
    import torch.nn as nn

    calls = []
    orig = nn.Module.load_state_dict

    def spy(self, *a, **k):
        calls.append(type(self).__name__)
        return orig(self, *a, **k)

    monkeypatch.setattr(nn.Module, "load_state_dict", spy)
    import hipsnapshot.snapshot as snap_mod

    monkeypatch.setattr(snap_mod, "_module_plain_load", snap_mod.weakref.WeakKeyDictionary())
    torch.manual_seed(0)
    m = nn.Sequential(nn.Linear(8, 4), nn.ReLU(), nn.Linear(4, 2))
    ref = {k: v.clone() for k, v in m.state_dict().items()}
    Snapshot.take(str(tmp_path / "a"), {"m": m})
    for p in m.parameters():
        p.data.zero_()
    Snapshot(str(tmp_path / "a")).restore({"m": m})
    assert calls == []
    for k, v in m.state_dict().items():
        assert torch.equal(v, ref[k]), k

    class Custom(nn.Linear):
        def _load_from_state_dict(self, *a, **k):
            calls.append("custom")
            return super()._load_from_state_dict(*a, **k)

    c = Custom(8, 4)
    cref = {k: v.clone() for k, v in c.state_dict().items()}
    Snapshot.take(str(tmp_path / "b"), {"c": c})
    for p in c.parameters():
        p.data.zero_()
    Snapshot(str(tmp_path / "b")).restore({"c": c})
    assert calls == ["Custom", "custom"]
    for k, v in c.state_dict().items():
        assert torch.equal(v, cref[k]), k


def test_local_metadata_cache_follows_the_file(tmp_path):
    """Two Snapshot objects of one committed local snapshot share the parsed
    metadata; a new take into the path replaces the file and is re-read."""
    import hipsnapshot.snapshot as snap_mod

    p = str(tmp_path / "s")
    Snapshot.take(p, {"sd": StateDict(a=torch.ones(3), n=1)})
    m1 = Snapshot(p).metadata
    assert Snapshot(p).metadata is m1
    Snapshot.take(p, {"sd": StateDict(a=torch.ones(3), n=2, extra=torch.zeros(5))})
    m2 = Snapshot(p).metadata
    assert m2 is not m1 and "0/sd/extra" in m2.manifest
    out = StateDict(a=torch.zeros(3), n=0, extra=torch.ones(5))
    Snapshot(p).restore({"sd": out})
    assert out["n"] == 2 and torch.equal(out["extra"], torch.zeros(5))
    assert len(snap_mod._metadata_cache) <= 4


@pytest.mark.parametrize("url", ["fs", "memory"])
def test_failed_coalesce_keeps_the_committed_snapshot(tmp_path, monkeypatch, url):
    """rank 0 takes the old commit away before the coalesce
    gather (no rank may write a blob while it names them), but a take that
    fails IN that gather has written nothing: the old commit comes back
    (renamed back on FS, re-written from the kept bytes elsewhere)."""
    import uuid

    from hipsnapshot import Snapshot, StateDict

    path = str(tmp_path / "s") if url == "fs" else f"memory://b{uuid.uuid4().hex[:8]}/s"
    sd = StateDict(w=torch.arange(10.0))
    Snapshot.take(path, {"sd": sd})

    def boom(*a, **k):
        raise RuntimeError("coalesce failed")

    monkeypatch.setattr(Snapshot, "_coalesce", classmethod(boom))
    with pytest.raises(RuntimeError, match="coalesce failed"):
        Snapshot.take(path, {"sd": StateDict(w=torch.zeros(10))})
    monkeypatch.undo()
    out = StateDict(w=torch.zeros(10))
    Snapshot(path).restore({"sd": out})
    assert torch.equal(out["w"], torch.arange(10.0))
    if url == "fs":
        assert not [f for f in os.listdir(path) if ".stash." in f]
    # a take that succeeds leaves no stash behind either
    Snapshot.take(path, {"sd": StateDict(w=torch.ones(10))})
    if url == "fs":
        assert not [f for f in os.listdir(path) if ".stash." in f]
    Snapshot(path).restore({"sd": out})
    assert torch.equal(out["w"], torch.ones(10))
