"""Take-plan reuse (hipsnapshot/engine/plan_cache.py).

On the GPU only device-resident leaves are cached; these CPU tests mark a
chosen set of host tensors "resident" so the cache logic (signatures, reuse,
stager reset, per-take leaves, busy plans, invalidation) runs here too.  The
GPU path is covered in tests/test_gpu.py."""

import asyncio
import gc

import pytest
import torch

from hipsnapshot import Snapshot, StateDict
from hipsnapshot.engine import plan_cache
from hipsnapshot.knobs import override_knob, override_max_chunk_size_bytes
from hipsnapshot.utils.test_utils import assert_state_dict_eq


@pytest.fixture
def resident(monkeypatch):
    """Tensors whose id is in the returned set count as device-resident."""
    ids = set()
    monkeypatch.setattr(plan_cache, "is_resident",
                        lambda obj: isinstance(obj, torch.Tensor) and id(obj) in ids)
    plan_cache.clear()
    for k in plan_cache.stats:
        plan_cache.stats[k] = 0
    yield ids
    plan_cache.clear()


def _state(ids, n=12, host=False):
    g = {f"g{i}": torch.randn(1000 + 37 * i) for i in range(n)}      # "device" (cached)
    g["big"] = torch.randn(3000, 100)                                  # chunked below
    ids.update(id(v) for v in g.values())
    # host tensors are planned per take; here they would share host slabs
    # with the "device" ones (on a GPU the two never share a slab)
    c = {f"c{i}": torch.randn(500 + i) for i in range(4)} if host else {}
    return StateDict(step=0, meta={"lr": 0.1, "tags": ["a"]}, **g, **c)


def _snap(sd):
    return {k: (v.clone() if isinstance(v, torch.Tensor) else
                {kk: (list(vv) if isinstance(vv, list) else vv) for kk, vv in v.items()}
                if isinstance(v, dict) else v) for k, v in sd.items()}


def _restore(path, like):
    out = StateDict(**{k: (torch.zeros_like(v) if isinstance(v, torch.Tensor) else None)
                       for k, v in like.items()})
    Snapshot(path).restore({"sd": out})
    return dict(out)


def test_second_take_reuses_plan_and_saves_new_values(tmp_path, resident):
    sd = _state(resident)
    with override_max_chunk_size_bytes(400_000):
        ref = []
        for i in range(3):
            for k, v in sd.items():
                if isinstance(v, torch.Tensor):
                    v.add_(1.0)           # new values, same tensors
            sd["step"] = i                # primitives and objects change too
            sd["meta"] = {"lr": 0.1 / (i + 1), "tags": ["a"] * (i + 1)}
            Snapshot.take(str(tmp_path / f"s{i}"), {"sd": sd})
            ref.append(_snap(sd))
    assert plan_cache.stats["hits"] == 2 and plan_cache.stats["stores"] == 1
    for i in range(3):
        got = _restore(str(tmp_path / f"s{i}"), ref[i])
        assert_state_dict_eq(got, ref[i])
    # the reused takes wrote the same tensor entries as the fresh plan
    m0 = Snapshot(str(tmp_path / "s0")).get_manifest()
    m2 = Snapshot(str(tmp_path / "s2")).get_manifest()
    tens = sorted(k for k in m0 if k.startswith(("0/sd/g", "0/sd/big")))
    assert len(tens) == 13
    assert [repr(m0[k]) for k in tens] == [repr(m2[k]) for k in tens]


def test_plan_sharing_slabs_with_per_take_leaves_is_not_cached(tmp_path, resident):
    sd = _state(resident, n=4, host=True)
    refs = []
    for i in range(2):
        sd["c0"].add_(1.0)
        sd["g0"].add_(1.0)
        Snapshot.take(str(tmp_path / f"s{i}"), {"sd": sd})
        refs.append(_snap(sd))
    assert plan_cache.stats["hits"] == 0 and plan_cache.stats["stores"] == 0
    for i in range(2):
        assert_state_dict_eq(_restore(str(tmp_path / f"s{i}"), refs[i]), refs[i])
    # unbatched, resident and per-take blobs are separate: reuse works
    from hipsnapshot.knobs import override_is_batching_disabled

    with override_is_batching_disabled(True):
        for i in range(2, 4):
            sd["c0"].add_(1.0)
            sd["g0"].add_(1.0)
            Snapshot.take(str(tmp_path / f"s{i}"), {"sd": sd})
            refs.append(_snap(sd))
    assert plan_cache.stats["hits"] == 1
    for i in range(2, 4):
        assert_state_dict_eq(_restore(str(tmp_path / f"s{i}"), refs[i]), refs[i])


def test_replaced_tensor_invalidates_plan(tmp_path, resident):
    sd = _state(resident, n=3)
    Snapshot.take(str(tmp_path / "a"), {"sd": sd})
    new = torch.full_like(sd["g1"], 7.0)   # same shape, different memory
    resident.add(id(new))
    sd["g1"] = new
    Snapshot.take(str(tmp_path / "b"), {"sd": sd})
    assert plan_cache.stats["hits"] == 0
    got = _restore(str(tmp_path / "b"), sd)
    assert torch.equal(got["g1"], new)


def test_knob_disables_reuse(tmp_path, resident):
    sd = _state(resident, n=3)
    with override_knob("PLAN_CACHE", "0"):
        Snapshot.take(str(tmp_path / "a"), {"sd": sd})
        Snapshot.take(str(tmp_path / "b"), {"sd": sd})
    assert plan_cache.stats["hits"] == 0 and plan_cache.stats["stores"] == 0


def test_async_takes_reuse_and_are_isolated(tmp_path, resident):
    sd = _state(resident, n=4)
    refs = []
    for i in range(3):
        for v in sd.values():
            if isinstance(v, torch.Tensor):
                v.mul_(2.0)
        refs.append(_snap(sd))
        p = Snapshot.async_take(str(tmp_path / f"a{i}"), {"sd": sd})
        for v in sd.values():  # must not leak into the snapshot
            if isinstance(v, torch.Tensor):
                v.fill_(-5.0)
        p.wait()
        for k, v in refs[-1].items():
            if isinstance(v, torch.Tensor):
                sd[k].copy_(v)
    assert plan_cache.stats["hits"] == 2
    for i in range(3):
        assert_state_dict_eq(_restore(str(tmp_path / f"a{i}"), refs[i]), refs[i])


def test_busy_plan_is_not_shared(tmp_path, resident, monkeypatch):
    """A take that starts while an async take still drains with the plan
    plans from scratch (the draining take owns the plan's stagers)."""
    from hipsnapshot.storage.fs import FSStoragePlugin

    sd = _state(resident, n=4)
    Snapshot.take(str(tmp_path / "warm"), {"sd": sd})  # plan stored (sync)
    Snapshot.async_take(str(tmp_path / "warm_a"), {"sd": sd}).wait()  # async plan stored
    orig = FSStoragePlugin.write

    async def slow_write(self, write_io):
        await asyncio.sleep(0.3)
        await orig(self, write_io)

    monkeypatch.setattr(FSStoragePlugin, "write", slow_write)
    ref = _snap(sd)
    p = Snapshot.async_take(str(tmp_path / "slow"), {"sd": sd})   # hit: plan busy
    hits = plan_cache.stats["hits"]
    p2 = Snapshot.async_take(str(tmp_path / "second"), {"sd": sd})  # must miss
    assert plan_cache.stats["hits"] == hits
    p.wait()
    p2.wait()
    monkeypatch.setattr(FSStoragePlugin, "write", orig)
    for name in ("slow", "second"):
        assert_state_dict_eq(_restore(str(tmp_path / name), ref), ref)


def test_plan_dropped_when_state_is_collected(tmp_path, resident):
    sd = _state(resident, n=3)
    Snapshot.take(str(tmp_path / "a"), {"sd": sd})
    assert len(plan_cache._plans) == 1
    del sd
    gc.collect()
    assert len(plan_cache._plans) == 0


def test_new_view_objects_each_take_still_reuse(tmp_path, resident, monkeypatch):
    """A state_dict that returns fresh views of the same memory on every call
    misses the identity fast path but matches the full signatures."""
    monkeypatch.setattr(plan_cache, "is_resident",
                        lambda obj: isinstance(obj, torch.Tensor) and obj.numel() >= 1000)

    class Holder:
        def __init__(self):
            self.w = torch.randn(4000)
            self.b = torch.randn(2000, 3)

        def state_dict(self):
            return {"w": self.w.detach(), "b": self.b[:, :]}

        def load_state_dict(self, sd):
            self.w.copy_(sd["w"])
            self.b.copy_(sd["b"])

    h = Holder()
    refs = []
    for i in range(3):
        h.w.add_(1)
        h.b.mul_(2)
        Snapshot.take(str(tmp_path / f"v{i}"), {"h": h})
        refs.append((h.w.clone(), h.b.clone()))
    assert plan_cache.stats["hits"] == 2
    for i, (w, b) in enumerate(refs):
        out = Holder()
        Snapshot(str(tmp_path / f"v{i}")).restore({"h": out})
        assert torch.equal(out.w, w) and torch.equal(out.b, b)


def test_fresh_app_state_dict_each_take_reuses_plan(tmp_path, resident):
    """``{"sd": sd, "progress": StateDict(step=i)}`` rebuilt every take: the
    resident leaves are the same, so the plan is reused."""
    sd = _state(resident, n=3)
    for i in range(3):
        Snapshot.take(str(tmp_path / f"f{i}"), {"sd": sd, "progress": StateDict(step=i)})
    assert plan_cache.stats["hits"] == 2
    prog = StateDict(step=-1)
    Snapshot(str(tmp_path / "f2")).restore({"progress": prog})
    assert prog["step"] == 2


@pytest.mark.parametrize("is_async", [False, True])
def test_failed_planning_releases_reused_plan(tmp_path, resident, monkeypatch, is_async):
    """A take that found a cached plan and then failed while planning the rest
    (batching here) must hand the plan back: the next take reuses it."""
    import hipsnapshot.snapshot as snapmod

    def take(path):
        if is_async:
            Snapshot.async_take(path, {"sd": sd}).wait()
        else:
            Snapshot.take(path, {"sd": sd})

    sd = _state(resident)
    take(str(tmp_path / "s0"))  # plans are per mode (sync / async)
    orig = snapmod.batch_write_requests

    def boom(*a, **k):
        raise RuntimeError("planning failed")

    monkeypatch.setattr(snapmod, "batch_write_requests", boom)
    with pytest.raises(RuntimeError, match="planning failed"):
        take(str(tmp_path / "s1"))
    monkeypatch.setattr(snapmod, "batch_write_requests", orig)
    assert plan_cache.stats["hits"] == 1
    for k, v in sd.items():
        if isinstance(v, torch.Tensor):
            v.add_(1.0)
    ref = _snap(sd)
    take(str(tmp_path / "s2"))
    assert plan_cache.stats["hits"] == 2, plan_cache.stats
    got = _restore(str(tmp_path / "s2"), ref)
    for k, v in ref.items():
        if isinstance(v, torch.Tensor):
            assert torch.equal(got[k], v), k


@pytest.mark.parametrize("is_async", [False, True])
def test_plan_building_take_collects_once(tmp_path, resident, monkeypatch, is_async):
    """The async take that stores a new plan runs ONE full GC pass in its
    commit thread; takes that reuse it run none; the knob turns it off.  A
    blocking take forces none (round 5: the pass is the process's first full
    collection, a one-time cost wherever it lands)."""
    calls = []
    real = gc.collect
    monkeypatch.setattr(gc, "collect", lambda *a, **k: calls.append(a) or real(*a, **k))
    sd = _state(resident)

    def take(i):
        if is_async:
            Snapshot.async_take(str(tmp_path / f"s{i}"), {"sd": sd}).wait()
        else:
            Snapshot.take(str(tmp_path / f"s{i}"), {"sd": sd})

    n = 1 if is_async else 0
    take(0)
    assert plan_cache.stats["stores"] == 1 and len(calls) == n
    take(1)
    take(2)
    assert plan_cache.stats["hits"] == 2 and len(calls) == n
    plan_cache.clear()
    with override_knob("GC_AFTER_PLAN", "0"):
        take(3)
    assert plan_cache.stats["stores"] == 2 and len(calls) == n
