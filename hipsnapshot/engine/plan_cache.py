"""Reuse of a take's plan across takes of the same device-resident state.

A training job snapshots the same tensors every N steps.  Planning them --
``state_dict`` flattening aside -- is pure CPU work whose result only depends
on WHICH tensors are saved (address, shape, strides, dtype, device, sharding)
and on the take's settings: the manifest entries, the write requests with
their stagers, the slab layout, the compression plan and each entry's JSON
fragment.  For Llama-3-8B FSDP that is ~5-7 ms per take on one MI355X
(``prepare_write`` 2 ms, batching 0.7 ms, compression planning 0.6 ms,
metadata JSON 2 ms; ``profiles/timeline_r2/``), i.e. the bulk of an
``async_take``'s time-to-unblock and a fixed cost per take that grows in
relative terms with the number of ranks (each rank plans its own shards).

Only DEVICE-RESIDENT tensor leaves (CUDA tensors, DTensor / ShardedTensor
with CUDA local shards) are cached.  Primitives, objects and host tensors --
the RNG state is a fresh host tensor on every call -- are planned on every
take and batched separately, into slabs with their own name prefix
(``r<rank>v_...``), so they never collide with the plan's slabs.

Soundness:

* a plan is reused only if every resident leaf has the same signature
  (data_ptr, shape, strides, dtype, device; DTensor placements + mesh +
  global shape; ShardedTensor shard boxes) in the same logical order, and
  the settings key (rank, world size, sync/async, quantize globs,
  compression, the knob values a plan depends on (``knobs.plan_settings``),
  the app-state keys) matches;
* the plan holds the leaves it was built from, so no address it matched can
  be recycled by the caching allocator while the plan exists -- equal
  data_ptr means the same memory.  The plan is dropped when an app-state
  object that owns a cached leaf is garbage collected (``weakref.finalize``),
  on the next mismatch, or by ``clear()``;
* a plan is used by one take at a time (``busy`` until its I/O completed --
  an ``async_take`` still draining owns its stagers); a take that finds the
  plan busy plans from scratch;
* stagers are reset before reuse (``TensorBufferStager.reset_for_reuse``:
  the async HBM freeze re-points them at arena views) and pick up the
  caller's CURRENT stream as producer.

Replicated state (DDP) is not cached: partitioning its writes is a
collective, and ranks must not disagree about running it.
"""

from __future__ import annotations

import os
import threading
import weakref
from typing import Any, Dict, Iterator, List, Optional

import torch

from .. import knobs
from ..format.manifest import Entry, iter_tensor_entries
from ..io_types import WriteReq

try:
    from torch.distributed.tensor import DTensor
except Exception:  # pragma: no cover
    DTensor = None  # type: ignore[assignment]

try:
    from torch.distributed._shard.sharded_tensor import ShardedTensor
except Exception:  # pragma: no cover
    ShardedTensor = None  # type: ignore[assignment]

_lock = threading.Lock()
_plans: Dict[tuple, "TakePlan"] = {}
stats = {"hits": 0, "misses": 0, "stores": 0}


def enabled() -> bool:
    return knobs.plan_cache_enabled()


def _local(obj: Any) -> Optional[torch.Tensor]:
    if DTensor is not None and isinstance(obj, DTensor):
        return obj._local_tensor
    if ShardedTensor is not None and isinstance(obj, ShardedTensor):
        shards = obj.local_shards()
        return shards[0].tensor if shards else None
    return obj if isinstance(obj, torch.Tensor) else None


def is_resident(obj: Any) -> bool:
    """Leaves whose plan can be reused: tensors in device memory (tests
    monkeypatch this to exercise the cache on the CPU)."""
    t = _local(obj)
    return t is not None and t.is_cuda


def _tsig(t: torch.Tensor) -> tuple:
    return (t.data_ptr(), tuple(t.shape), tuple(t.stride()), t.dtype, t.device)


def leaf_sig(obj: Any) -> tuple:
    if DTensor is not None and isinstance(obj, DTensor):
        return ("d", _tsig(obj._local_tensor), tuple(obj.placements), id(obj.device_mesh),
                tuple(obj.shape))
    if ShardedTensor is not None and isinstance(obj, ShardedTensor):
        return ("s", tuple((_tsig(s.tensor), tuple(s.metadata.shard_offsets),
                            tuple(s.metadata.shard_sizes)) for s in obj.local_shards()),
                tuple(obj.size()))
    return ("t",) + _tsig(obj)


def signatures(resident: Dict[str, Any]) -> tuple:
    return tuple((k, leaf_sig(v)) for k, v in resident.items())


def fast_signatures(resident: Dict[str, Any]) -> Optional[tuple]:
    """Identity-based signatures: the leaf OBJECT (plans keep theirs alive,
    so ids cannot be recycled) plus what can change under a live object --
    the local tensor's address / shape / strides and the DTensor spec
    object.  ~1 us per leaf instead of ~4 us for ``signatures``; None when a
    leaf needs the full comparison (ShardedTensor)."""
    out = []
    for k, v in resident.items():
        lt = getattr(v, "_local_tensor", None)
        if lt is not None:
            out.append((id(v), lt.data_ptr(), lt.shape, lt.stride(), lt.dtype, id(v._spec)))
        elif ShardedTensor is not None and isinstance(v, ShardedTensor):
            return None
        else:
            out.append((id(v), v.data_ptr(), v.shape, v.stride(), v.dtype, v.device))
    return tuple(out)


def capture(resident: Dict[str, Any]) -> Optional[tuple]:
    """What a plan must remember of its leaves, taken once when it is
    stored (~1 us per leaf; the full ``signatures`` cost ~4 us): the leaf
    object's id, its local tensor's address / shape / strides / dtype /
    device and, for a DTensor, its (immutable) spec object -- from which the
    full signature is derived only when a later take presents new leaf
    objects.  None when a leaf needs the full signature (ShardedTensor)."""
    out = []
    for v in resident.values():
        lt = getattr(v, "_local_tensor", None)
        if lt is not None:
            out.append((id(v), lt.data_ptr(), lt.shape, lt.stride(), lt.dtype, lt.device,
                        v._spec))
        elif ShardedTensor is not None and isinstance(v, ShardedTensor):
            return None
        else:
            out.append((id(v), v.data_ptr(), v.shape, v.stride(), v.dtype, v.device, None))
    return tuple(out)


def _same_objects(a: tuple, b: tuple) -> bool:
    """The same leaf objects pointing at the same memory in the same layout."""
    return len(a) == len(b) and all(x[:6] == y[:6] and x[6] is y[6] for x, y in zip(a, b))


def _same_layout(a: tuple, b: tuple) -> bool:
    """Possibly other leaf objects, over the same memory, shapes and
    sharding (``signatures`` equality, from captured facts)."""
    if len(a) != len(b):
        return False
    for x, y in zip(a, b):
        if x[1:6] != y[1:6]:
            return False
        sx, sy = x[6], y[6]
        if (sx is None) != (sy is None):
            return False
        if sx is not None and (tuple(sx.placements) != tuple(sy.placements)
                               or sx.mesh is not sy.mesh or tuple(sx.shape) != tuple(sy.shape)):
            return False
    return True


def settings_key(app_state: Dict[str, Any], rank: int, world_size: int, is_async: bool,
                 quantize, compression: str) -> tuple:
    """Everything besides the leaves that shapes a plan.  The app-state KEYS
    are part of it, not the objects: ``{"model": m, "progress": StateDict(
    step=i)}`` rebuilt for every take must still reuse the model's plan (the
    leaf signatures establish that the model's tensors are the same)."""
    return (tuple(sorted(app_state)), rank, world_size, bool(is_async),
            tuple(quantize or ()), compression, knobs.plan_settings())


_STAGER_TYPES: Optional[tuple] = None


def _stager_types() -> tuple:
    """(single-tensor stager, slab stagers); imported once (io imports this
    package: a function-level import on every call cost ~1 us each, ~0.9 ms
    of a cold async_take's unblock over its ~430 calls)."""
    global _STAGER_TYPES
    if _STAGER_TYPES is None:
        from ..io.batcher import BatchedBufferStager, GPUBatchedBufferStager
        from ..io.tensor import TensorBufferStager

        _STAGER_TYPES = (TensorBufferStager, (GPUBatchedBufferStager, BatchedBufferStager))
    return _STAGER_TYPES


def _tensor_stagers(write_reqs: List[WriteReq]) -> Iterator[Any]:
    single, slabs = _stager_types()
    for wr in write_reqs:
        st = wr.buffer_stager
        if isinstance(st, single):
            yield st
        elif isinstance(st, slabs):
            for _, m in st.members:
                yield m


class TakePlan:
    def __init__(self, key: tuple, sigs: Optional[tuple], keep: List[Any],
                 entries: Dict[str, Entry], write_reqs: List[WriteReq],
                 cap: Optional[tuple] = None) -> None:
        self.key = key
        self.sigs = sigs  # full signatures, only when ``capture`` cannot describe a leaf
        self.cap = cap
        self.keep = keep          # the leaves: their addresses stay reserved
        self.entries = entries    # logical path -> final Entry (batched / compressed)
        self.write_reqs = write_reqs
        self.json: Dict[str, str] = {}  # logical path -> entry JSON (metadata gather)
        self.owner_ids: set = set()  # ids of the app-state objects behind the leaves
        self.busy = True
        # stagers changed since the last reset (an async take's HBM freeze
        # re-points them); a blocking take leaves them as planned
        self.mutated = True
        # an async take's freeze resets only the stagers it does not re-point
        # (``lookup(defer_reset=True)``, ``reset_except``)
        self.pending_reset = False
        self._streams: Optional[tuple] = None  # producer streams at the last reset
        self._devices: tuple = ()

    def _current_streams(self) -> tuple:
        return tuple(int(torch.cuda.current_stream(d).cuda_stream) for d in self._devices)

    def reset(self) -> None:
        """Stagers back to their planned state, producer = current stream.
        Skipped when nothing changed them since the last reset and the
        devices' current streams are the same (every blocking take: ~0.35 ms
        of the 291 Llama-3-8B stagers)."""
        if not self.mutated and self._streams is not None and \
                self._current_streams() == self._streams:
            return
        from . import staging

        devs = set()
        with staging.plan_scope():
            for st in _tensor_stagers(self.write_reqs):
                st.reset_for_reuse()
                t = st.tensor
                if t.is_cuda:
                    devs.add(t.get_device())
        self._devices = tuple(sorted(devs))
        self._streams = self._current_streams()
        self.mutated = False
        self.pending_reset = False

    def reset_except(self, keep: set) -> None:
        """Reset every stager whose id is not in ``keep`` (the ones an HBM
        freeze just re-pointed at its arena, which it set up completely)."""
        from . import staging

        with staging.plan_scope():
            for st in _tensor_stagers(self.write_reqs):
                if id(st) not in keep:
                    st.reset_for_reuse()
        self.pending_reset = False


def lookup(key: tuple, resident: Dict[str, Any], defer_reset: bool = False
           ) -> Optional[TakePlan]:
    """The cached plan for ``key`` if every resident leaf still matches it
    (marked busy for the caller's take), else None.  ``defer_reset``: the
    take freezes the plan's device state next; the freeze resets only the
    stagers it does not re-point (~0.5 ms of every warm async unblock)."""
    with _lock:
        p = _plans.get(key)
        if p is None or p.busy:
            stats["misses"] += 1
            return None
    if p.cap is not None:
        cur = capture(resident)
        # new leaf objects (e.g. views a state_dict creates on every call):
        # compare what they point at
        ok = cur is not None and (_same_objects(cur, p.cap) or _same_layout(cur, p.cap))
    else:
        ok = signatures(resident) == p.sigs
    if not ok:
        stats["misses"] += 1
        return None
    with _lock:
        if p.busy or _plans.get(key) is not p:
            stats["misses"] += 1
            return None
        p.busy = True
        stats["hits"] += 1
    if defer_reset and p.mutated:
        p.pending_reset = True
    else:
        p.reset()
    return p


def store(key: tuple, resident: Dict[str, Any], object_entries: Dict[str, Entry],
          write_reqs: List[WriteReq], owners: List[Any]) -> Optional[TakePlan]:
    """Keep the resident part of a fresh plan; returns it marked busy (the
    caller's take is using it), or None when it cannot be cached.  ``owners``:
    the app-state objects the resident leaves come from -- the plan is
    dropped (and its tensors released) when any of them is collected."""
    cap = capture(resident)
    sigs = signatures(resident) if cap is None else None
    entries = {k: object_entries[k] for k in resident if k in object_entries}
    if len(entries) != len(resident):
        return None
    ids = {id(te) for e in entries.values() for te in iter_tensor_entries(e)}
    mine: List[WriteReq] = []
    covered = set()
    for wr in write_reqs:
        sts = list(_tensor_stagers([wr]))
        if sts and all(id(st.entry) in ids for st in sts):
            mine.append(wr)
            covered.update(id(st.entry) for st in sts)
    if covered != ids:
        # some resident blob is shared with a per-take leaf (e.g. a slab that
        # also holds a host tensor): the resident part cannot be replayed alone
        return None
    keep = list(resident.values())
    for v in resident.values():
        if DTensor is not None and isinstance(v, DTensor):
            keep.append(v.device_mesh)
    plan = TakePlan(key, sigs, keep, entries, mine, cap)
    plan.owner_ids = {id(v) for v in owners}
    for v in owners:
        if id(v) in _watched:
            continue
        try:
            weakref.finalize(v, _drop_object, id(v))
        except TypeError:  # not weak-referenceable: never cached
            return None
        _watched.add(id(v))
    with _lock:
        old = _plans.get(key)
        if old is not None and old.busy:
            return None  # an async take still drains with it: keep that one
        _plans[key] = plan
        stats["stores"] += 1
    global _stored_since_collect
    _stored_since_collect = True
    return plan


_stored_since_collect = False


def take_stored_flag() -> bool:
    """True once after a take stored a new plan (see ``tracing.paused_gc``)."""
    global _stored_since_collect
    f, _stored_since_collect = _stored_since_collect, False
    return f


_watched: set = set()  # ids of app-state objects with a finalizer


def _drop_object(obj_id: int) -> None:
    """An app-state object was garbage collected: drop every plan keyed on
    it (their tensors are released with them)."""
    with _lock:
        _watched.discard(obj_id)
        for key in [k for k, p in _plans.items() if obj_id in p.owner_ids]:
            del _plans[key]


def release(plan: Optional[TakePlan]) -> None:
    if plan is not None:
        with _lock:
            plan.busy = False


def clear() -> None:
    """Forget every cached plan (and release the tensors they hold)."""
    with _lock:
        _plans.clear()
