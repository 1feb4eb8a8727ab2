"""Reuse of a restore's native plan across restores of the same snapshot into
the same device-resident state.

Planning a restore -- the manifest for this rank, ``prepare_read`` for every
entry, read batching, the native job's items and copy descriptors -- is CPU
work whose result only depends on WHICH snapshot is read (its metadata file
identity) and on WHICH tensors receive it (address, shape, strides, dtype,
device, sharding).  For one rank's share of an 8-GPU Llama-3-8B restore that
was ~7 ms in front of a ~25 ms transfer (profiles/r4/restore_native/).  A
plan is recorded only when the whole restore of one stateful went through the
native job in place (every leaf read into its own tensor, nothing left to the
Python pipeline or to ``load_state_dict``); a later restore of the same
snapshot into the same leaves runs the recorded job directly.

Soundness (mirrors engine/plan_cache.py):

* the key holds the snapshot's metadata file identity (path, device, inode,
  size, mtime: a take rewrites the metadata last, by rename, so any new take
  at that path is a different key -- the blob sizes the plan read with
  ``stat`` belong to that snapshot), the stateful's key, rank, world size,
  the knob values a plan depends on (``knobs.plan_settings``: not tracing,
  thread counts or other variables that leave the plan as it is), and the
  identity signature of every leaf in order;
* the plan holds the leaves, so no address it matched can be recycled while
  it exists; it is dropped when the stateful object is garbage collected,
  on ``clear()``, or when more than ``_MAX`` plans are cached;
* the destinations' producer streams are taken again at every use (the
  caller's CURRENT streams).

Reference counterpart: the reference plans every restore from scratch
(`/root/reference/torchsnapshot/snapshot.py:650-729`).
"""

from __future__ import annotations

import os
import threading
import weakref
from collections import OrderedDict
from typing import Any, Dict, List, Optional

import torch

from .. import knobs
from .plan_cache import fast_signatures, leaf_sig

try:
    from torch.distributed.tensor import DTensor
except Exception:  # pragma: no cover
    DTensor = None  # type: ignore[assignment]

_MAX = 4
_lock = threading.Lock()
_plans: "OrderedDict[tuple, RestorePlan]" = OrderedDict()
stats = {"hits": 0, "misses": 0, "stores": 0}


class RestorePlan:
    def __init__(self, jobs: Dict[int, list], keep: List[Any], n_bytes: int) -> None:
        # (read req, item, producers) per device; the read requests are not
        # reused -- only their item tuples and paths (error messages)
        self.jobs = {dev: [(e[0].path, e[1]) for e in entries] for dev, entries in jobs.items()}
        self.keep = keep
        self.n_bytes = n_bytes


def enabled() -> bool:
    return knobs.restore_plan_cache_enabled()


def key_for(metadata_key: Optional[tuple], stateful_key: str, rank: int, world_size: int,
            flat: Dict[str, Any]) -> Optional[tuple]:
    """Cache key, or None when the restore cannot be cached (non-local
    snapshot, a leaf that is not a device tensor / DTensor)."""
    if metadata_key is None or not flat:
        return None
    for v in flat.values():
        if DTensor is not None and isinstance(v, DTensor):
            t = v._local_tensor
        elif type(v) is torch.Tensor or type(v) is torch.nn.Parameter:
            t = v
        else:  # ShardedTensor and tensor subclasses: planned every time
            return None
        if not t.is_cuda:
            return None
    sigs = fast_signatures(flat)
    if sigs is None:
        sigs = tuple((k, leaf_sig(v)) for k, v in flat.items())
    from .. import knobs

    return (metadata_key, stateful_key, rank, world_size, knobs.plan_settings(), tuple(flat),
            sigs)


def lookup(key: Optional[tuple]) -> Optional[RestorePlan]:
    if key is None or not enabled():
        return None
    with _lock:
        plan = _plans.get(key)
        if plan is None:
            stats["misses"] += 1
            return None
        _plans.move_to_end(key)
        stats["hits"] += 1
        return plan


def store(key: Optional[tuple], stateful: Any, jobs: Dict[int, list], flat: Dict[str, Any]
          ) -> None:
    if key is None or not enabled() or not jobs:
        return
    n_bytes = sum(e[1][4] for entries in jobs.values() for e in entries)
    plan = RestorePlan(jobs, list(flat.values()), n_bytes)
    with _lock:
        _plans[key] = plan
        _plans.move_to_end(key)
        stats["stores"] += 1
        while len(_plans) > _MAX:
            _plans.popitem(last=False)
    try:
        weakref.finalize(stateful, _drop, key)
    except TypeError:  # not weak-referenceable: bounded by _MAX only
        pass


def _drop(key: tuple) -> None:
    with _lock:
        _plans.pop(key, None)


def clear() -> None:
    with _lock:
        _plans.clear()


def run(plan: RestorePlan, budget: Optional[int] = None, verifier=None) -> int:
    """Run a recorded plan's native jobs, ordered after the callers' current
    streams on each device; returns the logical bytes restored.  ``verifier``:
    hash the whole blobs in the job (the caller finishes the partial ones)."""
    from . import native_restore

    jobs = {}
    for dev, entries in plan.jobs.items():
        prod = [int(torch.cuda.current_stream(dev).cuda_stream)]
        jobs[dev] = [(_Path(path), item, prod) for path, item in entries]
    return native_restore.run(jobs, budget, verifier)


class _Path:
    """Stands in for the read request in native_restore.run's error text."""

    __slots__ = ("path",)

    def __init__(self, path: str) -> None:
        self.path = path
