"""Observability: roctx ranges, a periodic write-progress reporter, JSON timing records.

* ``roctx_range(name)`` -- pushes a ROCTx range (``libroctx64.so`` from the torch
  ROCm wheel or ``/opt/rocm``) so ``rocprofv3 --marker-trace`` shows
  stage / D2H / write / commit phases next to the HIP kernels.  Enabled with
  ``HIPSNAPSHOT_ROCTX=1``; a no-op otherwise.
* ``WriteReporter`` -- the reference's ``_WriteReporter``
  (`/root/reference/torchsnapshot/scheduler.py:93-175`): a DEBUG-level table of
  per-rank progress (staged / written / in-flight bytes, RSS delta, budget)
  logged every ``interval_s`` while a write pipeline runs.
"""

from __future__ import annotations

import contextlib
import ctypes
import glob
import logging
import os
import time
from typing import Optional

import psutil

logger = logging.getLogger("hipsnapshot.scheduler")

_roctx = None
_roctx_tried = False


def _load_roctx():
    global _roctx, _roctx_tried
    if _roctx_tried:
        return _roctx
    _roctx_tried = True
    if os.environ.get("HIPSNAPSHOT_ROCTX", "0") != "1":
        return None
    cands = []
    try:
        import torch

        cands += glob.glob(os.path.join(os.path.dirname(torch.__file__), "lib", "libroctx64.so*"))
    except Exception:  # pragma: no cover
        pass
    cands += glob.glob("/opt/rocm/lib/libroctx64.so*")
    for c in cands:
        try:
            lib = ctypes.CDLL(c)
            lib.roctxRangePushA.argtypes = [ctypes.c_char_p]
            lib.roctxRangePushA.restype = ctypes.c_int
            lib.roctxRangePop.restype = ctypes.c_int
            _roctx = lib
            break
        except OSError:
            continue
    return _roctx


@contextlib.contextmanager
def roctx_range(name: str):
    lib = _load_roctx()
    if lib is None:
        yield
        return
    lib.roctxRangePushA(name.encode())
    try:
        yield
    finally:
        lib.roctxRangePop()


class WriteReporter:
    def __init__(self, rank: int, memory_budget_bytes: int, interval_s: float = 5.0) -> None:
        self.rank = rank
        self.budget = memory_budget_bytes
        self.interval_s = interval_s
        self.t0 = time.monotonic()
        self.last = self.t0
        self.rss0 = psutil.Process().memory_info().rss

    def maybe_report(self, n_pending: int, n_staging: int, n_io: int, in_use: int,
                     bytes_written: int, force: bool = False) -> Optional[str]:
        now = time.monotonic()
        if not force and now - self.last < self.interval_s:
            return None
        if not logger.isEnabledFor(logging.DEBUG) and not force:
            return None
        self.last = now
        rss = psutil.Process().memory_info().rss - self.rss0
        line = (f"rank {self.rank} t={now - self.t0:7.2f}s stage-able={n_pending:5d} "
                f"staging={n_staging:3d} writing={n_io:4d} in-use={in_use / 2**30:7.2f}GiB "
                f"rss-delta={rss / 2**30:7.2f}GiB budget={self.budget / 2**30:7.2f}GiB "
                f"written={bytes_written / 1e9:8.3f}GB")
        logger.debug(line)
        return line


class Timeline:
    """Per-process span recorder dumped as a Chrome/Perfetto trace.

    Enabled with ``HIPSNAPSHOT_TIMELINE=<path prefix>``: every take / restore
    writes ``<prefix>.rank<R>.<op><N>.json`` with one complete event per
    planning phase, per staged request (D2H / gather) and per storage write or
    read, on the thread that ran it.  Open it in ui.perfetto.dev next to a
    ``rocprofv3 --kernel-trace`` of the same run to see where a snapshot's
    wall time goes.  Disabled, ``span`` costs one attribute check.
    """

    def __init__(self) -> None:
        self.prefix = os.environ.get("HIPSNAPSHOT_TIMELINE") or None
        self.events: list = []
        self.t0 = time.perf_counter()
        self.counts: dict = {}
        self._captured: Optional[list] = None

    @contextlib.contextmanager
    def capture(self):
        """Record spans in memory for the duration, without writing trace
        files: yields the list the events land in (``bench.py``'s per-rank
        phase split)."""
        saved = (self.prefix, self.events, self._captured)
        out: list = []
        self.prefix = self.prefix or "<capture>"
        self.events = []
        self._captured = out
        try:
            yield out
        finally:
            out.extend(self.events)
            self.prefix, self.events, self._captured = saved

    @property
    def enabled(self) -> bool:
        return self.prefix is not None

    def add(self, name: str, cat: str, t_start: float, t_end: float, **args) -> None:
        if self.prefix is None:
            return
        import threading

        self.events.append({"name": name, "cat": cat, "ph": "X",
                            "ts": (t_start - self.t0) * 1e6, "dur": (t_end - t_start) * 1e6,
                            "pid": os.getpid(), "tid": threading.get_ident() % 100000,
                            "args": args})

    @contextlib.contextmanager
    def span(self, name: str, cat: str = "phase", **args):
        if self.prefix is None:
            yield
            return
        t = time.perf_counter()
        try:
            yield
        finally:
            self.add(name, cat, t, time.perf_counter(), **args)

    def dump(self, op: str, rank: int) -> Optional[str]:
        if self._captured is not None:
            self._captured.extend(self.events)
            self.events = []
            return None
        if self.prefix is None or not self.events:
            return None
        import json

        n = self.counts.get(op, 0)
        self.counts[op] = n + 1
        path = f"{self.prefix}.rank{rank}.{op}{n}.json"
        os.makedirs(os.path.dirname(os.path.abspath(path)), exist_ok=True)
        with open(path, "w") as f:
            json.dump({"traceEvents": self.events, "displayTimeUnit": "ms"}, f)
        self.events = []
        return path


timeline = Timeline()


class GcWatch:
    """Records the duration of every Python cyclic-GC pass (``gc.callbacks``).

    A generation-2 pass walks the whole heap -- 100+ ms in a process that
    imported torch and built a model -- and lands wherever the allocation
    counters run over, e.g. right after a take re-enables GC.  Benchmarks use
    this to report how much of a timed region was GC; with a timeline enabled
    each pass is also a ``gc`` span."""

    def __init__(self) -> None:
        self.events: list = []  # (generation, t_start, t_end)
        self._t = 0.0
        self._on = False

    def start(self) -> "GcWatch":
        import gc

        if not self._on:
            gc.callbacks.append(self._cb)
            self._on = True
        return self

    def stop(self) -> None:
        import gc

        if self._on:
            gc.callbacks.remove(self._cb)
            self._on = False

    def _cb(self, phase: str, info: dict) -> None:
        if phase == "start":
            self._t = time.perf_counter()
            return
        t1 = time.perf_counter()
        self.events.append((info.get("generation", -1), self._t, t1))
        timeline.add(f"gc_gen{info.get('generation', -1)}", "gc", self._t, t1,
                     collected=info.get("collected", 0))

    def ms_between(self, t_start: float, t_end: float, min_generation: int = 0) -> float:
        return 1e3 * sum(max(0.0, min(b, t_end) - max(a, t_start))
                         for g, a, b in self.events if g >= min_generation)


@contextlib.contextmanager
def paused_gc(defer_plan_gc: Optional[list] = None, plan_gc: bool = True):
    """Suspend Python's cyclic GC for a bounded critical section.

    Planning a snapshot allocates tens of thousands of small objects (entries,
    requests, futures); in a training process with a large heap that triggers
    generation-2 collections costing 10-100 ms each in the middle of a take
    (measured: parsing an 8-rank manifest 129 ms with GC vs 16 ms without).
    Garbage created meanwhile is collected after the section.

    A take that built (and cached) a new take plan ends with one full
    collection (``knobs.TUNING.gc_after_plan``, default on).  The plan's
    objects are long-lived; CPython runs a full pass once the objects that
    survived into the oldest generation since the last full pass reach 25 %
    of those counted by it, and a training loop allocates almost nothing
    else, so that pass (160-200 ms with Llama-3-8B + AdamW loaded,
    profiles/r3/overlap/) would otherwise fall into the NEXT take's unblock
    or a training step.  Collecting at the end of the plan-building take puts
    the one-time cost where the first take's other one-time costs are.

    ``defer_plan_gc`` (a list): instead of collecting, append True to it --
    ``async_take`` runs that pass in its commit thread once the drain is done,
    off the unblock path (while a GPU-bound training step waits on the
    device with the GIL released).

    ``plan_gc=False`` (blocking takes): no forced pass.  It is the process's
    first full collection -- 140 ms with torch loaded, whatever the plan --
    and a one-time cost either way; forced, it made the first blocking take
    of the Llama-3-8B bench 0.38 s instead of 0.24 s, and without it no full
    pass fell into a later timed take or restore (profiles/r5/cold_take/)."""
    import gc

    from .. import knobs

    was = gc.isenabled()
    gc.disable()
    try:
        yield
    finally:
        if was:
            gc.enable()
            from ..engine import plan_cache

            if plan_cache.take_stored_flag() and knobs.gc_after_plan() and plan_gc:
                if defer_plan_gc is not None:
                    defer_plan_gc.append(True)
                else:
                    with timeline.span("gc_after_plan"):
                        gc.collect()
