"""Memory-budgeted write / read pipelines.

Reference: `/root/reference/torchsnapshot/scheduler.py:27-461`.  Same contract --
write requests move ready -> staging -> ready-for-io -> io under a per-rank
host-memory budget, and ``execute_write_reqs`` returns a ``PendingIOWork`` as
soon as everything is STAGED (that is the async-take unblock point) -- with
these changes:

* admission and completion are O(1) per request (deques + one
  ``asyncio.wait`` over the in-flight set) instead of re-scanning sets every
  iteration (O(n^2), Appendix C / SURVEY 7.4 #10);
* staged buffers are released (back to the pinned pool) the moment their
  write finishes, and the budget is returned at the same time;
* read destinations are provided by the consumers (pinned memory for HBM
  targets, the target's own storage for CPU targets), so most reads perform
  no intermediate allocation;
* per-stage timings are recorded (``PendingIOWork.stats``) for
  time-to-unblock and GB/s reporting.
"""

from __future__ import annotations

import asyncio
import functools
import logging
import os
import socket
import threading
import time
from collections import deque
from concurrent.futures import ThreadPoolExecutor
from typing import Any, Callable, Dict, List, Optional

import psutil

from .. import knobs
from ..ops import checksum
from ..io_types import (ReadIO, ReadReq, StagedBuffer, StoragePlugin, WriteIO, WriteReq, as_staged,
                        run_sync)
from ..utils.tracing import timeline
from . import native_drain  # (on first use it cost the first async_take's unblock ~1 ms)

logger = logging.getLogger(__name__)

_budget_cache: Dict[tuple, int] = {}

# Worker pools outlive a take: a pipeline that finished cleanly hands its
# pool back instead of joining its threads, and the next take reuses them.
_idle_pools: Dict[tuple, List[ThreadPoolExecutor]] = {}
_pool_lock = threading.Lock()
_MAX_IDLE_POOLS = 2


def _acquire_pool(kind: str, n: int, rank: int) -> ThreadPoolExecutor:
    key = (os.getpid(), kind, n)
    with _pool_lock:
        lst = _idle_pools.get(key)
        if lst:
            return lst.pop()
    ex = ThreadPoolExecutor(max_workers=n, thread_name_prefix=f"hipsnapshot-{kind}-{rank}")
    ex._hs_key = key  # type: ignore[attr-defined]
    return ex


def _release_pool(ex: ThreadPoolExecutor, reusable: bool) -> None:
    """Give back a pool from ``_acquire_pool``.  ``reusable`` only when every
    task submitted to it has finished (a clean pipeline end); otherwise the
    pool is shut down as before."""
    key = getattr(ex, "_hs_key", None)
    if reusable and key is not None and key[0] == os.getpid():
        with _pool_lock:
            lst = _idle_pools.setdefault(key, [])
            if len(lst) < _MAX_IDLE_POOLS:
                lst.append(ex)
                return
    ex.shutdown(wait=reusable)


def get_local_world_size(pg) -> int:
    solo = getattr(pg, "solo", None)
    if pg is None or (solo() if solo is not None else pg.get_world_size() == 1):
        return 1
    names = [None] * pg.get_world_size()
    pg.all_gather_object(names, socket.gethostname())
    return names.count(socket.gethostname())


def get_process_memory_budget_bytes(pg=None) -> int:
    """min(0.6 * available / local_world_size, 32 GiB), env-overridable.

    Cached per process group so restore does not all-gather hostnames once
    per stateful (reference quirk)."""
    override = knobs.get_memory_budget_override()
    if override is not None:
        logger.info(f"Manually set process memory budget to {override} bytes.")
        return override
    key = (id(getattr(pg, "pg", pg)), pg.get_world_size() if pg is not None else 1)
    if key in _budget_cache:
        return _budget_cache[key]
    local_ws = get_local_world_size(pg)
    avail = psutil.virtual_memory().available
    budget = int(min(avail * 0.6 / max(local_ws, 1), knobs.MAX_PER_RANK_MEMORY_BUDGET_BYTES))
    _budget_cache[key] = budget
    return budget


_aux = {"pid": None, "pool": None}
_aux_lock = threading.Lock()


def aux_pool() -> ThreadPoolExecutor:
    """Process-wide pool for short host-side helpers of the pipelines (host
    hashing, pinned read destinations).  An event loop's default executor
    would do, but every take / restore runs its own loop, so its threads
    were started and joined again on every call."""
    pool = _aux["pool"]
    if pool is None or _aux["pid"] != os.getpid():
        with _aux_lock:
            if _aux["pool"] is None or _aux["pid"] != os.getpid():
                _aux["pool"] = ThreadPoolExecutor(max_workers=8,
                                                  thread_name_prefix="hipsnapshot-aux")
                _aux["pid"] = os.getpid()
            pool = _aux["pool"]
    return pool


async def _wait_ready(buf: StagedBuffer) -> None:
    """Wait (off the loop) for ``buf``'s asynchronous copy; a cancellation
    waits for the copy anyway, then re-raises (the buffer must not be
    released while the engine writes into it)."""
    fut = asyncio.get_running_loop().run_in_executor(aux_pool(), buf.ready)
    cancelled = False
    while True:
        try:
            await asyncio.shield(fut)
            break
        except asyncio.CancelledError:
            if fut.done():
                break
            cancelled = True
    buf.ready = None
    if cancelled:
        raise asyncio.CancelledError()
    fut.result()


class PipelineStats:
    def __init__(self) -> None:
        self.t_start = time.monotonic()
        self.t_staged: Optional[float] = None
        self.t_done: Optional[float] = None
        self.bytes_staged = 0
        self.bytes_written = 0
        self.n_reqs = 0
        self.checksums: Dict[str, int] = {}  # blob path -> hs64 (knobs.checksum_enabled)

    def as_dict(self) -> dict:
        d = {"n_reqs": self.n_reqs, "bytes": self.bytes_written}
        if self.t_staged is not None:
            d["stage_s"] = self.t_staged - self.t_start
        if self.t_done is not None:
            d["total_s"] = self.t_done - self.t_start
            if d["total_s"] > 0:
                d["GBps"] = self.bytes_written / d["total_s"] / 1e9
        return d


class MemoryGate:
    """Host-memory budget of one take, shared by every pipeline it runs.

    A request is admitted when its cost fits, or when nothing at all is held
    (so one oversized request still makes progress).  Releases wake every
    pipeline waiting on the gate, so an async take's deferred pipeline (see
    ``DeferredIOWork``) only stages what the first pipeline's in-flight
    writes have left of the budget."""

    def __init__(self, limit: int) -> None:
        self.limit = limit
        self.in_use = 0
        self._wakes: set = set()
        # staging worker threads admit under this condition (thread-driven
        # pipelines); releases happen on the event-loop thread
        self.cond = threading.Condition()

    def try_admit(self, cost: int) -> bool:
        with self.cond:
            if self.in_use + cost > self.limit and self.in_use > 0:
                return False
            self.in_use += cost
            return True

    def release(self, cost: int) -> None:
        with self.cond:
            self.in_use -= cost
            self.cond.notify_all()
        for ev in self._wakes:
            ev.set()

    def subscribe(self, ev: asyncio.Event) -> None:
        self._wakes.add(ev)

    def unsubscribe(self, ev: asyncio.Event) -> None:
        self._wakes.discard(ev)


class PendingIOWork:
    """Storage writes still in flight after staging completed."""

    def __init__(self, io_tasks: set, executor: ThreadPoolExecutor, stats: PipelineStats,
                 failure: List[BaseException], gate: Optional[MemoryGate] = None) -> None:
        self.io_tasks = io_tasks
        self.executor = executor
        self.stats = stats
        self._failure = failure
        self.gate = gate

    async def complete(self) -> None:
        done = False
        try:
            if self.io_tasks:
                await asyncio.gather(*self.io_tasks, return_exceptions=True)
            done = True
        finally:
            if self.executor is None:
                pass  # nothing was staged (empty_write_work)
            elif done:
                _release_pool(self.executor, reusable=True)
            else:  # cancelled while waiting: tasks may still run
                self.executor.shutdown(wait=True)
            self.stats.t_done = time.monotonic()
        if self._failure:
            raise self._failure[0]
        st = self.stats
        logger.info(f"Completed writing {st.bytes_written / 1e9:.3f} GB in "
                    f"{st.t_done - st.t_start:.3f}s")

    def sync_complete(self, event_loop: asyncio.AbstractEventLoop) -> None:
        run_sync(event_loop, self.complete())


def empty_write_work(memory_budget_bytes: int) -> PendingIOWork:
    """The ``PendingIOWork`` of an empty request list, without a pipeline (an
    async take whose every write was frozen in HBM stages nothing before it
    returns; starting the pipeline for nothing cost ~0.3 ms of its unblock)."""
    stats = PipelineStats()
    stats.n_reqs = 0
    return PendingIOWork(set(), None, stats, [], MemoryGate(memory_budget_bytes))


async def execute_write_reqs(write_reqs: List[WriteReq], storage: StoragePlugin,
                             memory_budget_bytes: int, rank: int,
                             stage_threads: Optional[int] = None,
                             io_concurrency: Optional[int] = None,
                             gate: Optional[MemoryGate] = None,
                             background: bool = False,
                             wait_copies: bool = False,
                             first_staged: Optional[threading.Event] = None) -> PendingIOWork:
    """``background``: the pipeline runs while the caller keeps using the GPU
    (async-take drain); its staging kernels get a capped grid.
    ``wait_copies``: return only once every staged buffer's asynchronous
    device copy (and on-device hash) has finished, i.e. nothing reads the
    source tensors any more (async take from live, un-frozen tensors).
    ``first_staged``: set once the first buffer is staged (its copy is
    queued), so helper work that needs the GIL can wait for it."""
    stage_threads = stage_threads or knobs.get_stage_threads()
    io_concurrency = io_concurrency or knobs.get_io_threads()
    executor = _acquire_pool("stage_bg" if background else "stage", stage_threads, rank)
    stats = PipelineStats()
    stats.n_reqs = len(write_reqs)
    failure: List[BaseException] = []
    pending = deque(write_reqs)
    gate = gate if gate is not None else MemoryGate(memory_budget_bytes)
    staging: Dict[asyncio.Task, tuple] = {}
    io_tasks: set = set()
    io_sem = asyncio.Semaphore(io_concurrency)
    wake = asyncio.Event()
    gate.subscribe(wake)
    from ..utils.tracing import WriteReporter

    reporter = WriteReporter(rank, memory_budget_bytes)

    want_sums = knobs.checksum_enabled()
    copies: List[asyncio.Future] = []  # waits for in-flight device -> host copies

    def _staged(wr: WriteReq, buf: StagedBuffer, cost: int, t_s: float) -> None:
        timeline.add("stage", "stage", t_s, time.perf_counter(), path=wr.path,
                     bytes=buf.nbytes)
        if first_staged is not None:
            first_staged.set()
        stats.bytes_staged += buf.nbytes
        copy = None
        if buf.ready is not None:
            # the blob's device -> host copy is still on the SDMA engine
            copy = asyncio.ensure_future(_wait_ready(buf))
            if wait_copies:
                copies.append(copy)
        io_tasks.add(asyncio.ensure_future(_write(wr, buf, cost, copy)))
        reporter.maybe_report(len(pending), 0, len(io_tasks), gate.in_use, stats.bytes_written)

    async def _copies_done() -> None:
        """``wait_copies``: block until no copy reads a source tensor."""
        res = await asyncio.gather(*copies, return_exceptions=True)
        copies.clear()
        errs = [r for r in res if isinstance(r, BaseException)]
        if errs:
            await asyncio.gather(*io_tasks, return_exceptions=True)
            raise errs[0]

    async def _write(wr: WriteReq, buf: StagedBuffer, cost: int,
                     copy: Optional[asyncio.Future]) -> None:
        hashing = None
        try:
            if copy is not None:
                await asyncio.shield(copy)
            if want_sums and buf.checksum is None:
                # host-staged blob: hash it on the host while it is written
                # (both only read the buffer; the GPU stager hashed the rest)
                # (2 threads per blob: several blobs hash at once on the pool)
                hashing = asyncio.get_running_loop().run_in_executor(
                    aux_pool(), checksum.hs64_host, buf.addr, buf.nbytes, 2)
            async with io_sem:
                if failure:  # the snapshot is failing: do not start more writes
                    return
                t_w = time.perf_counter()
                await storage.write(WriteIO(path=wr.path, buf=buf.view, addr=buf.addr,
                                            numa_node=buf.numa_node))
                timeline.add("write", "io", t_w, time.perf_counter(), path=wr.path,
                             bytes=buf.nbytes)
            stats.bytes_written += buf.nbytes
            if want_sums:
                stats.checksums[wr.path] = (await hashing) if hashing is not None \
                    else buf.checksum
        except BaseException as e:  # noqa: BLE001
            failure.append(e)
            raise
        finally:
            if hashing is not None and not hashing.done():
                # the hash still reads the buffer: it must finish before release
                await asyncio.gather(asyncio.shield(hashing), return_exceptions=True)
            if copy is not None and not copy.done():
                await asyncio.wait([copy])  # (a cancelled wait leaves the copy running)
            if buf.ready is not None:
                # an early exit (failure, cancellation): the copy may still be
                # writing into the buffer
                await asyncio.gather(_wait_ready(buf), return_exceptions=True)
            buf.release()
            gate.release(cost)
            wake.set()

    if pending and knobs.thread_staging_enabled() and \
            all(getattr(wr.buffer_stager, "thread_staging", False) for wr in pending):
        try:
            await _stage_on_threads(pending, stage_threads, executor, gate, failure,
                                    lambda wr, buf, cost, t_s: _staged(wr, buf, cost, t_s))
        except BaseException:
            gate.unsubscribe(wake)
            # writes already issued keep their buffers until the engine is done
            await asyncio.gather(*io_tasks, return_exceptions=True)
            executor.shutdown(wait=False)
            raise
        gate.unsubscribe(wake)
        if failure:
            await asyncio.gather(*io_tasks, return_exceptions=True)
            executor.shutdown(wait=True)
            raise failure[0]
        if wait_copies:
            await _copies_done()
        stats.t_staged = time.monotonic()
        logger.debug(f"Rank {rank} completed staging in {stats.t_staged - stats.t_start:.3f}s")
        return PendingIOWork(io_tasks, executor, stats, failure, gate)

    try:
        while pending or staging:
            while pending and len(staging) < stage_threads and not failure:
                cost = pending[0].buffer_stager.get_staging_cost_bytes()
                if not gate.try_admit(cost):
                    break
                wr = pending.popleft()
                task = asyncio.ensure_future(wr.buffer_stager.stage_buffer(executor))
                staging[task] = (wr, cost, time.perf_counter())
            if failure:
                break
            waiters = set(staging)
            wake.clear()
            waiter = asyncio.ensure_future(wake.wait())
            done, _ = await asyncio.wait(waiters | {waiter}, return_when=asyncio.FIRST_COMPLETED)
            if not waiter.done():
                waiter.cancel()
            reporter.maybe_report(len(pending), len(staging), len(io_tasks), gate.in_use,
                                  stats.bytes_written)
            for task in done:
                if task is waiter:
                    continue
                wr, cost, t_s = staging.pop(task)
                exc = task.exception()
                if exc is not None:
                    gate.release(cost)
                    failure.append(exc)
                    continue
                _staged(wr, as_staged(task.result()), cost, t_s)
        if failure:
            # stage tasks in flight are NOT cancelled: their executor jobs
            # would still submit copies whose buffers nobody waits for (a
            # leaked DMA slot, a pinned block the engine still writes into).
            # Let them finish, then wait for each copy and free its buffer.
            res = await asyncio.gather(*staging, return_exceptions=True)
            for (wr, cost, _t), r in zip(staging.values(), res):
                if not isinstance(r, BaseException):
                    buf = as_staged(r)
                    if buf.ready is not None:
                        await asyncio.gather(_wait_ready(buf), return_exceptions=True)
                    buf.release()
                gate.release(cost)
            staging.clear()
            # writes already handed to the I/O engine are NOT cancelled: their
            # pinned buffers may only go back to the pool once the engine is
            # done reading them (queued ones return without writing)
            await asyncio.gather(*io_tasks, return_exceptions=True)
            executor.shutdown(wait=True)
            raise failure[0]
    except BaseException:
        executor.shutdown(wait=False)
        raise
    finally:
        # staging is over: later wake-ups (write completions) are not needed
        gate.unsubscribe(wake)
    if wait_copies:
        await _copies_done()
    stats.t_staged = time.monotonic()
    logger.debug(f"Rank {rank} completed staging in {stats.t_staged - stats.t_start:.3f}s")
    return PendingIOWork(io_tasks, executor, stats, failure, gate)


async def _stage_on_threads(pending: deque, nthreads: int, executor: ThreadPoolExecutor,
                            gate: MemoryGate, failure: List[BaseException], on_staged) -> None:
    """Stage ``pending`` on ``nthreads`` long-running executor workers.

    Each worker takes the next request the memory gate admits, stages it
    (``stage_buffer_sync``: D2H / encode / gather on the worker's own copy
    stream) and goes straight on to the next one; only the hand-off of the
    staged buffer to the writer goes through the event loop.  With one
    round trip through the loop per request instead, the DMA engine sat idle
    for 0.7-1.4 ms between blobs whenever all workers waited for the loop
    (17 % of a take of one rank's 8-GPU share, profiles/rank_share/)."""
    loop = asyncio.get_running_loop()
    cond = gate.cond

    # The first blob is staged alone: with every worker starting at once they
    # share the GIL and the GPU's encoders, and the first DMA -- the start of
    # the PCIe-bound part of the take -- waited ~0.6 ms longer.  The others
    # start once it is handed off (or after 3 ms).
    head = threading.Event()

    head_alone = knobs.TUNING.stage_head_alone

    def worker(i: int) -> None:
        if i and head_alone:
            head.wait(0.003)
        while True:
            t_w = time.perf_counter()
            with cond:
                while True:
                    if failure or not pending:
                        return
                    wr = pending[0]
                    cost = wr.buffer_stager.get_staging_cost_bytes()
                    if gate.try_admit(cost):  # re-enters cond (an RLock)
                        pending.popleft()
                        break
                    cond.wait(0.05)
            t_s = time.perf_counter()
            timeline.add("admit", "stage", t_w, t_s)
            try:
                buf = as_staged(wr.buffer_stager.stage_buffer_sync())
            except BaseException as e:  # noqa: BLE001 - reported by the caller
                head.set()
                with cond:
                    failure.append(e)
                    cond.notify_all()
                loop.call_soon_threadsafe(gate.release, cost)
                return
            head.set()
            try:
                loop.call_soon_threadsafe(on_staged, wr, buf, cost, t_s)
            except RuntimeError:  # the loop is gone (the take was abandoned)
                from .staging import wait_ready

                try:
                    wait_ready(buf)  # the engine may still write into it
                finally:
                    buf.release()
                return

    futs = [executor.submit(worker, i) for i in range(max(1, min(nthreads, len(pending))))]
    try:
        await asyncio.gather(*(asyncio.wrap_future(f) for f in futs))
    except BaseException:
        with cond:  # stop the workers at their next request
            failure.append(asyncio.CancelledError())
            cond.notify_all()
        raise


class DeferredIOWork:
    """``PendingIOWork`` for an async take whose device state was frozen in
    HBM: the immediate part (host tensors, already copied) is staged before
    ``async_take`` returns; the deferred part (HBM arena -> pinned -> storage)
    runs its whole pipeline in the background commit thread.  Both pipelines
    draw on ONE ``MemoryGate``, so host memory stays within the per-rank
    budget while the first pipeline's staged buffers are still being written."""

    def __init__(self, first: PendingIOWork, deferred: List[WriteReq], storage: StoragePlugin,
                 memory_budget_bytes: int, rank: int) -> None:
        self.first = first
        self.deferred = deferred
        self.storage = storage
        self.budget = memory_budget_bytes
        self.rank = rank
        self.stats = first.stats
        self._second: Optional[PendingIOWork] = None
        self.booster = native_drain.Booster()  # PendingSnapshot.wait() -> all drain writers

    def boost(self) -> None:
        self.booster.boost()

    async def complete(self) -> None:
        native_reqs, py_reqs = native_drain.split(self.deferred, self.storage)
        native_out: Dict[str, Any] = {}
        native_fut: List[Any] = []  # the native drain's executor future

        async def run_deferred() -> None:
            if not py_reqs:
                return
            p = await execute_write_reqs(py_reqs, self.storage, self.budget, self.rank,
                                         gate=self.first.gate, background=True)
            self._second = p
            await p.complete()

        async def run_native() -> None:
            # one native call for every raw frozen blob: no Python (and no
            # GIL) between the arena and the files while the trainer runs
            if native_reqs:
                cf = aux_pool().submit(native_drain.drain, native_reqs, self.storage,
                                       self.booster)
                native_fut.append(cf)
                native_out["sums"], native_out["bytes"] = await asyncio.wrap_future(cf)

        try:
            res = await asyncio.gather(self.first.complete(), run_deferred(), run_native(),
                                       return_exceptions=True)
        finally:
            # a cancelled wait does not stop the native drain thread: it
            # still reads the arena, which is only free once it returned
            for cf in native_fut:
                try:
                    cf.result()
                except BaseException:  # noqa: BLE001 -- reported through ``res``
                    pass
            # every reader of the frozen arena is done: a kept arena is free
            from .hbm_staging import arena_done

            arena_done({id(a): a for a in (getattr(wr.buffer_stager, "frozen_region",
                                                   (None,))[0] for wr in self.deferred)
                        if a is not None}.values())
        if self._second is not None:
            self.stats.bytes_written += self._second.stats.bytes_written
            self.stats.n_reqs += self._second.stats.n_reqs
            self.stats.checksums.update(self._second.stats.checksums)
        if "bytes" in native_out:
            self.stats.bytes_written += native_out["bytes"]
            self.stats.n_reqs += len(native_reqs)
            self.stats.checksums.update(native_out["sums"])
        self.stats.t_done = time.monotonic()
        for r in res:
            if isinstance(r, BaseException):
                raise r

    def sync_complete(self, event_loop: asyncio.AbstractEventLoop) -> None:
        run_sync(event_loop, self.complete())


def sync_execute_write_reqs(write_reqs: List[WriteReq], storage: StoragePlugin,
                            memory_budget_bytes: int, rank: int,
                            event_loop: asyncio.AbstractEventLoop,
                            wait_copies: bool = False,
                            first_staged: Optional[threading.Event] = None) -> PendingIOWork:
    try:
        return run_sync(event_loop,
            execute_write_reqs(write_reqs, storage, memory_budget_bytes, rank,
                               wait_copies=wait_copies, first_staged=first_staged))
    finally:
        if first_staged is not None:
            first_staged.set()


def _expected_read_bytes(rr: ReadReq) -> Optional[int]:
    if rr.byte_range is not None:
        return rr.byte_range[1] - rr.byte_range[0]
    c = rr.buffer_consumer
    entry = getattr(c, "entry", None)
    if entry is not None and getattr(entry, "type", None) == "Tensor":
        if entry.serializer == "buffer_protocol":
            from ..io.tensor import tensor_nbytes_from_entry

            return tensor_nbytes_from_entry(entry)
        if getattr(entry, "quant", None):
            return int(entry.quant["total_bytes"])
    return None


async def execute_read_reqs(read_reqs: List[ReadReq], storage: StoragePlugin,
                            memory_budget_bytes: int, rank: int,
                            consume_threads: Optional[int] = None,
                            io_concurrency: Optional[int] = None,
                            native_jobs: Optional[dict] = None,
                            verifier=None) -> PipelineStats:
    """Run ``read_reqs``.  Reads whose bytes all land in HBM go to one native
    job per device (engine/native_restore.py) beside the Python pipeline for
    the rest; ``native_jobs``: a split the caller already made
    (``native_restore.split``), ``read_reqs`` then being the Python part.
    ``verifier`` (engine/blob_verify.py): check every blob read against the
    take's checksums."""
    from . import native_restore

    if native_jobs is None:
        native_jobs, read_reqs = native_restore.split(read_reqs, storage, memory_budget_bytes)
    native_fut = None
    py_budget = memory_budget_bytes
    if native_jobs:
        native_fut = asyncio.get_running_loop().run_in_executor(
            aux_pool(), native_restore.run, native_jobs, memory_budget_bytes, verifier)
        # the job's pinned slots count against the same host budget as the
        # Python part running beside it (a mixed restore pinned
        # ~1.5x the budget); one oversized read still runs (MemoryGate)
        py_budget = max(1, memory_budget_bytes - len(native_jobs) *
                        native_restore.pinned_bytes(memory_budget_bytes))
    try:
        stats = await _execute_python_reads(read_reqs, storage, py_budget, rank,
                                            consume_threads, io_concurrency, verifier) \
            if read_reqs or not native_jobs else PipelineStats()
    finally:
        if native_fut is not None:
            # never leave the job running: it writes into the destinations
            native_bytes = await asyncio.gather(native_fut, return_exceptions=True)
    if native_fut is not None:
        if isinstance(native_bytes[0], BaseException):
            raise native_bytes[0]
        stats.bytes_written += native_bytes[0]
        stats.n_reqs += sum(len(v) for v in native_jobs.values())
    if verifier is not None:
        await verifier.finish(storage, memory_budget_bytes)
    return stats


async def _execute_python_reads(read_reqs: List[ReadReq], storage: StoragePlugin,
                                memory_budget_bytes: int, rank: int,
                                consume_threads: Optional[int] = None,
                                io_concurrency: Optional[int] = None,
                                verifier=None) -> PipelineStats:
    consume_threads = consume_threads or knobs.get_stage_threads()
    io_concurrency = io_concurrency or knobs.get_io_threads()
    # reads are split across all I/O workers by the native engine, so a few
    # whole-blob reads in flight saturate it; more would only pin more memory
    max_inflight = knobs.get_read_inflight()
    executor = _acquire_pool("consume", consume_threads, rank)
    stats = PipelineStats()
    stats.n_reqs = len(read_reqs)
    pending = deque(read_reqs)
    in_use = [0]
    inflight: set = set()
    io_sem = asyncio.Semaphore(io_concurrency)
    # set on the first failed read: queued reads then return without reading.
    # Reads already handed to storage are NOT cancelled -- the plugin (e.g.
    # the native engine) may still be writing into their pinned destination,
    # which must not go back to the pool before that write has finished.
    failing: List[BaseException] = []

    async def _one_compressed(rr: ReadReq) -> None:
        from ..ops import codec as hsz
        from ..io_types import CompressedSpan, SpanTail

        info = rr.codec
        logical = int(info["blob_bytes"])
        nf = hsz.n_frames_for(logical, int(info["frame_bytes"]))
        dest = None
        tail = None
        rest_task = None
        try:
            async with io_sem:
                if failing:
                    return
                t_r = time.perf_counter()
                whole = rr.byte_range is None or tuple(rr.byte_range) == (0, logical)
                stored = await storage.size(rr.path) if whole else None
                if stored is not None:
                    # whole blob: header + frames without a header round trip
                    # (reads enter the engine queue in request order).  A large
                    # blob is read as a head and the rest: the consumer moves
                    # the head's frames to the GPU while the rest arrives.
                    t_d = time.perf_counter()
                    full = await asyncio.get_running_loop().run_in_executor(
                        aux_pool(), rr.buffer_consumer.get_compressed_read_dest, stored)
                    timeline.add("read_dest", "io", t_d, time.perf_counter(), bytes=stored)
                    if full is None:
                        full = as_staged(bytearray(max(stored, 1)))
                    dest = full
                    head_n = knobs.get_read_head_bytes()
                    split = 0 < head_n and 2 * head_n <= stored \
                        and hsz.payload_start(nf) <= head_n
                    head_end = head_n if split else stored
                    head_read = storage.read(ReadIO(
                        path=rr.path, byte_range=(0, head_end),
                        dest=StagedBuffer(full.view[:head_end], full.addr)))
                    if split:
                        rest_task = asyncio.ensure_future(storage.read(ReadIO(
                            path=rr.path, byte_range=(head_end, stored),
                            dest=StagedBuffer(full.view[head_end:], full.addr + head_end))))
                    await head_read
                    header = hsz.parse_header(full.view[:hsz.payload_start(nf)])
                    hsz.validate_offsets(header, stored)
                    lo, hi = 0, header.logical_size
                    first, last = 0, header.n_frames
                    c_lo, c_hi = header.offsets[0], header.offsets[-1]
                    dest = StagedBuffer(full.view[c_lo:c_hi], full.addr + c_lo,
                                        release=full.release, keepalive=full)
                    if rest_task is not None:
                        tail = SpanTail(max(head_end - c_lo, 0))
                        rest_task.add_done_callback(
                            lambda t, tl=tail: tl.arrived(
                                None if t.cancelled() or t.exception() is None
                                else t.exception()))
                else:
                    if verifier is not None:
                        verifier.note_partial(rr.path)
                    head_io = ReadIO(path=rr.path, byte_range=(0, hsz.payload_start(nf)))
                    await storage.read(head_io)
                    header = hsz.parse_header(head_io.data())
                    lo, hi = rr.byte_range if rr.byte_range is not None \
                        else (0, header.logical_size)
                    first, last = header.frames_covering(lo, hi)
                    c_lo, c_hi = header.offsets[first], header.offsets[last]
                    hsz.validate_offsets(header, header.offsets[-1])
                    dest = await asyncio.get_running_loop().run_in_executor(
                        aux_pool(), rr.buffer_consumer.get_compressed_read_dest, c_hi - c_lo)
                    if dest is None:
                        dest = as_staged(bytearray(max(c_hi - c_lo, 1)))
                    body_io = ReadIO(path=rr.path, byte_range=(c_lo, c_hi), dest=dest)
                    if c_hi > c_lo:
                        await storage.read(body_io)
                t_c = time.perf_counter()
        except BaseException:
            if rest_task is not None:
                # the engine may still be filling the rest: not before it is done
                await asyncio.gather(rest_task, return_exceptions=True)
            if dest is not None:
                dest.release()
            raise
        span = CompressedSpan(dest, header, first, last, lo, hi, tail=tail)
        timeline.add("read", "io", t_r, t_c, path=rr.path, bytes=c_hi - c_lo, logical=hi - lo)
        stats.bytes_written += hi - lo
        try:
            await rr.buffer_consumer.consume_buffer(span, executor)
            if rest_task is not None:
                await asyncio.gather(rest_task, return_exceptions=True)
            if verifier is not None and stored is not None and (
                    rest_task is None or (not rest_task.cancelled()
                                          and rest_task.exception() is None)):
                # the whole stored blob sits in ``full``: hash it before the
                # buffer goes back to the pool
                await asyncio.get_running_loop().run_in_executor(
                    aux_pool(), verifier.check_host, rr.path, full.addr, stored)
        finally:
            if rest_task is not None:
                await asyncio.gather(rest_task, return_exceptions=True)
            span.release()
        if rest_task is not None and not rest_task.cancelled() \
                and rest_task.exception() is not None:
            raise rest_task.exception()
        timeline.add("consume", "stage", t_c, time.perf_counter(), path=rr.path, bytes=hi - lo)

    async def _one(rr: ReadReq, cost: int) -> None:
        if rr.codec is not None:
            try:
                await _one_compressed(rr)
            finally:
                in_use[0] -= cost
            return
        dest = None
        try:
            if failing:
                return
            nbytes = _expected_read_bytes(rr)
            if nbytes is not None:
                # pinned-pool misses cost a hipHostMalloc: keep them off the
                # event loop so completions of earlier reads are not delayed
                dest = await asyncio.get_running_loop().run_in_executor(
                    aux_pool(), rr.buffer_consumer.get_read_dest, nbytes)
            read_io = ReadIO(path=rr.path, byte_range=rr.byte_range, dest=dest)
            async with io_sem:
                if failing:
                    return
                t_r = time.perf_counter()
                await storage.read(read_io)
                t_c = time.perf_counter()
            data = read_io.data()
            nb = memoryview(data).nbytes
            timeline.add("read", "io", t_r, t_c, path=rr.path, bytes=nb)
            if verifier is not None:
                await _verify_raw_read(verifier, storage, rr, data, nb)
            stats.bytes_written += nb
            await rr.buffer_consumer.consume_buffer(dest if dest is not None else data,
                                                    executor)
            timeline.add("consume", "stage", t_c, time.perf_counter(), path=rr.path, bytes=nb)
        finally:
            if dest is not None:
                dest.release()
            in_use[0] -= cost

    from . import staging

    clean = False
    try:
        # consumers may leave their decode / scatter kernels running: the
        # scope waits for them (and raises corrupt frames) at its end
        with staging.deferred_device_work():
            while pending or inflight:
                while pending and len(inflight) < max_inflight:
                    cost = pending[0].buffer_consumer.get_consuming_cost_bytes()
                    if in_use[0] + cost > memory_budget_bytes and inflight:
                        break
                    rr = pending.popleft()
                    in_use[0] += cost
                    inflight.add(asyncio.ensure_future(_one(rr, cost)))
                done, inflight = await asyncio.wait(inflight,
                                                    return_when=asyncio.FIRST_COMPLETED)
                inflight = set(inflight)
                for t in done:
                    if t.exception() is not None:
                        failing.append(t.exception())
                        # drain, do not cancel: see ``failing`` above
                        await asyncio.gather(*inflight, return_exceptions=True)
                        raise t.exception()
        clean = True
    finally:
        if clean:
            _release_pool(executor, reusable=True)
        else:
            executor.shutdown(wait=True)
    stats.t_done = time.monotonic()
    logger.debug(f"Rank {rank} read {stats.bytes_written / 1e9:.3f} GB in "
                 f"{stats.t_done - stats.t_start:.3f}s")
    return stats


async def _verify_raw_read(verifier, storage: StoragePlugin, rr: ReadReq, data, nb: int) -> None:
    from ..io_types import buffer_address
    from .blob_verify import whole_read

    stored = None
    if rr.byte_range is not None and rr.byte_range[0] == 0:
        stored = await storage.size(rr.path)
    if whole_read(rr, stored):
        mv = memoryview(data).cast("B")
        await asyncio.get_running_loop().run_in_executor(
            aux_pool(), verifier.check_host, rr.path, buffer_address(mv) if nb else 0, nb)
    else:
        verifier.note_partial(rr.path)


def sync_execute_read_reqs(read_reqs: List[ReadReq], storage: StoragePlugin,
                           memory_budget_bytes: int, rank: int,
                           event_loop: asyncio.AbstractEventLoop,
                           native_jobs: Optional[dict] = None, verifier=None) -> PipelineStats:
    return run_sync(event_loop,
        execute_read_reqs(read_reqs, storage, memory_budget_bytes, rank,
                          native_jobs=native_jobs, verifier=verifier))


def hostname() -> str:
    return socket.gethostname()


def cpu_count() -> int:
    return os.cpu_count() or 1
