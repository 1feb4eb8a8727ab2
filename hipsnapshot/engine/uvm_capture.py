"""Async takes of host-resident UVM tables: capture on the CPU, gate the GPU.

A managed (UVM) embedding table whose pages live in host DRAM (TorchRec's
``uvm_tensor`` tables larger than HBM; ``ops/uvm.py``) cannot be aliased by
an ``async_take``: the trainer keeps updating it.  The HBM freeze
(``hbm_staging``) copied it into the arena with a kernel on the trainer's
stream, reading every byte over PCIe (55 GB/s).  That is ~150 ms of
trainer-stream stall per 8 GB, and the drain then sends the bytes back over
PCIe.

Here the tables are captured by CPU threads on the pages' NUMA node into
pinned host blocks: 160-196 GB/s on the box (``scripts/probes/
uvm_capture_probe.py``, ``profiles/r6/uvmcap/``).  Meanwhile the trainer's
stream waits on a gate (``hipStreamWaitValue32`` on a host word,
``csrc/hsgpu.hip``), armed right behind the work that may still write the
tables:

    trainer stream:  [queued kernels] -> event E -> [gate >= v] -> [later work]
    capture thread:  wait E -> copy table 0, 1, ... -> release v (always)

``async_take`` returns at once.  The drain writes each table from its block
as soon as that table is copied.  No PCIe crossing, no HBM arena.

Reference: `/root/reference/torchsnapshot/io_preparers/tensor.py:257-260`
(UVM tensors go through ``uvm_to_cpu`` before an async take returns).
"""

from __future__ import annotations

import logging
import threading
import time
from typing import Dict, List, Optional

import torch

from .. import knobs
from ..io_types import StagedBuffer, WriteReq
from ..ops import native
from ..utils.tracing import timeline

logger = logging.getLogger(__name__)


_resolved: tuple = ()


def _deps() -> tuple:
    """(TensorBufferStager, SER.BUFFER_PROTOCOL, staging), imported once: a
    function-level import per write request cost ~0.5 ms of unblock time per
    take of the 8B model (291 leaves, ``profiles/r6/cold/``)."""
    global _resolved
    if not _resolved:
        from ..format.serialization import SER
        from ..io.tensor import TensorBufferStager
        from . import staging

        _resolved = (TensorBufferStager, SER.BUFFER_PROTOCOL, staging)
    return _resolved


def _eligible(wr: WriteReq, deps: tuple):
    """The contiguous host-resident managed tensor ``wr`` saves as raw bytes,
    or None."""
    stager_cls, buffer_protocol, staging = deps
    st = wr.buffer_stager
    if type(st) is not stager_cls or st.codec is not None \
            or st._tensor_prepare_func is not None or st.entry.serializer != buffer_protocol:
        return None
    t = st.tensor
    if not t.is_cuda or not t.is_contiguous() or t.numel() == 0:
        return None
    # a tensor is managed or not for life: the pointer query (a HIP call)
    # runs once per stager, not on every async take's unblock path
    ptr = t.data_ptr()
    if st.__dict__.get("_not_managed") == ptr:
        return None
    if not staging._is_managed(t):
        st._not_managed = ptr
        return None
    if not staging.host_resident_managed(t):
        return None
    return t


class Capture:
    """One async take's CPU capture of host-resident UVM tables on a device."""

    def __init__(self, dev: int, items: List[tuple]) -> None:
        self.dev = dev
        self.items = items  # [(stager, tensor, nbytes)]
        self.blocks: List[Optional[native.PinnedBuffer]] = [None] * len(items)
        self.done = [threading.Event() for _ in items]
        self.error: Optional[BaseException] = None
        self.value: Optional[int] = None
        self.stats: Dict[str, object] = {}
        self._thread: Optional[threading.Thread] = None
        self._t_start = self._t_blocks = 0.0

    # -- start (async_take's thread) -------------------------------------------

    def start(self) -> None:
        """Allocate the blocks, arm the gate on every producer stream, start
        the copy thread.  Raises (nothing armed) if a block cannot be had."""
        from ..utils.affinity import pages_node

        self._t_start = time.perf_counter()
        for i, (_st, t, n) in enumerate(self.items):
            # on the table's own node: the copy and the later write stay local
            # (blocks first touched elsewhere made the copy 60-200 GB/s from
            # one process to the next, profiles/r6/uvmcap/)
            self.blocks[i] = native.PinnedBuffer(n, pages_node(t.data_ptr(), n))
        self._t_blocks = time.perf_counter()
        producers = sorted({st.producer if st.producer is not None
                            else int(torch.cuda.current_stream(self.dev).cuda_stream)
                            for st, _t, _n in self.items})
        events = []
        for p in producers:
            ev = torch.cuda.Event()
            ev.record(torch.cuda.ExternalStream(p, device=f"cuda:{self.dev}") if p
                      else torch.cuda.default_stream(self.dev))
            events.append(ev)
        armed: List[int] = []
        try:
            for p in producers:
                armed.append(native.gate_arm(self.dev, p))
            self.value = max(armed)
            self._thread = threading.Thread(target=self._run, args=(events,),
                                            name="hs-uvm-capture", daemon=True)
            self._thread.start()
        except BaseException:
            for v in armed:
                native.gate_release(self.dev, v)
            self.release_blocks()
            raise

    # -- the copy thread ------------------------------------------------------------

    def _run(self, events) -> None:
        from ..utils.affinity import node_cpus, pages_node

        t0 = time.perf_counter()
        try:
            for ev in events:  # the trainer's writes queued before the take
                ev.synchronize()
            t1 = time.perf_counter()
            lib = native.hsio()
            nthreads = max(1, int(knobs.TUNING.uvm_capture_threads))
            # tables in parallel, each split over its share of the threads:
            # sequential tables at 16 threads each copied at ~100 GB/s, this
            # at 160-196 (scripts/probes/uvm_capture_probe.py)
            per = max(1, nthreads // max(1, len(self.items)))
            # (a work queue of 32 MiB pieces over the tables copied at 97-182
            # GB/s where this split did 131-200: profiles/r6/uvmcap/r6b/)
            errs: List[BaseException] = []
            per_table: List[Optional[tuple]] = [None] * len(self.items)
            sem = threading.Semaphore(nthreads)

            def copy(i: int, t, n: int) -> None:
                try:
                    node = pages_node(t.data_ptr(), n)
                    mask = None
                    if node is not None:
                        import os

                        mask = node_cpus(node) & os.sched_getaffinity(0) or None
                        if mask:
                            os.sched_setaffinity(0, mask)  # this thread, then its helpers
                    ts = time.perf_counter()
                    lib.hsio_parallel_memcpy(self.blocks[i].ptr, t.data_ptr(), n, per)
                    te = time.perf_counter()
                    timeline.add("uvm_capture", "d2h", ts, te, bytes=n, node=node)
                    per_table[i] = (n, te - ts, node, self.blocks[i].ptr)
                    if knobs.TUNING.uvm_capture_overlap:
                        self.done[i].set()
                except BaseException as e:  # noqa: BLE001
                    errs.append(e)
                finally:
                    sem.release()

            workers = []
            for i, (_st, t, n) in enumerate(self.items):
                sem.acquire()
                th = threading.Thread(target=copy, args=(i, t, n), name="hs-uvm-copy",
                                      daemon=True)
                th.start()
                workers.append(th)
            for i, th in enumerate(workers):
                th.join()
            if errs:
                raise errs[0]
            for d in self.done:
                d.set()
            self.stats = {"wait_s": t1 - t0, "copy_s": time.perf_counter() - t1,
                          "bytes": float(sum(n for _s, _t, n in self.items)),
                          "start_to_release_s": time.perf_counter() - self._t_start,
                          "blocks_s": self._t_blocks - self._t_start,
                          "threads_per_table": per,
                          # (bytes, seconds, pages' node, block address) per table
                          "tables": [r for r in per_table if r is not None]}
        except BaseException as e:  # noqa: BLE001 - reported by the stagers
            self.error = e
        finally:
            native.gate_release(self.dev, self.value)
            for d in self.done:
                d.set()
            last.clear()
            last.update(self.stats)

    # -- the drain ----------------------------------------------------------------

    def buffer(self, i: int) -> StagedBuffer:
        """Table ``i``'s captured bytes.  Waits for its copy -- or, unless
        ``uvm_capture_overlap``, for the whole capture: the drain's writers
        then do not compete with the copy threads for the CPUs while the
        trainer's stream waits (``profiles/r6/uvmcap/``)."""
        if knobs.TUNING.uvm_capture_overlap:
            self.done[i].wait()
        else:
            self.done[-1].wait()
            self.wait()
        if self.error is not None:
            raise RuntimeError(f"UVM capture failed: {self.error}") from self.error
        pb, self.blocks[i] = self.blocks[i], None
        if pb is None:
            raise RuntimeError("UVM capture block handed out twice")
        from ..utils.affinity import pages_node

        sb = StagedBuffer(pb.view, pb.ptr, release=pb.release, keepalive=pb)
        sb.numa_node = pages_node(pb.ptr, pb.view.nbytes)  # the writer reads it there
        return sb

    def drop(self, i: int) -> None:
        """Table ``i``'s block was never written (the take failed): give it
        back once its copy is over."""
        self.done[i].wait()
        pb, self.blocks[i] = self.blocks[i], None
        if pb is not None:
            pb.release()

    def wait(self) -> None:
        if self._thread is not None:
            self._thread.join()

    def release_blocks(self) -> None:
        for i, pb in enumerate(self.blocks):
            if pb is not None:
                pb.release()
                self.blocks[i] = None


last: Dict[str, object] = {}  # the last capture's seconds (benchmarks)


def capture_host_uvm(write_reqs: List[WriteReq], budget: Optional[int] = None) -> List[WriteReq]:
    """Start CPU captures of the host-resident UVM tables among
    ``write_reqs`` (gating their producer streams); returns the requests
    taken over, whose stagers now hand out the captured blocks.  Nothing is
    taken over when the feature is off, the GPU cannot wait on a host word,
    or the tables exceed the host ``budget``."""
    if not knobs.TUNING.uvm_async_capture or not native.gpu_available():
        return []
    by_dev: Dict[int, list] = {}
    deps = _deps()
    for wr in write_reqs:
        t = _eligible(wr, deps)
        if t is not None:
            dev = t.device.index if t.device.index is not None else torch.cuda.current_device()
            by_dev.setdefault(dev, []).append((wr, t, t.numel() * t.element_size()))
    taken: List[WriteReq] = []
    for dev, rows in by_dev.items():
        total = sum(n for _w, _t, n in rows)
        if budget is not None and total > budget:
            logger.info(f"UVM capture on cuda:{dev}: {total} B over the host budget {budget} B; "
                        "the HBM freeze copies them")
            continue
        if not native.gate_supported(dev):
            continue
        cap = Capture(dev, [(wr.buffer_stager, t, n) for wr, t, n in rows])
        try:
            with timeline.span("uvm_capture_start", bytes=total):
                cap.start()
        except Exception as e:  # noqa: BLE001 - fall back to the HBM freeze
            logger.info(f"UVM capture on cuda:{dev} not started ({e}); the HBM freeze copies "
                        "them")
            continue
        for i, (wr, _t, _n) in enumerate(rows):
            st = wr.buffer_stager
            st.captured = (cap, i)
            st.frozen = True  # deferrable: the bytes are taken care of
            taken.append(wr)
    return taken
