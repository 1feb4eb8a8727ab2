"""Shared launcher helpers for the benchmark scripts (torchrun or single process)."""

from __future__ import annotations

import json
import os
import socket
import sys
import time

import torch
import torch.distributed as dist


def init_dist(backend: str = None, gpu: bool = None):
    """Process group + this rank's device.  ``backend="gloo"`` with ``gpu``
    (default: a GPU is visible) rehearses several ranks sharing one GPU --
    correctness and planning cost, not scaling (RCCL refuses shared GPUs)."""
    if "RANK" not in os.environ:
        s = socket.socket()
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
        s.close()
        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK="0",
                          WORLD_SIZE="1", LOCAL_RANK="0")
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if backend is None:
        backend = "nccl" if torch.cuda.is_available() else "gloo"
    if backend == "nccl":
        torch.cuda.set_device(local_rank)
        dist.init_process_group(backend, device_id=torch.device("cuda", local_rank))
        dev = torch.device("cuda", local_rank)
    else:
        dist.init_process_group(backend)
        if gpu is None:
            gpu = torch.cuda.is_available()
        if gpu:
            idx = local_rank % torch.cuda.device_count()
            torch.cuda.set_device(idx)
            dev = torch.device("cuda", idx)
        else:
            dev = torch.device("cpu")
    return dist.get_rank(), dist.get_world_size(), dev


def log(msg: str) -> None:
    if not dist.is_initialized() or dist.get_rank() == 0:
        print(msg, file=sys.stderr, flush=True)


def emit(d: dict) -> None:
    if not dist.is_initialized() or dist.get_rank() == 0:
        print(json.dumps(d), flush=True)


def max_over_ranks(x: float, dev) -> float:
    if not dist.is_initialized() or dist.get_world_size() == 1:
        return x
    t = torch.tensor([x], dtype=torch.float64, device=dev)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def sync(dev) -> None:
    if dev.type == "cuda":
        torch.cuda.synchronize()
    if dist.is_initialized():
        dist.barrier()


class Timer:
    def __enter__(self):
        self.t0 = time.perf_counter()
        return self

    def __exit__(self, *a):
        self.s = time.perf_counter() - self.t0


def cpu_s() -> float:
    import resource

    ru = resource.getrusage(resource.RUSAGE_SELF)
    return ru.ru_utime + ru.ru_stime


def _sibling_main(i: int, sizes, root: str, dma_pass: bool, go, done, hint: int) -> None:
    """One sibling rank's host work per take (no GPU): a write pass over its
    staging memory (the D2H DMA's DRAM writes), then every blob through the
    native FS engine."""
    import asyncio

    import numpy as np

    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    from hipsnapshot import knobs
    from hipsnapshot.io_types import WriteIO
    from hipsnapshot.storage.fs import FSStoragePlugin

    knobs.set_local_ranks_hint(hint)  # I/O threads of one of `hint` ranks on this host

    buf = np.ones(max(sizes), dtype=np.uint8)  # touched: resident like the pinned pool
    staging = np.empty(sum(sizes), dtype=np.uint8)
    staging[:] = 1
    d = os.path.join(root, f"sibling{i}")
    os.makedirs(d, exist_ok=True)
    loop = asyncio.new_event_loop()
    fs = FSStoragePlugin(d)

    async def write_all():
        from hipsnapshot import knobs

        sem = asyncio.Semaphore(knobs.get_io_threads())

        async def one(j, n):
            async with sem:
                src = staging[sum(sizes[:j]): sum(sizes[:j]) + n] if dma_pass else buf[:n]
                await fs.write(WriteIO(path=f"b{j}", buf=memoryview(src)))

        await asyncio.gather(*(one(j, n) for j, n in enumerate(sizes)))

    while go.get() is not None:
        t0 = time.perf_counter()
        c0 = cpu_s()
        if dma_pass:
            staging.fill(2)
        loop.run_until_complete(write_all())
        done.put((time.perf_counter() - t0, cpu_s() - c0))
    fs.sync_close(loop)
    loop.close()


class Siblings:
    """K host-only processes replaying, per take, the host work of sibling
    ranks (benchmarks/rank_share/main.py ``--host-siblings``)."""

    def __init__(self, k: int, sizes, root: str, dma_pass: bool) -> None:
        import multiprocessing as mp

        ctx = mp.get_context("spawn")
        self.sizes = sizes
        self.go_qs = [ctx.Queue() for _ in range(k)]
        self.done = ctx.Queue()
        self.procs = [ctx.Process(target=_sibling_main,
                                  args=(i, sizes, root, dma_pass, self.go_qs[i], self.done,
                                        k + 1))
                      for i in range(k)]
        for p in self.procs:
            p.start()

    def go(self) -> None:
        for q in self.go_qs:
            q.put(1)

    def wait(self):
        return [self.done.get(timeout=120) for _ in self.procs]

    def stop(self) -> None:
        for q in self.go_qs:
            q.put(None)
        for p in self.procs:
            p.join(30)
