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
