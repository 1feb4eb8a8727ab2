"""Test helpers: tensor equality, random tensors of every dtype, multi-process runner.

Reference: `/root/reference/torchsnapshot/test_utils.py:41-290` (patched ``__eq__``,
``rand_tensor``, ``tensor_eq``, torchelastic ``run_with_pet``).  The runner here
spawns ``world_size`` processes with a TCP rendezvous on 127.0.0.1 (the
container hostname may not resolve), initialises the requested backend (gloo
on CPU; RCCL only when one GPU per rank exists) and re-raises the first
worker failure with its traceback.
"""

from __future__ import annotations

import asyncio
import functools
import time
import os
import socket
import traceback
from contextlib import contextmanager
from typing import Any, Callable, Dict, Generator, List, Optional

import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from ..format.serialization import SUPPORTED_QUANTIZED_DTYPES


def rand_tensor(shape, dtype: torch.dtype = torch.float32, device: str = "cpu") -> torch.Tensor:
    shape = list(shape) if not isinstance(shape, int) else [shape]
    if dtype in SUPPORTED_QUANTIZED_DTYPES:
        base = torch.rand(shape) * 10
        if dtype == torch.qint32:
            return torch.quantize_per_tensor(base, 0.1, 10, torch.qint32)
        return torch.quantize_per_tensor(base, 0.1, 10, dtype)
    if dtype == torch.bool:
        return torch.randint(0, 2, shape, device=device).bool()
    if dtype in (torch.uint8, torch.int8, torch.int16, torch.int32, torch.int64):
        info = torch.iinfo(dtype)
        lo, hi = max(info.min, -1000), min(info.max, 1000)
        return torch.randint(lo, hi, shape, dtype=dtype, device=device)
    if dtype.is_complex:
        return torch.randn(shape, dtype=dtype, device=device)
    if str(dtype).startswith("torch.float8"):
        return torch.randn(shape, device=device).to(dtype)
    return torch.randn(shape, device=device).to(dtype)


def _dense(t: Any) -> Any:
    try:
        from torch.distributed.tensor import DTensor

        if isinstance(t, DTensor):
            return t.full_tensor()
    except Exception:  # pragma: no cover
        pass
    return t


def _is_sharded_tensor(t: Any) -> bool:
    try:
        from torch.distributed._shard.sharded_tensor import ShardedTensor
    except Exception:  # pragma: no cover
        return False
    return isinstance(t, ShardedTensor)


def sharded_tensor_eq(a: Any, b: Any) -> bool:
    """Local comparison of two ShardedTensors (no collective): same global
    metadata and bitwise-equal local shards at the same offsets
    (reference: `/root/reference/torchsnapshot/test_utils.py:65-101`)."""
    if not (_is_sharded_tensor(a) and _is_sharded_tensor(b)):
        return False
    ma, mb = a.metadata(), b.metadata()
    if list(ma.size) != list(mb.size) or ma.tensor_properties.dtype != mb.tensor_properties.dtype:
        return False
    if [(s.shard_offsets, s.shard_sizes) for s in ma.shards_metadata] != \
            [(s.shard_offsets, s.shard_sizes) for s in mb.shards_metadata]:
        return False
    la, lb = a.local_shards(), b.local_shards()
    if len(la) != len(lb):
        return False
    for x, y in zip(la, lb):
        if x.metadata.shard_offsets != y.metadata.shard_offsets or \
                not tensor_eq(x.tensor, y.tensor):
            return False
    return True


def tensor_eq(a: torch.Tensor, b: torch.Tensor) -> bool:
    if _is_sharded_tensor(a) or _is_sharded_tensor(b):
        return sharded_tensor_eq(a, b)
    a, b = _dense(a), _dense(b)
    if a.is_quantized != b.is_quantized:
        return False
    if a.is_quantized:
        return (a.qscheme() == b.qscheme() and torch.equal(a.int_repr(), b.int_repr())
                and torch.equal(a.dequantize(), b.dequantize()))
    if a.dtype != b.dtype or a.shape != b.shape:
        return False
    if str(a.dtype).startswith("torch.float8"):
        return torch.equal(a.view(torch.uint8).cpu(), b.view(torch.uint8).cpu())
    return torch.equal(a.cpu(), b.cpu())


def assert_state_dict_eq(a: Any, b: Any, path: str = "") -> None:
    if isinstance(a, torch.Tensor) or isinstance(b, torch.Tensor):
        assert isinstance(a, torch.Tensor) and isinstance(b, torch.Tensor), path
        assert tensor_eq(a, b), f"tensor mismatch at {path}"
    elif isinstance(a, dict):
        assert isinstance(b, dict) and list(a.keys()) == list(b.keys()), \
            f"keys differ at {path}: {list(a.keys())} vs {list(b.keys())}"
        for k in a:
            assert_state_dict_eq(a[k], b[k], f"{path}/{k}")
    elif isinstance(a, (list, tuple)):
        assert type(a) is type(b) and len(a) == len(b), path
        for i, (x, y) in enumerate(zip(a, b)):
            assert_state_dict_eq(x, y, f"{path}/{i}")
    else:
        assert a == b, f"{path}: {a!r} != {b!r}"


def free_port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _worker(rank: int, world_size: int, port: int, backend: str, fn: Callable, args, kwargs,
            errq) -> None:
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world_size), LOCAL_RANK=str(rank),
                      LOCAL_WORLD_SIZE=str(world_size))
    try:
        if backend:
            if backend == "nccl":
                torch.cuda.set_device(rank)
            dist.init_process_group(backend, rank=rank, world_size=world_size,
                                    init_method=f"tcp://127.0.0.1:{port}")
        fn(*args, **kwargs)
        if backend and dist.is_initialized():
            dist.barrier()
            dist.destroy_process_group()
    except BaseException:  # noqa: BLE001
        errq.put((rank, traceback.format_exc()))
        raise


def run_distributed(fn: Callable, world_size: int, *args, backend: str = "gloo",
                    timeout: float = 240.0, **kwargs) -> None:
    """Run ``fn(*args, **kwargs)`` in ``world_size`` spawned ranks."""
    ctx = mp.get_context("spawn")
    errq = ctx.SimpleQueue()
    port = free_port()
    procs = [ctx.Process(target=_worker, args=(r, world_size, port, backend, fn, args, kwargs,
                                               errq), daemon=False)
             for r in range(world_size)]
    for p in procs:
        p.start()
    # poll: once a rank has failed, its peers usually block in a collective
    # with it -- give them a short grace period instead of the full timeout
    deadline = time.monotonic() + timeout
    failed_at = None
    while any(p.is_alive() for p in procs) and time.monotonic() < deadline:
        if failed_at is None and any(p.exitcode not in (None, 0) for p in procs):
            failed_at = time.monotonic()
        if failed_at is not None and time.monotonic() - failed_at > 15:
            break
        for p in procs:
            p.join(0.05)
    alive = [p for p in procs if p.is_alive()]
    for p in alive:
        p.kill()
        p.join()
    errors = []
    while not errq.empty():
        errors.append(errq.get())
    if errors:
        # a peer's "connection closed" is a consequence: report the cause
        secondary = ("Connection closed by peer", "Connection reset by peer")
        rank, tb = sorted(errors, key=lambda e: (any(s in e[1] for s in secondary), e[0]))[0]
        raise RuntimeError(f"rank {rank} failed:\n{tb}")
    if alive:
        raise TimeoutError(f"{len(alive)} rank(s) timed out after {timeout}s")
    bad = [p.exitcode for p in procs if p.exitcode != 0]
    if bad:
        raise RuntimeError(f"worker exit codes {bad}")


def run_with_pet(nproc: int, timeout: float = 240.0) -> Callable:
    """Decorator: run the (module-level) test function in ``nproc`` gloo ranks."""

    def deco(fn):
        @functools.wraps(fn)
        def wrapper(*args, **kwargs):
            run_distributed(fn.__wrapped_target__, nproc, *args, timeout=timeout, **kwargs)

        fn.__wrapped_target__ = fn
        return wrapper

    return deco


def async_test(coro_fn):
    @functools.wraps(coro_fn)
    def wrapper(*args, **kwargs):
        loop = asyncio.new_event_loop()
        try:
            return loop.run_until_complete(coro_fn(*args, **kwargs))
        finally:
            loop.close()

    return wrapper


@contextmanager
def env(**overrides: str) -> Generator[None, None, None]:
    prev: Dict[str, Optional[str]] = {k: os.environ.get(k) for k in overrides}
    os.environ.update({k: str(v) for k, v in overrides.items()})
    try:
        yield
    finally:
        for k, v in prev.items():
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = v


def local_shard_bytes(obj: Any) -> int:
    from ..io.sharded import local_boxes

    return sum(b.tensor.numel() * b.tensor.element_size() for b in local_boxes(obj))


def all_dtypes() -> List[torch.dtype]:
    from ..format.serialization import ALL_SUPPORTED_DTYPES

    return [d for d in ALL_SUPPORTED_DTYPES
            if d not in (getattr(torch, "uint16", None), getattr(torch, "uint32", None),
                         getattr(torch, "uint64", None))]


def hsz_deep_tree_frame(n: int = 65536) -> bytes:
    """One bf16-shaped HSZ1 frame (``2 * n`` bytes) whose index histogram needs
    a length-limited Huffman code: 14 rare high bytes with Fibonacci counts
    (1, 1, 2, ... 377) placed exactly on the dictionary's sample positions, so
    all of them enter the dictionary, plus one dominant high byte.  The
    unlimited tree is deeper than ``codec.HUFF_MAX_LEN``, so encoders must run
    the Kraft fix-up (``codec.huffman_lengths``)."""
    import numpy as np

    from ..ops import codec

    at = codec.sample_indices(n)
    hi = np.full(n, 0x3C, dtype=np.uint8)
    fib = [1, 1]
    while len(fib) < 14:
        fib.append(fib[-1] + fib[-2])
    vals = [v for v in range(0x30, 0x50) if v != 0x3C][:14]
    pos = 0
    for v, c in zip(vals, fib):
        hi[at[pos:pos + c]] = v
        pos += c
    lo = np.random.default_rng(5).integers(0, 256, n, dtype=np.uint8)
    return np.stack([lo, hi], 1).reshape(-1).tobytes()


def low_byte_offset(blob_bytes: bytes) -> int:
    """File offset of a byte in frame 0's low-byte plane of an HSZ1 blob
    (stored verbatim: a flip there decodes without error, to a wrong value)."""
    from hipsnapshot.ops import codec

    hdr = codec.parse_header(blob_bytes)
    mode = codec.frame_modes(blob_bytes)[0]
    lo = hdr.offsets[0] + 32
    if mode == 1:
        n = min(hdr.frame_bytes, hdr.logical_size) // hdr.elem_width
        lo += (n + 1) // 2
    assert mode in (1, 2), mode
    return lo + 100
