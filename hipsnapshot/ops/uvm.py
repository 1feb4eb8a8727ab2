"""Managed-memory (UVM) tensors -- the fbgemm ``uvm_tensor`` equivalent (K11).

Reference: `/root/reference/torchsnapshot/uvm_tensor.py:11-42` binds fbgemm_gpu's
``new_managed_tensor / is_uvm_tensor / uvm_to_cpu``.  fbgemm is not available
for this stack, so managed memory is allocated natively with
``hipMallocManaged`` (``_hsgpu.so``) and exposed to torch as a CUDA tensor via
``torch.from_blob``-style storage wrapping; detection uses
``hipPointerGetAttributes(...).isManaged``.  Staging a UVM tensor goes
through the same SDMA path as any other device tensor (the driver migrates
pages as needed), i.e. no separate ``uvm_to_cpu`` copy.
"""

from __future__ import annotations

import weakref
from typing import Dict, List

import torch

from . import native

_managed: Dict[int, int] = {}


def is_uvm_tensor(t: torch.Tensor) -> bool:
    if not isinstance(t, torch.Tensor) or not t.is_cuda:
        return False
    ptr = t.untyped_storage().data_ptr()
    if ptr in _managed:
        return True
    return native.is_managed_ptr(ptr)


def residency(t: torch.Tensor) -> str:
    """Where a managed tensor's pages live: ``"host"`` / ``"device"`` when
    advised or prefetched (``place``); never-placed pages are in host DRAM
    unless XNACK migrates them (``knobs.uvm_assume_host``), else
    ``"unknown"``.  Not a managed tensor: ``"not_managed"`` (the range query
    is only valid on managed memory)."""
    if not is_uvm_tensor(t):
        return "not_managed"
    ptr = t.untyped_storage().data_ptr()
    nbytes = max(t.untyped_storage().nbytes(), 1)
    pref, last = native.managed_location(ptr, nbytes)
    loc = last if last != -2 else pref
    if loc == -2:
        from .. import knobs

        return "host" if knobs.uvm_assume_host() else "unknown"
    return "host" if loc == -1 else "device"


def place(t: torch.Tensor, where: str) -> None:
    """Advise + prefetch a managed tensor's pages to host DRAM (``"host"``,
    TorchRec's UVM tables larger than HBM) or to its GPU (``"device"``);
    asynchronous on the current stream."""
    if where not in ("host", "device"):
        raise ValueError(f"where must be 'host' or 'device' (got {where!r})")
    dev = t.device.index if t.device.index is not None else torch.cuda.current_device()
    native.managed_place(dev, t.untyped_storage().data_ptr(),
                         max(t.untyped_storage().nbytes(), 1), -1 if where == "host" else dev,
                         int(torch.cuda.current_stream(dev).cuda_stream))


def uvm_to_cpu(t: torch.Tensor) -> torch.Tensor:
    return t.detach().cpu()


def new_managed_tensor(shape: List[int], dtype: torch.dtype = torch.float32,
                       device: int = 0) -> torch.Tensor:
    """Allocate a managed-memory tensor visible to the given HIP device."""
    lib = native.require_gpu_lib()
    numel = 1
    for s in shape:
        numel *= int(s)
    nbytes = max(numel * torch.empty(0, dtype=dtype).element_size(), 1)
    ptr = lib.hsg_managed_alloc(device, nbytes)
    if not ptr:
        raise MemoryError(f"hipMallocManaged({nbytes}) failed: {lib.hsg_last_error().decode()}")
    _managed[ptr] = nbytes

    def _free(p=ptr):
        _managed.pop(p, None)
        lib.hsg_managed_free(p)

    # wrap as a CUDA tensor through DLPack-free __cuda_array_interface__
    class _Holder:
        pass

    # the pages as bytes, then viewed as ``dtype``: the array interface has no
    # type string torch accepts for bf16 / fp8 (a "<V2" bf16 table failed to
    # wrap -- tests/test_uvm_random.py)
    holder = _Holder()
    holder.__cuda_array_interface__ = {
        "shape": (nbytes,), "typestr": "|u1", "data": (ptr, False), "version": 3,
        "strides": None,
    }
    with torch.cuda.device(device):
        raw = torch.as_tensor(holder, device=f"cuda:{device}")
    t = raw[: numel * torch.empty(0, dtype=dtype).element_size()].view(dtype).view(
        [int(s) for s in shape])
    weakref.finalize(t.untyped_storage(), _free)
    return t
