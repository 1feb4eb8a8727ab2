#!/usr/bin/env python3
"""HBM->HBM copy rate of the freeze kernel (hs_copy_nd, one launch over the
Llama-3-8B FSDP tensors' sizes) against torch's copy_ and a single
hipMemcpyAsync-backed copy of the same bytes."""

import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

from hipsnapshot.ops import native  # noqa: E402

dev = 0
torch.cuda.set_device(dev)
# the 8B model's parameter sizes (bf16), 32 layers
sizes = [128256 * 4096, 128256 * 4096, 4096]
for _ in range(32):
    sizes += [4096 * 4096, 1024 * 4096, 1024 * 4096, 4096 * 4096, 14336 * 4096,
              4096 * 14336, 14336 * 4096, 4096, 4096]
srcs = [torch.empty(n, dtype=torch.bfloat16, device="cuda").normal_() for n in sizes]
total = sum(n * 2 for n in sizes)
arena = torch.empty(total + 256 * len(sizes), dtype=torch.uint8, device="cuda")
stream = torch.cuda.current_stream()


def freeze_once():
    b = native.CopyBatch()
    off = 0
    for t in srcs:
        b.add_tensor(t, arena.data_ptr() + off)
        off += (t.numel() * 2 + 255) // 256 * 256
    arr = b.pack()
    return arr


arr = freeze_once()
res = {}
for name, fn in (
        ("hs_copy_nd", lambda: native.launch_packed(arr, dev, int(stream.cuda_stream), sync=False)),
        ("torch_copy_", lambda: [arena[:t.numel() * 2].view(torch.bfloat16).copy_(t) for t in srcs]),
        ("one_memcpy_d2d", lambda: arena[:total // 2 * 2].copy_(arena[total // 2 * 2: total // 2 * 2 + total // 2 * 2])
         if False else torch.cuda.memory.caching_allocator_alloc)):
    pass
ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
for name in ("hs_copy_nd", "torch_copy_"):
    times = []
    for it in range(6):
        torch.cuda.synchronize()
        ev0.record()
        if name == "hs_copy_nd":
            keep = native.launch_packed(arr, dev, int(stream.cuda_stream), sync=False)
        else:
            off = 0
            for t in srcs:
                arena[off: off + t.numel() * 2].view(torch.bfloat16).copy_(t)
                off += (t.numel() * 2 + 255) // 256 * 256
        ev1.record()
        torch.cuda.synchronize()
        times.append(ev0.elapsed_time(ev1))
    best = min(times[1:])
    res[name] = {"ms": round(best, 3), "payload_TBps": round(total / best / 1e9, 2)}
# one contiguous D2D memcpy of the same byte count (runtime's copy path)
half = total
src_flat = torch.empty(half, dtype=torch.uint8, device="cuda")
times = []
for it in range(6):
    torch.cuda.synchronize()
    ev0.record()
    arena[:half].copy_(src_flat)
    ev1.record()
    torch.cuda.synchronize()
    times.append(ev0.elapsed_time(ev1))
best = min(times[1:])
res["one_contiguous_copy_"] = {"ms": round(best, 3), "payload_TBps": round(half / best / 1e9, 2)}
res["bytes"] = total
print(res, flush=True)
