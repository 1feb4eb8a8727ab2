#!/usr/bin/env python3
"""Persistent DMA-able mapping of a checkpoint file: register once, then per
"take" DMA into it and re-dirty every page from the CPU (a DMA write does not
mark page-cache pages dirty).  Measures the re-dirty cost when the pages are
still dirty and after writeback cleaned them (fdatasync: write-protect faults),
and checks the bytes reach the file."""

import ctypes
import mmap
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

hip = ctypes.CDLL("libamdhip64.so")
hip.hipHostRegister.argtypes = [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_uint]
hip.hipHostUnregister.argtypes = [ctypes.c_void_p]
hip.hipMemcpy.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int]
N = 1 << 30
D = os.environ.get("HSBENCH_DIR", "/tmp")


def dirty(arr):
    t0 = time.perf_counter()
    v = arr[::4096]
    np.add(v, 0, out=v, casting="unsafe")  # one store per page
    return (time.perf_counter() - t0) * 1e3


path = os.path.join(D, "fmp")
fd = os.open(path, os.O_RDWR | os.O_CREAT | os.O_TRUNC, 0o644)
os.ftruncate(fd, N)
mm = mmap.mmap(fd, N, mmap.MAP_SHARED, mmap.PROT_READ | mmap.PROT_WRITE)
buf = (ctypes.c_char * N).from_buffer(mm)
addr = ctypes.addressof(buf)
arr = np.frombuffer(mm, dtype=np.uint8)
t0 = time.perf_counter()
assert hip.hipHostRegister(addr, N, 0) == 0
print({"register_ms": round((time.perf_counter() - t0) * 1e3, 1)}, flush=True)
for take in range(4):
    src = torch.randint(0, 255, (N,), dtype=torch.uint8, device="cuda")
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    rc = hip.hipMemcpy(addr, src.data_ptr(), N, 2)
    t_cp = time.perf_counter() - t0
    d_ms = dirty(arr)
    t0 = time.perf_counter()
    if take % 2 == 1:
        os.fdatasync(fd)  # writeback: the pages are clean (write-protected) for the next take
    t_sync = time.perf_counter() - t0
    # the file content through the page cache and after dropping it
    with open(path, "rb") as f:
        f.seek(N // 2)
        ok = f.read(4096) == src[N // 2: N // 2 + 4096].cpu().numpy().tobytes()
    print({"take": take, "copy_rc": rc, "copy_GBps": round(N / t_cp / 1e9, 1),
           "dirty_ms": round(d_ms, 1), "fdatasync_ms": round(t_sync * 1e3, 1), "ok": ok},
          flush=True)
t0 = time.perf_counter()
hip.hipHostUnregister(addr)
print({"unregister_ms": round((time.perf_counter() - t0) * 1e3, 1)}, flush=True)
os.fdatasync(fd)
posix_fadvise = getattr(os, "posix_fadvise", None)
del arr, buf
mm.close()
if posix_fadvise:
    os.posix_fadvise(fd, 0, N, os.POSIX_FADV_DONTNEED)  # drop the clean cache
os.close(fd)
with open(path, "rb") as f:
    f.seek(N // 2)
    print({"after_drop_ok": f.read(4096) == src[N // 2: N // 2 + 4096].cpu().numpy().tobytes()},
          flush=True)
os.unlink(path)
