#!/usr/bin/env python3
"""Costs of DMA-ing straight into a file's page cache (see
filemap_dma_probe.py): hipHostRegister of a MAP_SHARED mapping of a NEW
(truncated) file vs an EXISTING fully cached one, split over 1 / 4 / 8
threads; the D2H itself; dirtying one byte per page from the CPU; unregister
and munmap.  Compared with the pwrite path's rate from a pinned buffer."""

import ctypes
import mmap
import os
import sys
import threading
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


def run(existing: bool, nthreads: int, src):
    path = os.path.join(D, f"fmc_{int(existing)}_{nthreads}")
    if existing:
        with open(path, "wb") as f:
            f.write(np.ones(N, dtype=np.uint8).tobytes())
    fd = os.open(path, os.O_RDWR | os.O_CREAT | (0 if existing else os.O_TRUNC), 0o644)
    os.ftruncate(fd, N)
    mm = mmap.mmap(fd, N, mmap.MAP_SHARED, mmap.PROT_READ | mmap.PROT_WRITE)
    buf = (ctypes.c_char * N).from_buffer(mm)
    addr = ctypes.addressof(buf)
    part = N // nthreads
    rcs = [None] * nthreads
    t0 = time.perf_counter()

    def reg(i):
        rcs[i] = hip.hipHostRegister(addr + i * part, part, 0)

    ths = [threading.Thread(target=reg, args=(i,)) for i in range(nthreads)]
    [t.start() for t in ths]
    [t.join() for t in ths]
    t_reg = time.perf_counter() - t0
    t0 = time.perf_counter()
    r = hip.hipMemcpy(addr, src.data_ptr(), N, 2)
    t_cp = time.perf_counter() - t0
    arr = np.frombuffer(mm, dtype=np.uint8)
    t0 = time.perf_counter()
    arr[::4096] = arr[::4096]  # dirty every page
    t_dirty = time.perf_counter() - t0
    t0 = time.perf_counter()
    for i in range(nthreads):
        hip.hipHostUnregister(addr + i * part)
    t_unreg = time.perf_counter() - t0
    del arr, buf
    t0 = time.perf_counter()
    mm.close()
    os.close(fd)
    t_unmap = time.perf_counter() - t0
    with open(path, "rb") as f:
        ok = f.read(4096) == src[:4096].cpu().numpy().tobytes()
    print({"existing": existing, "threads": nthreads, "rcs": rcs, "copy_rc": r,
           "register_GBps": round(N / t_reg / 1e9, 1), "copy_GBps": round(N / t_cp / 1e9, 1),
           "dirty_ms": round(t_dirty * 1e3, 1), "unregister_ms": round(t_unreg * 1e3, 1),
           "munmap_ms": round(t_unmap * 1e3, 1), "ok": ok}, flush=True)
    os.unlink(path)


def pwrite_rate(existing: bool, pinned):
    path = os.path.join(D, "pw_probe")
    if existing:
        with open(path, "wb") as f:
            f.write(np.ones(N, dtype=np.uint8).tobytes())
    fd = os.open(path, os.O_WRONLY | os.O_CREAT | (0 if existing else os.O_TRUNC), 0o644)
    mv = memoryview(pinned.numpy())
    t0 = time.perf_counter()
    os.pwrite(fd, mv, 0)
    t = time.perf_counter() - t0
    os.close(fd)
    os.unlink(path)
    print({"pwrite_1thread_existing": existing, "GBps": round(N / t / 1e9, 2)}, flush=True)


if __name__ == "__main__":
    src = torch.randint(0, 255, (N,), dtype=torch.uint8, device="cuda")
    torch.cuda.synchronize()
    pinned = torch.empty(N, dtype=torch.uint8, pin_memory=True)
    pinned.copy_(src.cpu())
    for existing in (False, True):
        pwrite_rate(existing, pinned)
        for nt in (1, 4, 8):
            run(existing, nt, src)
