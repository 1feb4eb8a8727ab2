"""SDMA straight into page-cache pages, part 2: is it SAFE, and is it fast
with several threads?

Part 1 (``pagecache_dma_probe.py``, profiles/r3/pagecache_dma.json) showed
hipHostRegister accepts an mmap(MAP_SHARED) file mapping and the SDMA
engine writes it at 56.7 GB/s.  Open questions answered here:

persistence
  After register -> DMA -> unregister -> munmap, are the pages DIRTY (so the
  kernel writes them back)?  ``posix_fadvise(DONTNEED)`` drops only CLEAN
  page-cache pages: if the file still reads back the new bytes after it
  (without any fsync), the pages were dirty; after ``fdatasync`` + DONTNEED
  the bytes must come from the disk.
throughput
  ``threads`` x 256 MiB pieces of one 2 GiB blob, per path:
  * ``mapped``  -- mmap + hipHostRegister + SDMA + unregister + munmap,
    rewriting an existing file (pages cached) and into a fresh file;
  * ``pinned``  -- SDMA into a pinned block + pwrite (what the engine does).
Prints one JSON line.
"""

import ctypes
import json
import mmap
import os
import sys
import threading
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))

import torch  # noqa: E402

from hipsnapshot.ops import native  # noqa: E402


def hip_lib():
    for line in open("/proc/self/maps"):
        if "libamdhip64.so" in line:
            lib = ctypes.CDLL(line.split()[-1], mode=os.RTLD_NOLOAD | os.RTLD_GLOBAL)
            lib.hipHostRegister.argtypes = [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_uint]
            lib.hipHostUnregister.argtypes = [ctypes.c_void_p]
            return lib
    raise RuntimeError("libamdhip64 not loaded")


libc = ctypes.CDLL("libc.so.6", use_errno=True)
libc.mmap.restype = ctypes.c_void_p
libc.mmap.argtypes = [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                      ctypes.c_long]
libc.munmap.argtypes = [ctypes.c_void_p, ctypes.c_size_t]
PROT_RW, MAP_SHARED = 0x3, 0x01


def mapped_write(hip, fd, off, n, src_ptr, dev=0):
    """One piece: map [off, off+n) of fd, register, DMA, unregister, unmap."""
    t0 = time.perf_counter()
    addr = libc.mmap(None, n, PROT_RW, MAP_SHARED, fd, off)
    if addr in (None, ctypes.c_void_p(-1).value):
        raise OSError(ctypes.get_errno(), "mmap")
    t1 = time.perf_counter()
    r = hip.hipHostRegister(addr, n, 0)
    if r != 0:
        libc.munmap(addr, n)
        raise RuntimeError(f"hipHostRegister rc={r}")
    t2 = time.perf_counter()
    native.sdma_d2h(dev, addr, src_ptr, n, 0)
    t3 = time.perf_counter()
    hip.hipHostUnregister(addr)
    libc.munmap(addr, n)
    t4 = time.perf_counter()
    return {"map": t1 - t0, "register": t2 - t1, "dma": t3 - t2, "unmap": t4 - t3}


def run_threads(fn, threads, n_total, piece):
    offs = list(range(0, n_total, piece))
    parts, lock = [], threading.Lock()

    def worker(i):
        for k in range(i, len(offs), threads):
            r = fn(offs[k], min(piece, n_total - offs[k]))
            with lock:
                parts.append(r)

    t0 = time.perf_counter()
    ts = [threading.Thread(target=worker, args=(i,)) for i in range(threads)]
    for t in ts:
        t.start()
    for t in ts:
        t.join()
    dt = time.perf_counter() - t0
    agg = {k: round(sum(p[k] for p in parts), 4) for k in parts[0]} if parts and \
        isinstance(parts[0], dict) else {}
    return round(n_total / dt / 1e9, 2), agg


def main():
    d = sys.argv[1] if len(sys.argv) > 1 else "/tmp"
    n = 2 << 30
    piece = 256 << 20
    torch.cuda.set_device(0)
    src = torch.empty(n, dtype=torch.uint8, device="cuda").random_(0, 255)
    torch.cuda.synchronize()
    hip = hip_lib()
    out = {}

    # ---------------- persistence
    p = os.path.join(d, "pc2_persist")
    fd = os.open(p, os.O_CREAT | os.O_RDWR | os.O_TRUNC, 0o644)
    os.ftruncate(fd, piece)
    os.pwrite(fd, bytes(piece), 0)  # old content: zeros, already on the page cache
    os.fdatasync(fd)
    want = src[:piece].cpu().numpy().tobytes()
    mapped_write(hip, fd, 0, piece, src.data_ptr())
    os.posix_fadvise(fd, 0, piece, os.POSIX_FADV_DONTNEED)
    out["after_dontneed_no_sync_matches"] = os.pread(fd, piece, 0) == want
    os.fdatasync(fd)
    os.posix_fadvise(fd, 0, piece, os.POSIX_FADV_DONTNEED)
    out["after_fdatasync_dontneed_matches"] = os.pread(fd, piece, 0) == want
    # a second DMA over the same (now clean, cached) pages
    src[:piece].add_(7)
    torch.cuda.synchronize()
    want2 = src[:piece].cpu().numpy().tobytes()
    mapped_write(hip, fd, 0, piece, src.data_ptr())
    os.posix_fadvise(fd, 0, piece, os.POSIX_FADV_DONTNEED)
    out["rewrite_after_dontneed_no_sync_matches"] = os.pread(fd, piece, 0) == want2
    os.fdatasync(fd)
    os.posix_fadvise(fd, 0, piece, os.POSIX_FADV_DONTNEED)
    out["rewrite_after_fdatasync_dontneed_matches"] = os.pread(fd, piece, 0) == want2
    os.close(fd)
    os.remove(p)

    # ---------------- throughput
    for threads in (1, 2, 4):
        # mapped, fresh file each rep (pages allocated by the register)
        pf = os.path.join(d, f"pc2_fresh_{threads}")
        fd = os.open(pf, os.O_CREAT | os.O_RDWR | os.O_TRUNC, 0o644)
        os.ftruncate(fd, n)
        gbps, agg = run_threads(lambda o, k: mapped_write(hip, fd, o, k, src.data_ptr() + o),
                                threads, n, piece)
        out[f"mapped_fresh_t{threads}_GBps"] = gbps
        out[f"mapped_fresh_t{threads}_s"] = agg
        # same file again: pages are cached (the in-place rewrite case)
        gbps, agg = run_threads(lambda o, k: mapped_write(hip, fd, o, k, src.data_ptr() + o),
                                threads, n, piece)
        out[f"mapped_rewrite_t{threads}_GBps"] = gbps
        out[f"mapped_rewrite_t{threads}_s"] = agg
        os.close(fd)
        os.remove(pf)

        # pinned + pwrite, fresh file then rewrite
        bufs = [native.PinnedBuffer(piece) for _ in range(threads)]
        pp = os.path.join(d, f"pc2_pinned_{threads}")
        fd = os.open(pp, os.O_CREAT | os.O_RDWR | os.O_TRUNC, 0o644)
        idx = {}

        def pinned(o, k, fd=fd):
            b = bufs[idx.setdefault(threading.get_ident(), len(idx)) % threads]
            t0 = time.perf_counter()
            native.sdma_d2h(0, b.ptr, src.data_ptr() + o, k, 0)
            t1 = time.perf_counter()
            os.pwrite(fd, b.view[:k], o)
            return {"dma": t1 - t0, "pwrite": time.perf_counter() - t1}

        for tag in ("fresh", "rewrite"):
            gbps, agg = run_threads(pinned, threads, n, piece)
            out[f"pinned_{tag}_t{threads}_GBps"] = gbps
            out[f"pinned_{tag}_t{threads}_s"] = agg
        os.close(fd)
        os.remove(pp)
        for b in bufs:
            b.release()
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
