"""Pinned host memory: hipHostMalloc vs THP-backed anonymous memory that is
registered with hipHostRegister.

For each kind: pread() of a page-cached file into it (16 threads x 8 MiB),
SDMA device -> host into it, and host -> device copy from it.  One JSON line.
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

MADV_HUGEPAGE = 14


def hip_lib():
    for line in open("/proc/self/maps"):
        if "libamdhip64.so" in line:
            return ctypes.CDLL(line.split()[-1], mode=os.RTLD_NOLOAD | os.RTLD_GLOBAL)
    raise RuntimeError("libamdhip64 not loaded")


def par_pread(fd, addr, n, nthreads=16, piece=8 << 20):
    buf = (ctypes.c_char * n).from_address(addr)
    mv = memoryview(buf).cast("B")
    offs = list(range(0, n, piece))
    idx = [0]
    lock = threading.Lock()

    def th():
        while True:
            with lock:
                if idx[0] >= len(offs):
                    return
                o = offs[idx[0]]
                idx[0] += 1
            os.preadv(fd, [mv[o:o + piece]], o)

    ts = [threading.Thread(target=th) for _ in range(nthreads)]
    t0 = time.perf_counter()
    for t in ts:
        t.start()
    for t in ts:
        t.join()
    return n / (time.perf_counter() - t0) / 1e9


def main():
    d = sys.argv[1]
    n = 1 << 30
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    src = torch.empty(n, dtype=torch.uint8, device=dev).random_(0, 255)
    dst = torch.empty(n, dtype=torch.uint8, device=dev)
    torch.cuda.synchronize()
    path = os.path.join(d, "thp_probe.bin")
    with open(path, "wb") as f:
        f.write(os.urandom(1 << 20) * 1024)
    fd = os.open(path, os.O_RDONLY)
    hip = hip_lib()
    hip.hipHostRegister.argtypes = [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_uint]
    hip.hipHostUnregister.argtypes = [ctypes.c_void_p]
    libc = ctypes.CDLL("libc.so.6", use_errno=True)
    libc.madvise.argtypes = [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int]
    out = {}
    pb = native.PinnedBuffer(n)
    mm = mmap.mmap(-1, n + (2 << 20), mmap.MAP_PRIVATE | mmap.MAP_ANONYMOUS)
    cbuf = ctypes.c_char.from_buffer(mm)
    base = ctypes.addressof(cbuf)
    addr = (base + (2 << 20) - 1) & ~((2 << 20) - 1)
    out["madvise_rc"] = libc.madvise(addr, n, MADV_HUGEPAGE)
    ctypes.memset(addr, 1, n)  # fault the pages in (THP where granted)
    t0 = time.perf_counter()
    out["register_rc"] = hip.hipHostRegister(addr, n, 0)
    out["register_s"] = round(time.perf_counter() - t0, 3)
    for name, a in (("hipHostMalloc", pb.ptr), ("thp_registered", addr)):
        par_pread(fd, a, n)
        out[f"pread_{name}_GBps"] = round(par_pread(fd, a, n), 1)
        cs = torch.cuda.Stream()
        native.sdma_d2h(0, a, src.data_ptr(), n, cs)
        t0 = time.perf_counter()
        for _ in range(3):
            native.sdma_d2h(0, a, src.data_ptr(), n, cs)
        out[f"sdma_d2h_{name}_GBps"] = round(3 * n / (time.perf_counter() - t0) / 1e9, 1)
        native.memcpy(0, 5, dst.data_ptr(), a, n, native.H2D, None, sync=True)
        t0 = time.perf_counter()
        for _ in range(3):
            native.memcpy(0, 5, dst.data_ptr(), a, n, native.H2D, None, sync=True)
        out[f"h2d_{name}_GBps"] = round(3 * n / (time.perf_counter() - t0) / 1e9, 1)
    ok = torch.equal(dst, src)
    out["h2d_roundtrip_ok"] = ok
    hip.hipHostUnregister(addr)
    pb.release()
    del cbuf
    mm.close()
    os.close(fd)
    os.remove(path)
    thp = [l for l in open("/sys/kernel/mm/transparent_hugepage/enabled")]
    out["thp_mode"] = thp[0].strip() if thp else "?"
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
