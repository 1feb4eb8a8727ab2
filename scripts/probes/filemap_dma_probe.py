#!/usr/bin/env python3
"""Can the GPU DMA straight into a file's page cache?  mmap(MAP_SHARED) a
file on the bench disk (and on /dev/shm), hipHostRegister the mapping, copy
device bytes into it (hipMemcpy D2H and an SDMA copy), dirty each page from
the CPU, munmap, and read the file back.  Prints what worked."""

import ctypes
import mmap
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

hip = ctypes.CDLL("libamdhip64.so")
hip.hipHostRegister.argtypes = [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_uint]
hip.hipHostUnregister.argtypes = [ctypes.c_void_p]
hip.hipMemcpy.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int]
hip.hipGetErrorString.restype = ctypes.c_char_p


def err(e):
    return hip.hipGetErrorString(e).decode()


def probe(d: str, n: int, flags: int):
    path = os.path.join(d, f"fm_probe_{flags}")
    fd = os.open(path, os.O_RDWR | os.O_CREAT | os.O_TRUNC, 0o644)
    os.ftruncate(fd, n)
    mm = mmap.mmap(fd, n, mmap.MAP_SHARED, mmap.PROT_READ | mmap.PROT_WRITE)
    buf = (ctypes.c_char * n).from_buffer(mm)
    addr = ctypes.addressof(buf)
    t0 = time.perf_counter()
    r = hip.hipHostRegister(addr, n, flags)
    out = {"dir": d, "flags": flags, "register": err(r),
           "register_ms": round((time.perf_counter() - t0) * 1e3, 2)}
    if r == 0:
        src = torch.randint(0, 255, (n,), dtype=torch.uint8, device="cuda")
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        r2 = hip.hipMemcpy(addr, src.data_ptr(), n, 2)  # D2H
        out["memcpy"] = err(r2)
        out["memcpy_GBps"] = round(n / (time.perf_counter() - t0) / 1e9, 2)
        from hipsnapshot.ops import native

        try:
            t0 = time.perf_counter()
            src2 = src.flip(0).contiguous()
            torch.cuda.synchronize()
            native.sdma_d2h(0, addr, src2.data_ptr(), n, native.copy_stream(0, 3))
            out["sdma_GBps"] = round(n / (time.perf_counter() - t0) / 1e9, 2)
            expect = src2.cpu().numpy().tobytes()
        except Exception as e:  # noqa: BLE001
            out["sdma"] = repr(e)
            expect = src.cpu().numpy().tobytes()
        # dirty every page from the CPU (a DMA write does not mark it dirty)
        for off in range(0, n, 4096):
            mm[off] = mm[off]
        hip.hipHostUnregister(addr)
    del buf
    mm.flush()
    mm.close()
    os.close(fd)
    if r == 0:
        with open(path, "rb") as f:
            got = f.read()
        out["file_ok"] = got == expect
    os.unlink(path)
    print(out, flush=True)


if __name__ == "__main__":
    n = 256 << 20
    for d in (os.environ.get("HSBENCH_DIR", "/tmp"), "/dev/shm", "/var/tmp"):
        for flags in (0, 1, 2):  # default, portable, mapped
            try:
                probe(d, n, flags)
            except Exception as e:  # noqa: BLE001
                print({"dir": d, "flags": flags, "error": repr(e)}, flush=True)
