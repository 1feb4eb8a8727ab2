"""Can the SDMA engine write a checkpoint blob straight into the page cache?

Today a blob crosses host DRAM three times: the DMA writes it into a pinned
buffer, then pwrite() reads that buffer and writes the page-cache pages.
If the file's page-cache pages are mmap()ed and registered with HIP
(hipHostRegister), the DMA can write them directly: one pass.

This probe measures, for a 1 GiB blob:
  * pinned path: SDMA -> pinned, then pwrite() into the file (page cache);
  * mapped path: ftruncate + mmap(MAP_SHARED) + hipHostRegister (first time:
    pages allocated; again: pages already cached), SDMA into the mapping,
    then checks the file's bytes with pread();
and prints one JSON line.
"""

import ctypes
import json
import mmap
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))

import torch  # noqa: E402

from hipsnapshot.ops import native  # noqa: E402


def hip_lib():
    for line in open("/proc/self/maps"):
        if "libamdhip64.so" in line:
            return ctypes.CDLL(line.split()[-1], mode=os.RTLD_NOLOAD | os.RTLD_GLOBAL)
    raise RuntimeError("libamdhip64 not loaded")


def main():
    d = sys.argv[1] if len(sys.argv) > 1 else "/tmp"
    n = 1 << 30
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    src = torch.empty(n, dtype=torch.uint8, device=dev).random_(0, 255)
    torch.cuda.synchronize()
    ref = src.cpu().numpy()
    hip = hip_lib()
    hip.hipHostRegister.argtypes = [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_uint]
    hip.hipHostUnregister.argtypes = [ctypes.c_void_p]
    hip.hipHostGetDevicePointer.argtypes = [ctypes.POINTER(ctypes.c_void_p), ctypes.c_void_p,
                                            ctypes.c_uint]
    out = {}

    # --- pinned path
    pb = native.PinnedBuffer(n)
    p1 = os.path.join(d, "pc_probe_pinned")
    fd = os.open(p1, os.O_CREAT | os.O_WRONLY, 0o644)
    for it in range(3):
        t0 = time.perf_counter()
        native.sdma_d2h(0, pb.ptr, src.data_ptr(), n, 0)
        t1 = time.perf_counter()
        os.pwrite(fd, pb.view, 0)
        t2 = time.perf_counter()
        out[f"pinned_sdma_GBps_{it}"] = round(n / (t1 - t0) / 1e9, 1)
        out[f"pinned_pwrite_GBps_{it}"] = round(n / (t2 - t1) / 1e9, 1)
    os.close(fd)

    # --- mapped path
    p2 = os.path.join(d, "pc_probe_mapped")
    fd = os.open(p2, os.O_CREAT | os.O_RDWR, 0o644)
    os.ftruncate(fd, n)
    for it in range(3):
        t0 = time.perf_counter()
        mm = mmap.mmap(fd, n, mmap.MAP_SHARED, mmap.PROT_READ | mmap.PROT_WRITE)
        buf = ctypes.c_char.from_buffer(mm)
        addr = ctypes.addressof(buf)
        t1 = time.perf_counter()
        r = hip.hipHostRegister(addr, n, 0)
        t2 = time.perf_counter()
        out[f"map_s_{it}"] = round(t1 - t0, 4)
        out[f"register_rc_{it}"] = r
        out[f"register_GBps_{it}"] = round(n / (t2 - t1) / 1e9, 2)
        if r != 0:
            del buf
            mm.close()
            break
        dptr = ctypes.c_void_p()
        hip.hipHostGetDevicePointer(ctypes.byref(dptr), addr, 0)
        out["dev_ptr_equals_host"] = dptr.value == addr
        src.add_(1)
        torch.cuda.synchronize()
        t3 = time.perf_counter()
        try:
            native.sdma_d2h(0, dptr.value, src.data_ptr(), n, 0)
            out[f"mapped_sdma_GBps_{it}"] = round(n / (time.perf_counter() - t3) / 1e9, 1)
        except native.HipError as e:
            out[f"mapped_sdma_error_{it}"] = str(e)
        t4 = time.perf_counter()
        hip.hipHostUnregister(addr)
        out[f"unregister_s_{it}"] = round(time.perf_counter() - t4, 4)
        del buf
        mm.close()
        got = os.pread(fd, n, 0)
        want = src.cpu().numpy().tobytes()
        out[f"file_matches_{it}"] = got == want
    os.close(fd)
    pb.release()
    for p in (p1, p2):
        os.remove(p)
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
