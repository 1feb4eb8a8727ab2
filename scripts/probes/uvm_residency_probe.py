#!/usr/bin/env python3
"""Where do hipMallocManaged pages live on this box, and what do advise /
prefetch change?  (BASELINE config 4 saves UVM embedding tables.)

For a 4 GB managed tensor filled by a GPU kernel: the range attributes
(preferred / last-prefetch location), the GPU read rate (a reduction kernel:
~5 TB/s when the pages are in HBM, PCIe rate when they are in host DRAM) and
the CPU read rate (memcpy into a pinned buffer), first as allocated, then
after advise+prefetch to the GPU, then after advise+prefetch to the CPU.
One JSON line per state.
"""

import ctypes
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))

import torch  # noqa: E402

from hipsnapshot.ops import native  # noqa: E402
from hipsnapshot.ops.uvm import new_managed_tensor  # noqa: E402

CPU = -1


def main() -> None:
    n = int(float(os.environ.get("PROBE_GB", "4")) * 1e9) // 4
    hip = ctypes.CDLL(native.hip_runtime_path())
    hip.hipMemRangeGetAttribute.argtypes = [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int,
                                            ctypes.c_void_p, ctypes.c_size_t]
    hip.hipMemAdvise.argtypes = [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int, ctypes.c_int]
    hip.hipMemPrefetchAsync.argtypes = [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int,
                                        ctypes.c_void_p]
    t = new_managed_tensor([n], torch.float32, 0)
    t.normal_()
    torch.cuda.synchronize()
    ptr, nbytes = t.data_ptr(), n * 4
    pinned = torch.empty(nbytes, dtype=torch.uint8, pin_memory=True)

    def attr(a):
        v = ctypes.c_int(-99)
        rc = hip.hipMemRangeGetAttribute(ctypes.byref(v), 4, a, ptr, nbytes)
        return v.value if rc == 0 else f"err{rc}"

    def gpu_read():
        torch.cuda.synchronize()
        best = 1e9
        for _ in range(3):
            t0 = time.perf_counter()
            t.sum()
            torch.cuda.synchronize()
            best = min(best, time.perf_counter() - t0)
        return nbytes / best / 1e9

    def cpu_read():
        best = 1e9
        for _ in range(2):
            t0 = time.perf_counter()
            ctypes.memmove(pinned.data_ptr(), ptr, nbytes)
            best = min(best, time.perf_counter() - t0)
        return nbytes / best / 1e9

    def report(state, **kw):
        print(json.dumps({"state": state, "GB": nbytes / 1e9,
                          "preferred": attr(2), "last_prefetch": attr(4),
                          "gpu_read_GBps": round(gpu_read(), 1),
                          "cpu_read_GBps": round(cpu_read(), 1),
                          "HSA_XNACK": os.environ.get("HSA_XNACK"), **kw}), flush=True)

    report("allocated+gpu_fill")
    s = torch.cuda.current_stream().cuda_stream
    rc1 = hip.hipMemAdvise(ptr, nbytes, 3, 0)
    rc2 = hip.hipMemPrefetchAsync(ptr, nbytes, 0, s)
    torch.cuda.synchronize()
    report("advise+prefetch gpu", advise_rc=rc1, prefetch_rc=rc2)
    rc1 = hip.hipMemAdvise(ptr, nbytes, 3, CPU)
    rc2 = hip.hipMemPrefetchAsync(ptr, nbytes, CPU, s)
    torch.cuda.synchronize()
    report("advise+prefetch cpu", advise_rc=rc1, prefetch_rc=rc2)


if __name__ == "__main__":
    main()
