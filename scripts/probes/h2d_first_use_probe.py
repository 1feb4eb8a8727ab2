"""Is the first hipMemcpyAsync H2D from a pinned block slow?

For fresh 46 MB pinned blocks: time of the copy call + sync on first use,
on second use, after a 1-byte warm-up copy, and after the block was first
used by the SDMA D2H path.  One JSON line.
"""

import json
import os
import statistics
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))

import torch  # noqa: E402

from hipsnapshot.ops import native  # noqa: E402


def timed_h2d(dst, pb, n):
    t0 = time.perf_counter()
    native.memcpy(0, 3, dst.data_ptr(), pb.ptr, n, native.H2D, None, sync=False)
    t1 = time.perf_counter()
    native.stream_sync(0, 3)
    return (t1 - t0) * 1e3, (time.perf_counter() - t0) * 1e3


def main():
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    n = 46 << 20
    dst = torch.empty(n, dtype=torch.uint8, device=dev)
    src = torch.empty(n, dtype=torch.uint8, device=dev)
    out = {}
    lib = native.require_gpu_lib()
    for case in ("fresh", "warm1", "after_sdma"):
        first_call, first_total, second_total = [], [], []
        for _ in range(6):
            # a never-pooled block: hipHostMalloc directly through the pool
            # with an odd size so no cached block fits
            pb = native.PinnedBuffer(n + 4096 * (len(first_call) + 1) + 123)
            if case == "warm1":
                native.memcpy(0, 3, dst.data_ptr(), pb.ptr, 1, native.H2D, None, sync=True)
            elif case == "after_sdma":
                native.sdma_d2h(0, pb.ptr, src.data_ptr(), n, 0)
            c, t = timed_h2d(dst, pb, n)
            first_call.append(c)
            first_total.append(t)
            second_total.append(timed_h2d(dst, pb, n)[1])
            pb.release()
            lib.hsg_pinned_trim()
        out[case] = {"first_call_ms": round(statistics.median(first_call), 2),
                     "first_total_ms": round(statistics.median(first_total), 2),
                     "second_total_ms": round(statistics.median(second_total), 2)}
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
