"""Host -> device copies from pinned memory: API blocking and throughput.

N threads each loop: hipMemcpyAsync(H2D, 46 MB, own copy stream) + stream
sync, like the restore consumers.  Prints per-N JSON with the aggregate
GB/s and the max / p50 time spent inside the (asynchronous) copy call.
"""

import json
import os
import statistics
import sys
import threading
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))

import torch  # noqa: E402

from hipsnapshot.ops import native  # noqa: E402


def main():
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    n = 46 << 20
    iters = 40
    serial = threading.Lock()
    for nthreads, locked in ((1, False), (4, False), (4, True), (8, False), (8, True)):
        bufs = [native.PinnedBuffer(n) for _ in range(nthreads)]
        dsts = [torch.empty(n, dtype=torch.uint8, device=dev) for _ in range(nthreads)]
        call_ms = []
        lock = threading.Lock()

        def work(i):
            torch.cuda.set_device(dev)
            slot = 20 + i
            for _ in range(iters):
                t0 = time.perf_counter()
                if locked:
                    with serial:
                        native.memcpy(0, slot, dsts[i].data_ptr(), bufs[i].ptr, n, native.H2D,
                                      None, sync=False)
                else:
                    native.memcpy(0, slot, dsts[i].data_ptr(), bufs[i].ptr, n, native.H2D, None,
                                  sync=False)
                t1 = time.perf_counter()
                native.stream_sync(0, slot)
                with lock:
                    call_ms.append((t1 - t0) * 1e3)

        work(0) if nthreads == 1 else None
        call_ms.clear()
        ths = [threading.Thread(target=work, args=(i,)) for i in range(nthreads)]
        t0 = time.perf_counter()
        for t in ths:
            t.start()
        for t in ths:
            t.join()
        dt = time.perf_counter() - t0
        print(json.dumps({"probe": "h2d_hipMemcpyAsync", "threads": nthreads, "locked": locked,
                          "GBps": round(nthreads * iters * n / dt / 1e9, 1),
                          "call_ms_p50": round(statistics.median(call_ms), 3),
                          "call_ms_max": round(max(call_ms), 3)}), flush=True)
        for b in bufs:
            b.release()


if __name__ == "__main__":
    main()
