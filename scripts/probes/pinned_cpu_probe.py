"""Host-side speed of pinned (hipHostMalloc) vs pageable buffers.

pread() of a page-cached 1 GiB file into the buffer and pwrite() from it,
16 threads x 8 MiB pieces (like the native I/O engine), plus a plain
numpy copy into / out of the buffer.  One JSON line.
"""

import json
import os
import sys
import threading
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))

import numpy as np  # noqa: E402
import torch  # noqa: E402

from hipsnapshot.ops import native  # noqa: E402


def par_io(fn, fd, mv, nthreads=16, piece=8 << 20):
    n = len(mv)
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
            fn(fd, mv[o:o + piece], o)

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
    torch.cuda.init()
    path = os.path.join(d, "pinned_probe.bin")
    with open(path, "wb") as f:
        f.write(os.urandom(1 << 20) * 1024)
    fd = os.open(path, os.O_RDWR)
    pb = native.PinnedBuffer(n)
    pinned = pb.view
    page = memoryview(bytearray(n))
    out = {}
    for name, mv in (("pinned", pinned), ("pageable", page)):
        par_io(lambda fd, m, o: os.preadv(fd, [m], o), fd, mv)  # warm
        out[f"pread_{name}_GBps"] = round(par_io(lambda fd, m, o: os.preadv(fd, [m], o), fd, mv), 1)
        out[f"pwrite_{name}_GBps"] = round(par_io(lambda fd, m, o: os.pwritev(fd, [m], o), fd, mv), 1)
        a = np.frombuffer(mv, dtype=np.uint8)
        src = np.ones(n, dtype=np.uint8)
        t0 = time.perf_counter()
        np.copyto(a, src)
        out[f"np_copy_into_{name}_GBps"] = round(n / (time.perf_counter() - t0) / 1e9, 1)
        t0 = time.perf_counter()
        np.copyto(src, a)
        out[f"np_copy_from_{name}_GBps"] = round(n / (time.perf_counter() - t0) / 1e9, 1)
    os.close(fd)
    os.remove(path)
    pb.release()
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
