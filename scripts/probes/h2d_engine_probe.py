"""Pinned-host -> HBM upload bandwidth: hipMemcpyAsync into ordinary device
memory vs one SDMA request (csrc/hsdma.hip) into an uncached block vs into
ordinary device memory, vs the same bytes split over 2 / 4 concurrent SDMA
requests (one thread each; ROCr spreads them over its engines).  Sizes 16 MiB
.. 1 GiB; every upload is checked against the source once.  One JSON line per
(mode, size)."""
import json
import os
import statistics
import sys
import threading
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch  # noqa: E402

from hipsnapshot.ops import native  # noqa: E402

dev = 0
torch.cuda.set_device(dev)
N = 1 << 30
pb = native.PinnedBuffer(N)
host = torch.frombuffer(pb.view, dtype=torch.uint8)
host.copy_(torch.randint(0, 255, (N,), dtype=torch.uint8))
plain = torch.empty(N, dtype=torch.uint8, device="cuda:0")
ub = native.UncachedBlock(dev, N)
print(json.dumps({"sdma_engines": native.sdma_engines(dev)}), flush=True)


def split_sdma(dst: int, n: int, k: int) -> None:
    part = (n // k + 4095) // 4096 * 4096
    ths = []
    for i in range(k):
        lo = i * part
        ln = min(part, n - lo)
        if ln <= 0:
            break
        ths.append(threading.Thread(target=native.sdma_h2d, args=(dev, dst + lo, pb.ptr + lo, ln)))
    for t in ths:
        t.start()
    for t in ths:
        t.join()


def hip(n: int) -> None:
    native.memcpy(dev, 0, plain.data_ptr(), pb.ptr, n, native.H2D, None, sync=True)


modes = {
    "hip_plain": hip,
    "sdma_uncached": lambda n: native.sdma_h2d(dev, ub.ptr, pb.ptr, n),
    "sdma_plain": lambda n: native.sdma_h2d(dev, plain.data_ptr(), pb.ptr, n),
    "sdma_uncached_x2": lambda n: split_sdma(ub.ptr, n, 2),
    "sdma_uncached_x4": lambda n: split_sdma(ub.ptr, n, 4),
}


def check(mode: str, n: int) -> bool:
    if mode.startswith("sdma_uncached"):
        got = torch.empty(n, dtype=torch.uint8, device="cuda:0")
        native.memcpy(dev, 0, got.data_ptr(), ub.ptr, n, native.D2D, None, sync=True)
        return bool(torch.equal(got.cpu(), host[:n]))
    torch.cuda.synchronize()
    return bool(torch.equal(plain[:n].cpu(), host[:n]))


for size in (16 << 20, 64 << 20, 256 << 20, 1 << 30):
    for mode, fn in modes.items():
        fn(size)
        ok = check(mode, size)
        ts = []
        for _ in range(6 if size >= (256 << 20) else 20):
            t0 = time.perf_counter()
            fn(size)
            ts.append(time.perf_counter() - t0)
        print(json.dumps({"mode": mode, "bytes": size, "ok": ok,
                          "GBps_median": round(size / statistics.median(ts) / 1e9, 2),
                          "GBps_best": round(size / min(ts) / 1e9, 2)}), flush=True)
