"""Does a D2H copy take compute away from training?  Times a bf16 GEMM loop
alone and while 1 GiB D2H copies (the data plane's memcpy, pinned host
memory) run from another thread, and the D2H bandwidth in both cases.  Run
under different HIP runtime settings (GPU_BLIT_ENGINE_TYPE, HSA_ENABLE_SDMA)
to see whether the copy runs as blit kernels on the CUs or on SDMA."""
import json
import os
import sys
import threading
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch  # noqa: E402

from hipsnapshot.ops import native  # noqa: E402

n = 1 << 30
src = torch.empty(n, dtype=torch.uint8, device="cuda:0").random_(0, 255)
pb = native.PinnedBuffer(n)
cs = torch.cuda.Stream()


def d2h():
    native.memcpy(0, 0, pb.ptr, src.data_ptr(), n, native.D2H, int(cs.cuda_stream), sync=True)


for _ in range(2):
    d2h()
t0 = time.perf_counter()
for _ in range(4):
    d2h()
alone_gbps = 4 * n / (time.perf_counter() - t0) / 1e9

a = torch.randn(8192, 8192, device="cuda:0", dtype=torch.bfloat16)
s2 = torch.cuda.Stream()


def gemm_ms(iters=60):
    global a
    ev, ev2 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    ev.record(s2)
    with torch.cuda.stream(s2):
        for _ in range(iters):
            a = (a @ a).clamp_(-1, 1)
    ev2.record(s2)
    ev2.synchronize()
    return ev.elapsed_time(ev2)


gemm_ms()
g_alone = min(gemm_ms() for _ in range(3))
done = threading.Event()
copied = [0]


def copier():
    while not done.is_set():
        d2h()
        copied[0] += n


th = threading.Thread(target=copier)
t0 = time.perf_counter()
th.start()
g_busy = min(gemm_ms() for _ in range(3))
done.set()
th.join()
busy_gbps = copied[0] / (time.perf_counter() - t0) / 1e9
print(json.dumps({"env": {k: v for k, v in os.environ.items()
                          if k.startswith(("GPU_BLIT", "HSA_ENABLE_SDMA", "GPU_FORCE"))},
                  "d2h_GBps": round(alone_gbps, 1), "d2h_during_gemm_GBps": round(busy_gbps, 1),
                  "gemm60_ms": round(g_alone, 1), "gemm60_with_d2h_ms": round(g_busy, 1),
                  "gemm_slowdown": round(g_busy / g_alone - 1, 3)}), flush=True)
