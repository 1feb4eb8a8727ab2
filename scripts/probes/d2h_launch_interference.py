"""Does a saturating D2H stream slow down LAUNCH-BOUND GPU work?

``d2h_interference.py`` showed that a concurrent D2H costs a long bf16 GEMM
only ~1.5 %.  Training steps also contain thousands of short kernels whose
cost is dominated by dispatch: the command processor fetches every AQL packet
(and, unless HIP_FORCE_DEV_KERNARG, its kernel arguments) from host memory over
the same PCIe link that a drain saturates with device->host writes.  This
probe times three workloads on the default stream alone and while a
background thread streams 256 MiB D2H copies (pinned host memory, the data
plane's memcpy) at full rate and at rate limits:

* ``tiny``   3000 x add_ on 1 K floats (pure dispatch latency)
* ``medium`` 600 x add_ on 16 M floats (~HBM-bound, ~20 us each)
* ``gemm``   100 x 2048^2 bf16 matmul

Prints one JSON line per (rate limit) with the slowdown of each workload.
"""
import json
import os
import sys
import threading
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch  # noqa: E402

from hipsnapshot.ops import native  # noqa: E402

CHUNK = 256 << 20
src = torch.empty(CHUNK, dtype=torch.uint8, device="cuda:0").random_(0, 255)
pb = native.PinnedBuffer(CHUNK)
cs = torch.cuda.Stream()
ws = torch.cuda.Stream()  # the "training" workload's stream


SDMA = os.environ.get("PROBE_KIND") == "sdma"


def d2h_chunk():
    if SDMA:  # ROCr copy engines (csrc/hsdma.hip)
        native.sdma_d2h(0, pb.ptr, src.data_ptr(), CHUNK, cs)
    else:  # hipMemcpyAsync: the runtime's blit kernel
        native.memcpy(0, 0, pb.ptr, src.data_ptr(), CHUNK, native.D2H, int(cs.cuda_stream),
                      sync=True)


tiny = torch.zeros(1024, device="cuda:0")
med = torch.zeros(16 << 20, device="cuda:0")
ga = torch.randn(2048, 2048, device="cuda:0", dtype=torch.bfloat16)


def w_tiny():
    for _ in range(3000):
        tiny.add_(1.0)


def w_medium():
    for _ in range(600):
        med.add_(1.0)


def w_gemm():
    for _ in range(100):
        torch.mm(ga, ga)


WORK = {"tiny": w_tiny, "medium": w_medium, "gemm": w_gemm}


def timed(fn, reps=6):
    """Mean over reps (a rate-limited copier is idle part of the time: the
    mean, not the minimum, is what a training loop experiences)."""
    tot = 0.0
    for _ in range(reps):
        # stream-local syncs: a device-wide sync would also wait for the
        # copier's in-flight chunks and measure the copy, not the workload
        ws.synchronize()
        t0 = time.perf_counter()
        with torch.cuda.stream(ws):
            fn()
        ws.synchronize()
        tot += time.perf_counter() - t0
    return tot / reps * 1e3


def measure(limit_gbps):
    """Workload times while a copier thread runs (None = no copier)."""
    stop = threading.Event()
    moved = [0]

    def copier():
        t_start = time.perf_counter()
        while not stop.is_set():
            d2h_chunk()
            moved[0] += CHUNK
            if limit_gbps:
                ahead = moved[0] / (limit_gbps * 1e9) - (time.perf_counter() - t_start)
                if ahead > 0:
                    time.sleep(ahead)

    th = None
    if limit_gbps is not None:
        th = threading.Thread(target=copier, daemon=True)
        th.start()
        time.sleep(0.2)
    t0 = time.perf_counter()
    res = {k: timed(f) for k, f in WORK.items()}
    el = time.perf_counter() - t0
    if th is not None:
        stop.set()
        th.join()
        res["d2h_GBps"] = round(moved[0] / (el + 0.2) / 1e9, 1)
    return res


# correctness of the copy path under test
d2h_chunk()
assert torch.equal(torch.frombuffer(pb.view[:1 << 20], dtype=torch.uint8),
                   src[:1 << 20].cpu()), "D2H copy produced wrong bytes"
with torch.cuda.stream(ws):
    for f in WORK.values():  # warm up
        f()
torch.cuda.synchronize()
base = measure(None)
env = {k: v for k, v in os.environ.items()
       if k.startswith(("GPU_", "HSA_", "HIP_FORCE", "ROC_", "PROBE_"))}
print(json.dumps({"env": env, "limit_GBps": "none (no D2H)",
                  **{k: round(v, 2) for k, v in base.items()}}), flush=True)
for lim in (0, 40, 25, 10):
    r = measure(lim)
    print(json.dumps({"env": env, "limit_GBps": lim or "unlimited",
                      **{k: (round(v, 2) if k == "d2h_GBps" else
                             f"{v:.2f} ms ({v / base[k] - 1:+.1%})") for k, v in r.items()}}),
          flush=True)
