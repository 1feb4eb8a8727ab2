"""D2H bandwidth of the data-plane memcpy (1 GiB, pinned) -- run under
different HIP runtime settings to see which copy engine configuration
reaches the PCIe rate."""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch  # noqa: E402

from hipsnapshot.ops import native  # noqa: E402

n = 1 << 30
src = torch.empty(n, dtype=torch.uint8, device="cuda:0").random_(0, 255)
pb = native.PinnedBuffer(n)
for _ in range(2):
    native.memcpy(0, 0, pb.ptr, src.data_ptr(), n, native.D2H, None, sync=True)
ts = []
for _ in range(5):
    t0 = time.perf_counter()
    native.memcpy(0, 0, pb.ptr, src.data_ptr(), n, native.D2H, None, sync=True)
    ts.append(time.perf_counter() - t0)
# the same copy while a GEMM loop keeps every CU busy on another stream
a = torch.randn(8192, 8192, device="cuda:0", dtype=torch.bfloat16)
s2 = torch.cuda.Stream()
torch.cuda.synchronize()
with torch.cuda.stream(s2):
    for _ in range(40):
        a = (a @ a).clamp_(-1, 1)
t0 = time.perf_counter()
native.memcpy(0, 0, pb.ptr, src.data_ptr(), n, native.D2H, None, sync=True)
busy = time.perf_counter() - t0
ev = torch.cuda.Event(enable_timing=True)
ev2 = torch.cuda.Event(enable_timing=True)
torch.cuda.synchronize()
ev.record(s2)
with torch.cuda.stream(s2):
    for _ in range(40):
        a = (a @ a).clamp_(-1, 1)
ev2.record(s2)
torch.cuda.synchronize()
gemm_alone = ev.elapsed_time(ev2)
print(json.dumps({"env": {k: v for k, v in os.environ.items() if k.startswith(("GPU_", "DEBUG_CLR", "HSA_", "ROC_"))},
                  "d2h_GBps": n / min(ts) / 1e9, "d2h_under_gemm_GBps": n / busy / 1e9,
                  "gemm40_ms": gemm_alone}), flush=True)
