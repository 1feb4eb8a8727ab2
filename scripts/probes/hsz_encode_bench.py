"""HSZ1 encode of 1 GiB of bf16 in HBM (a blocking take's device encode):
host-timed rate of the whole encode over 20 launches.  Run under
rocprofv3 --kernel-trace --stats for the per-kernel split (analyze /
layout / encode / encode2x)."""
import json
import os
import statistics
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch  # noqa: E402

from hipsnapshot.ops import codec  # noqa: E402

torch.cuda.set_device(0)
g = torch.Generator(device="cuda:0").manual_seed(0)
x = (torch.randn((1 << 30) // 2, device="cuda:0", generator=g) * 0.02).to(torch.bfloat16)
x = x.view(torch.uint8)
st = torch.cuda.current_stream()
ts = []
for _ in range(20):
    st.synchronize()
    t0 = time.perf_counter()
    out, total, meta = codec.encode_device(x, 2, int(st.cuda_stream))
    st.synchronize()
    ts.append(time.perf_counter() - t0)
print(json.dumps({"encode_1GiB_bf16": True, "ratio": round(int(total.item()) / x.numel(), 4),
                  "GBps_best": round(x.numel() / min(ts) / 1e9, 1),
                  "GBps_median": round(x.numel() / statistics.median(ts) / 1e9, 1),
                  "ms_best": round(min(ts) * 1e3, 3)}), flush=True)
