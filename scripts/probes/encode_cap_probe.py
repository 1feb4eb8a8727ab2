"""HSZ1 encode throughput (bf16 logical bytes) vs the thread grid cap."""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch  # noqa: E402

from hipsnapshot.ops import codec, native  # noqa: E402

x = (torch.randn(512 << 20, device="cuda:0") * 0.02).to(torch.bfloat16).view(torch.uint8)  # 1 GiB
s = torch.cuda.Stream()
out, total, meta = codec.encode_device(x, 2, int(s.cuda_stream))
s.synchronize()
for cap in (0, 512, 256, 128, 64, 32, 16):
    native.set_thread_grid_cap(cap)
    codec.launch_encode(x, 2, int(s.cuda_stream), codec.DEFAULT_FRAME_BYTES, out, total, meta)
    s.synchronize()
    t0 = time.perf_counter()
    for _ in range(5):
        codec.launch_encode(x, 2, int(s.cuda_stream), codec.DEFAULT_FRAME_BYTES, out, total, meta)
    s.synchronize()
    gbps = 5 * x.numel() / (time.perf_counter() - t0) / 1e9
    print(json.dumps({"grid_cap": cap, "encode_GBps_logical": round(gbps, 1)}), flush=True)
