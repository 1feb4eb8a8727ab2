"""HSZ1 decode of 1 GiB of bf16 in HBM (the restore's decode kernels):
host-timed rate of hsz_decode + hsz_decode2 over 20 launches, checked
bitwise.  Run under rocprofv3 --pmc for the LDS counters of hsz_decode2."""
import json
import os
import statistics
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch  # noqa: E402

from hipsnapshot.ops import codec, native  # noqa: E402

dev = 0
torch.cuda.set_device(dev)
g = torch.Generator(device="cuda:0").manual_seed(0)
for std in (0.02,):
    x = (torch.randn((1 << 30) // 2, device="cuda:0", generator=g) * std).to(torch.bfloat16)
    x = x.view(torch.uint8)
    st = torch.cuda.current_stream()
    out, total, meta = codec.encode_device(x, 2, int(st.cuda_stream))
    st.synchronize()
    nf = codec.n_frames_for(x.numel(), codec.DEFAULT_FRAME_BYTES)
    hdr = codec.parse_header(out[:codec.payload_start(nf)].cpu().numpy().tobytes())
    offs = torch.tensor(hdr.offsets, dtype=torch.int64, device="cuda:0")
    back = torch.empty_like(x)
    ts = []
    for _ in range(20):
        st.synchronize()
        t0 = time.perf_counter()
        native.hsz_decode_gpu(dev, out.data_ptr(), offs.data_ptr(), 0, hdr.n_frames,
                              hdr.logical_size, 2, hdr.frame_bytes, back.data_ptr(),
                              int(st.cuda_stream))
        st.synchronize()
        ts.append(time.perf_counter() - t0)
    ok = bool(torch.equal(back, x))
    print(json.dumps({"decode_1GiB_bf16_std": std, "ratio": round(int(total.item()) / x.numel(), 4),
                      "GBps_best": round(x.numel() / min(ts) / 1e9, 1),
                      "GBps_median": round(x.numel() / statistics.median(ts) / 1e9, 1),
                      "ms_best": round(min(ts) * 1e3, 3), "bitwise_ok": ok}), flush=True)
