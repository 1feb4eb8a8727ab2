"""Interleaved A/B of the mode-2 decoders (HIPSNAPSHOT_HSZ_DECODE2, read per
launch) in one process: for each blob size, rounds of 10 timed decodes per
variant, variants alternating, every output checked bitwise.  One JSON line
per (size, variant)."""
import json
import os
import statistics
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch  # noqa: E402

from hipsnapshot.ops import codec, native  # noqa: E402

VARIANTS = os.environ.get("VARIANTS", "lds staged staged-pf").split()
SIZES = [int(s) << 20 for s in os.environ.get("SIZES_MIB", "1024 64").split()]
dev = 0
torch.cuda.set_device(dev)
g = torch.Generator(device="cuda:0").manual_seed(0)
st = torch.cuda.current_stream()
for size in SIZES:
    x = (torch.randn(size // 2, device="cuda:0", generator=g) * 0.02).to(torch.bfloat16)
    x = x.view(torch.uint8)
    out, total, meta = codec.encode_device(x, 2, int(st.cuda_stream))
    st.synchronize()
    nf = codec.n_frames_for(x.numel(), codec.DEFAULT_FRAME_BYTES)
    hdr = codec.parse_header(out[:codec.payload_start(nf)].cpu().numpy().tobytes())
    offs = torch.tensor(hdr.offsets, dtype=torch.int64, device="cuda:0")
    back = torch.empty_like(x)
    ts = {v: [] for v in VARIANTS}
    ok = {v: True for v in VARIANTS}
    for _rnd in range(4):
        for v in VARIANTS:
            os.environ["HIPSNAPSHOT_HSZ_DECODE2"] = v
            back.zero_()
            for _ in range(10):
                st.synchronize()
                t0 = time.perf_counter()
                native.hsz_decode_gpu(dev, out.data_ptr(), offs.data_ptr(), 0, hdr.n_frames,
                                      hdr.logical_size, 2, hdr.frame_bytes, back.data_ptr(),
                                      int(st.cuda_stream))
                st.synchronize()
                ts[v].append(time.perf_counter() - t0)
            ok[v] = ok[v] and bool(torch.equal(back, x))
    for v in VARIANTS:
        print(json.dumps({"MiB": size >> 20, "variant": v, "frames": hdr.n_frames,
                          "GBps_best": round(size / min(ts[v]) / 1e9, 1),
                          "GBps_median": round(size / statistics.median(ts[v]) / 1e9, 1),
                          "ms_median": round(statistics.median(ts[v]) * 1e3, 3),
                          "bitwise_ok": ok[v]}), flush=True)
    del x, out, back, offs
