"""Device -> pinned-host copy bandwidth: hipMemcpyAsync (runtime blit kernel)
vs the ROCr SDMA engines (csrc/hsdma.hip) with 1..all engines; every copy is
checked byte for byte against the source."""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch  # noqa: E402

from hipsnapshot.ops import native  # noqa: E402

n_eng = native.sdma_engines(0)
print(json.dumps({"sdma_engines": n_eng}), flush=True)
N = 1 << 30
src = torch.empty(N, dtype=torch.uint8, device="cuda:0").random_(0, 255)
pb = native.PinnedBuffer(N)
host = torch.frombuffer(pb.view, dtype=torch.uint8)
s = torch.cuda.Stream()


def run(fn, n, reps=4):
    fn(n)
    host[:n].zero_()
    fn(n)
    ok = torch.equal(host[:n], src[:n].cpu())
    t0 = time.perf_counter()
    for _ in range(reps):
        fn(n)
    return reps * n / (time.perf_counter() - t0) / 1e9, ok


def blit(n):
    native.memcpy(0, 0, pb.ptr, src.data_ptr(), n, native.D2H, int(s.cuda_stream), sync=True)


for n in (16 << 20, 256 << 20, N):
    row = {"MiB": n >> 20}
    row["blit_GBps"], row["blit_ok"] = run(blit, n)
    g, ok = run(lambda m: native.sdma_d2h(0, pb.ptr, src.data_ptr(), m, s), n)
    row["sdma_auto_GBps"], row["sdma_auto_ok"] = round(g, 1), ok
    for k in sorted({1, 2, 4, n_eng} - {0}):
        if k > n_eng:
            continue
        g, ok = run(lambda m, k=k: native.sdma_d2h(0, pb.ptr, src.data_ptr(), m, s, k), n)
        row[f"sdma{k}_GBps"], row[f"sdma{k}_ok"] = round(g, 1), ok
    row["blit_GBps"] = round(row["blit_GBps"], 1)
    print(json.dumps(row), flush=True)
