"""fp8 quantize / dequantize kernels alone on 1 GiB of bf16 (for rocprofv3
--stats / --pmc passes): MX (E8M0 per 32), fp32 scale per 128, MFMA
Hadamard-32.  Prints one JSON line per kernel with host-timed GB/s of HBM
traffic (read + written bytes)."""

import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from hipsnapshot.ops import native, quant  # noqa: E402


def timeit(fn, iters=10):
    fn()
    torch.cuda.synchronize()
    ts = []
    for _ in range(iters):
        t0 = time.perf_counter()
        fn()
        torch.cuda.synchronize()
        ts.append(time.perf_counter() - t0)
    return min(ts), sorted(ts)[len(ts) // 2]


def main():
    dev = 0
    torch.cuda.set_device(dev)
    modes = sys.argv[1:] or ["mx_e8m0", "none", "hadamard32"]
    w = torch.empty(512 << 20, dtype=torch.bfloat16, device="cuda:0").normal_()
    nw = w.numel()
    hs = int(torch.cuda.current_stream().cuda_stream)
    for mode in modes:
        if mode == "mx_e8m0":
            info = quant.fp8_entry_quant_info(w, rotation="none")
        else:
            os.environ["HIPSNAPSHOT_FP8_SCALE"] = "fp32"
            info = quant.fp8_entry_quant_info(w, rotation=mode)
            del os.environ["HIPSNAPSHOT_FP8_SCALE"]
        blob = torch.zeros(info["total_bytes"], dtype=torch.uint8, device="cuda:0")
        p = info["payload_bytes"]
        sc = blob[p:] if mode == "mx_e8m0" else blob[p:].view(torch.float32)
        back = torch.empty_like(w)
        if mode == "mx_e8m0":
            q = lambda: native.mx8_quantize(dev, w, blob[:p], sc, hs)  # noqa: E731
            dq = lambda: native.mx8_dequantize(dev, blob[:nw], sc, back, hs)  # noqa: E731
        elif mode == "none":
            q = lambda: native.fp8_quantize(dev, w, blob[:p], sc, info["vpt"], hs)  # noqa: E731
            dq = lambda: native.fp8_dequantize(dev, blob[:nw], sc, back, info["vpt"], hs)  # noqa
        else:
            q = lambda: native.fp8_hadamard_quantize(dev, w, blob[:p], sc, hs)  # noqa: E731
            dq = lambda: native.fp8_hadamard_dequantize(dev, blob[:p], sc, back, hs)  # noqa
        traffic = nw * 2 + info["total_bytes"]
        for name, fn in (("quant", q), ("dequant", dq)):
            best, med = timeit(fn)
            print(json.dumps({"kernel": f"{name}_{mode}", "ms_best": round(best * 1e3, 4),
                              "TBps_best": round(traffic / best / 1e12, 3),
                              "TBps_median": round(traffic / med / 1e12, 3),
                              "traffic_bytes": traffic}), flush=True)
        del blob, back


if __name__ == "__main__":
    main()
