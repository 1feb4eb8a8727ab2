"""hs64 device hash: kernel rate, and what it does to a concurrent SDMA copy.

Prints JSON lines:
  {"probe": "hash", "MB": .., "GBps": ..}       hash kernel alone (stream-timed)
  {"probe": "sdma", "alone_GBps": .., "with_hash_GBps": .., "with_encode_GBps": ..}
"""

import json
import os
import sys
import threading
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))

import torch  # noqa: E402

from hipsnapshot.ops import checksum, codec, native  # noqa: E402


def main():
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    for grid in (0, 16, 32, 64, 128, 256):
        for mb in (1, 16, 256):
            x = torch.randint(0, 256, (mb << 20,), dtype=torch.uint8, device=dev)
            torch.cuda.synchronize()
            h = checksum.device_hash_start(0, 9, x.data_ptr(), x.numel(), max_grid=grid)
            checksum.device_hash_result(0, 9, h, x.numel())
            reps = 20
            t0 = time.perf_counter()
            for _ in range(reps):
                h = checksum.device_hash_start(0, 9, x.data_ptr(), x.numel(), max_grid=grid)
                checksum.device_hash_result(0, 9, h, x.numel())
            dt = (time.perf_counter() - t0) / reps
            print(json.dumps({"probe": "hash", "grid": grid, "MB": mb,
                              "us": round(dt * 1e6, 1),
                              "GBps": round(x.numel() / dt / 1e9, 1)}), flush=True)

    n = 1 << 30
    src = torch.empty(n, dtype=torch.uint8, device=dev).random_(0, 255)
    pb = native.PinnedBuffer(n)
    cs = torch.cuda.Stream()

    def sdma_rate(reps=4):
        native.sdma_d2h(0, pb.ptr, src.data_ptr(), n, cs)
        t0 = time.perf_counter()
        for _ in range(reps):
            native.sdma_d2h(0, pb.ptr, src.data_ptr(), n, cs)
        return n * reps / (time.perf_counter() - t0) / 1e9

    out = {"probe": "sdma", "alone_GBps": round(sdma_rate(), 1)}
    y = torch.randint(0, 256, (256 << 20,), dtype=torch.uint8, device=dev)
    bf = (torch.randn(128 << 20, device=dev) * 0.02).to(torch.bfloat16).view(torch.uint8)
    es = torch.cuda.Stream()
    for what in ("hash0", "hash64", "hash128", "encode"):
        stop = threading.Event()
        count = [0]

        def load():
            torch.cuda.set_device(dev)
            while not stop.is_set():
                if what.startswith("hash"):
                    h = checksum.device_hash_start(0, 10, y.data_ptr(), y.numel(),
                                                   max_grid=int(what[4:]))
                    checksum.device_hash_result(0, 10, h, y.numel())
                    count[0] += y.numel()
                else:
                    codec.encode_device(bf, 2, int(es.cuda_stream))
                    es.synchronize()
                    count[0] += bf.numel()

        th = threading.Thread(target=load)
        th.start()
        time.sleep(0.2)
        t0 = time.perf_counter()
        c0 = count[0]
        r = sdma_rate(8)
        load_rate = (count[0] - c0) / (time.perf_counter() - t0) / 1e9
        stop.set()
        th.join()
        out[f"with_{what}_GBps"] = round(r, 1)
        out[f"{what}_load_GBps"] = round(load_rate, 1)
    print(json.dumps(out), flush=True)
    pb.release()


if __name__ == "__main__":
    main()
