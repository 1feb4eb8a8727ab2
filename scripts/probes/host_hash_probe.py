#!/usr/bin/env python3
"""Host hs64 (csrc/hschk.cpp) against a plain memcpy, one thread, on a 1 GiB
buffer (DRAM-resident, not cache): what hashing a host-staged blob costs
the writer's CPU budget.  Prints one JSON line."""

import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))

import torch  # noqa: E402

from hipsnapshot.ops import native  # noqa: E402


def best(fn, reps=5):
    out = []
    for _ in range(reps):
        t0 = time.perf_counter()
        fn()
        out.append(time.perf_counter() - t0)
    return min(out)


def main():
    lib = native.hsio()
    n = 1 << 30
    src = torch.randint(0, 256, (n,), dtype=torch.uint8)
    dst = torch.empty_like(src)
    p, q = src.data_ptr(), dst.data_ptr()
    res = {"bytes": n, "cpu": open("/proc/cpuinfo").read().split("model name")[1].split("\n")[0]
           .strip(" :\t")}
    for th in (1, 2, 4):
        res[f"hash_{th}t_GBps"] = round(n / best(lambda: lib.hs64_partial(p, n, 0, th)) / 1e9, 2)
    res["memcpy_1t_GBps"] = round(n / best(lambda: lib.hsio_parallel_memcpy(q, p, n, 1)) / 1e9, 2)
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
