#!/usr/bin/env python3
"""Native drain throughput with the GPU idle vs saturated by a GEMM loop,
with and without on-GPU blob hashing.

Question: in the training-overlap bench at seq 2048 a 48 GB drain took
11-14 s, against 3.5-6 s at seq 512 (profiles/r3/overlap/).  Which part of
the drain waits for the busy compute units -- the hs64 hash launches and
their result read-backs, or the SDMA copies?

    python scripts/drain_contention_probe.py --gb 8 --blob-mb 96
"""

from __future__ import annotations

import argparse
import json
import os
import shutil
import sys
import threading
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))

import torch  # noqa: E402

from hipsnapshot.ops import native  # noqa: E402


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--gb", type=float, default=8.0)
    ap.add_argument("--blob-mb", type=int, default=96)
    ap.add_argument("--dir", default=os.path.join(os.environ.get("HSBENCH_DIR", "/tmp"),
                                                  "drain_probe"))
    ap.add_argument("--gemm", type=int, default=8192)
    args = ap.parse_args()
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    total = int(args.gb * (1 << 30))
    arena = torch.empty(total, dtype=torch.uint8, device=dev)
    arena.view(torch.int32)[: total // 4].random_()
    blob = args.blob_mb << 20
    blobs = [(arena.data_ptr() + o, min(blob, total - o), os.path.join(args.dir, f"b{i}"))
             for i, o in enumerate(range(0, total, blob))]
    torch.cuda.synchronize()

    stop = threading.Event()
    a = torch.randn(args.gemm, args.gemm, device=dev, dtype=torch.bfloat16)
    b = torch.randn(args.gemm, args.gemm, device=dev, dtype=torch.bfloat16)
    gemms = [0]

    def busy():
        s = torch.cuda.Stream(dev)
        with torch.cuda.stream(s):
            while not stop.is_set():
                for _ in range(8):
                    torch.mm(a, b)
                gemms[0] += 8
                s.synchronize()

    def run(hash_blobs: bool, load: bool, high: bool = True) -> dict:
        shutil.rmtree(args.dir, ignore_errors=True)
        os.makedirs(args.dir, exist_ok=True)
        th = None
        if load:
            stop.clear()
            gemms[0] = 0
            th = threading.Thread(target=busy, daemon=True)
            th.start()
            time.sleep(0.5)
        g0 = gemms[0]
        t0 = time.perf_counter()
        job = native.NativeDrain(0, blobs, 32 << 20, 12, 8, False, hash_blobs, 16, nice=10,
                                 hash_high_priority=high)
        _, written = job.wait()
        dt = time.perf_counter() - t0
        g1 = gemms[0]
        if th is not None:
            stop.set()
            th.join()
        flops = 2 * args.gemm ** 3 * (g1 - g0) / dt
        return {"hash": hash_blobs, "hash_stream_high_prio": high if hash_blobs else None,
                "gemm_load": load, "s": round(dt, 3), "phases": job.stats,
                "GBps": round(written / dt / 1e9, 2),
                "gemm_TFLOPs_during": round(flops / 1e12, 1) if load else None}

    out = []
    for load in (False, True):
        for h, high in ((False, True), (True, False), (True, True)):
            run(h, load, high)  # warm (files exist: in-place overwrite as in the bench)
            out.append(run(h, load, high))
            print(json.dumps(out[-1]), flush=True)
    # the GEMM loop alone
    stop.clear()
    gemms[0] = 0
    th = threading.Thread(target=busy, daemon=True)
    th.start()
    time.sleep(0.5)
    g0, t0 = gemms[0], time.perf_counter()
    time.sleep(3.0)
    g1, dt = gemms[0], time.perf_counter() - t0
    stop.set()
    th.join()
    print(json.dumps({"gemm_alone_TFLOPs": round(2 * args.gemm ** 3 * (g1 - g0) / dt / 1e12, 1)}))
    shutil.rmtree(args.dir, ignore_errors=True)


if __name__ == "__main__":
    main()
