#!/usr/bin/env python3
"""How fast can a host-resident UVM table be captured for an async take?

* GPU freeze (today's async path): the copy kernel reads the managed pages
  over PCIe into HBM on the trainer's stream.
* CPU capture: threads on the pages' NUMA node copy them into pinned host
  blocks (the trainer's stream would wait on a host flag meanwhile).

Prints one JSON object: GB/s per method and thread count, for ``--gb`` GB of
tables placed in host DRAM.
"""

import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gb", type=float, default=8.0)
    ap.add_argument("--tables", type=int, default=8)
    args = ap.parse_args()
    import torch

    from hipsnapshot.ops import native, uvm
    from hipsnapshot.utils.affinity import node_cpus, pages_node, threads_with_mask

    dev = 0
    per = int(args.gb * 1e9 / args.tables) // 4 * 4
    tabs = [uvm.new_managed_tensor([per // 4], torch.float32, dev) for _ in range(args.tables)]
    for t in tabs:
        t.normal_()
        uvm.place(t, "host")
    torch.cuda.synchronize()
    node = pages_node(tabs[0].data_ptr(), per)
    total = per * args.tables
    out = {"bytes": total, "tables": args.tables, "pages_node": node,
           "residency": sorted({uvm.residency(t) for t in tabs})}
    # GPU freeze: one copy kernel into an HBM arena (as hbm_staging does)
    arena = torch.empty(total, dtype=torch.uint8, device=f"cuda:{dev}")
    b = native.CopyBatch()
    for i, t in enumerate(tabs):
        b.add_tensor(t, arena.data_ptr() + i * per)
    arr = b.pack()
    times = []
    for _ in range(3):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        native.launch_packed(arr, dev, int(torch.cuda.current_stream(dev).cuda_stream), sync=True)
        torch.cuda.synchronize()
        times.append(time.perf_counter() - t0)
    out["gpu_freeze_GBps"] = round(total / min(times) / 1e9, 1)
    del arena
    # CPU capture into pinned blocks, threads on the pages' node
    pbs = [native.PinnedBuffer(per, node) for _ in tabs]
    mask = (node_cpus(node) & os.sched_getaffinity(0)) if node is not None else None
    lib = native.hsio()
    for nthreads in (16, 32):
        times = []
        for _ in range(5):
            t0 = time.perf_counter()
            with threads_with_mask(mask):
                import threading

                # one parallel copy per table, tables in parallel too
                k = max(1, nthreads // len(tabs))
                ths = [threading.Thread(target=lib.hsio_parallel_memcpy,
                                        args=(pb.ptr, t.data_ptr(), per, k))
                       for pb, t in zip(pbs, tabs)]
                for th in ths:
                    th.start()
                for th in ths:
                    th.join()
            times.append(time.perf_counter() - t0)
        out[f"cpu_capture_{nthreads}t_GBps"] = round(total / min(times) / 1e9, 1)
        out[f"cpu_capture_{nthreads}t_GBps_median"] = round(
            total / sorted(times)[len(times) // 2] / 1e9, 1)
    # the library's capture loop (engine/uvm_capture.py): 32 MiB pieces that
    # a pool of workers pulls, each worker on the pages' node
    import statistics
    import types

    from hipsnapshot.engine import uvm_capture
    from hipsnapshot.knobs import override_tuning

    uvm_capture.native.gate_release = lambda dev, v: None  # no gate armed here
    for nthreads in (16, 32):
        times = []
        for _ in range(5):
            cap = uvm_capture.Capture(dev, [(types.SimpleNamespace(), t, per) for t in tabs])
            cap.blocks = list(pbs)
            with override_tuning(uvm_capture_threads=nthreads):
                t0 = time.perf_counter()
                cap._run([])
                times.append(time.perf_counter() - t0)
            assert cap.error is None, cap.error
        out[f"pieces_{nthreads}t_GBps"] = round(total / min(times) / 1e9, 1)
        out[f"pieces_{nthreads}t_GBps_median"] = round(total / statistics.median(times) / 1e9, 1)
    ok = all(torch.equal(torch.frombuffer(pb.view, dtype=torch.float32)[: per // 4],
                         t.cpu()) for pb, t in zip(pbs, tabs))
    out["capture_bitwise"] = ok
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
