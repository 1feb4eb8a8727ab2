#!/usr/bin/env python3
"""DLRM with large row-wise sharded embedding tables on managed (UVM) memory.

BASELINE config 4 (TorchRec DLRM, 100 GB tables, uvm_tensor path); reference
script /root/reference/benchmarks/torchrec/main.py:54-151 (sync vs async take,
time-to-unblock).  Tables are DTensors over the ranks in the ``--sharding``
layout (row = Shard(0), column = Shard(1), table = each table whole on one
rank, round-robin); ``--uvm`` puts every local shard in hipMallocManaged
memory.
"""

import argparse
import os
import shutil
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

from common import Timer, emit, init_dist, log, max_over_ranks, sync  # noqa: E402
from hipsnapshot import Snapshot  # noqa: E402
from hipsnapshot.models.dlrm import DLRM  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--total-gb", type=float, default=8.0, help="total embedding bytes (all ranks)")
    ap.add_argument("--tables", type=int, default=8)
    ap.add_argument("--dim", type=int, default=128)
    ap.add_argument("--uvm", action="store_true")
    ap.add_argument("--sharding", default="row", choices=["row", "column", "table"])
    ap.add_argument("--uvm-place", default=None, choices=["host", "device"],
                    help="advise + prefetch the UVM tables to host DRAM or HBM first")
    ap.add_argument("--work-dir", default=os.environ.get("HSBENCH_DIR", "/tmp"))
    ap.add_argument("--host-siblings", type=int, default=0,
                    help="K host-only processes replaying the other ranks' host work (one "
                         "staging pass + the same blob bytes written) with every timed take: "
                         "one rank's share of a (K+1)-GPU node sharing this host")
    ap.add_argument("--single-path", action="store_true",
                    help="every take rewrites ONE snapshot path (100 GB runs: one copy on storage)")
    args = ap.parse_args()
    rank, ws, dev = init_dist()
    from torch.distributed.device_mesh import init_device_mesh

    mesh = init_device_mesh(dev.type, (ws,))
    rows = int(args.total_gb * 1e9 / 4 / args.dim / args.tables)
    model = DLRM([rows] * args.tables, dim=args.dim, device=dev, mesh=mesh, uvm=args.uvm,
                 sharding=args.sharding)
    nbytes = sum(p.numel() * 4 for p in model.parameters())
    residency = None
    if args.uvm:
        from hipsnapshot.ops.uvm import is_uvm_tensor, place, residency as uvm_residency

        locals_ = [t for t in (getattr(p, "_local_tensor", p) for p in model.parameters())
                   if is_uvm_tensor(t)]
        if args.uvm_place:
            for t in locals_:
                if t.numel():
                    place(t, args.uvm_place)
            torch.cuda.synchronize()
        residency = sorted({uvm_residency(t) for t in locals_ if t.numel()})
    log(f"DLRM: {args.tables} tables x {rows} rows x {args.dim} (uvm={args.uvm}, "
        f"{args.sharding}-wise), "
        f"{nbytes / 1e9:.2f} GB")
    root = os.path.join(args.work_dir, "hs_dlrm")
    if rank == 0:
        shutil.rmtree(root, ignore_errors=True)
    sync(dev)
    p_warm, p_sync, p_async = ((root + "/ckpt",) * 3 if args.single_path
                               else (root + "/warm", root + "/sync", root + "/async"))
    Snapshot.take(p_warm, {"model": model})
    sync(dev)
    sib = None
    if args.host_siblings > 0:
        from common import Siblings
        from hipsnapshot import knobs

        knobs.set_local_ranks_hint(args.host_siblings + 1)
        # what one sibling rank writes per take: this rank's blob sizes
        sizes = [os.path.getsize(os.path.join(dp, f)) for dp, _, fs in os.walk(p_warm)
                 for f in fs if not f.startswith(".")]
        sib_root = os.environ.get("HSBENCH_SIBLING_DIR") or os.path.join(root, "siblings")
        sib = Siblings(args.host_siblings, sizes, sib_root, True)
    sib_ms = []
    with Timer() as t:
        if sib is not None:
            sib.go()
        Snapshot.take(p_sync, {"model": model})
        sync(dev)
    sync_s = max_over_ranks(t.s, dev)
    if sib is not None:
        sib_ms.append(max(x[0] for x in sib.wait()) * 1e3)
    sync(dev)
    # the first async_take of a state builds its plan: untimed, reported as cold
    with Timer() as tc:
        Snapshot.async_take(p_async, {"model": model}).wait()
    cold_s = max_over_ranks(tc.s, dev)
    sync(dev)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    with Timer() as ta:
        with Timer() as tu:
            if sib is not None:
                sib.go()
            pending = Snapshot.async_take(p_async, {"model": model})
        e1.record()
        e1.synchronize()
        pending.wait()
    freeze_ms = e0.elapsed_time(e1)  # the trainer stream's busy time (HBM freeze)
    unblock = max_over_ranks(tu.s, dev)
    async_total = max_over_ranks(ta.s, dev)
    if sib is not None:
        sib_ms.append(max(x[0] for x in sib.wait()) * 1e3)
        sib.stop()
    sync(dev)
    restore_s = None
    if os.environ.get("DLRM_RESTORE", "1") == "1":
        refs = [getattr(p, "_local_tensor", p).detach().clone() for p in model.parameters()]
        with torch.no_grad():
            for p in model.parameters():
                getattr(p, "_local_tensor", p).zero_()
        sync(dev)
        with Timer() as tr:
            Snapshot(p_sync).restore({"model": model})
            sync(dev)
        restore_s = max_over_ranks(tr.s, dev)
        ok = all(torch.equal(r, getattr(p, "_local_tensor", p))
                 for r, p in zip(refs, model.parameters()))
        del refs
    else:
        ok = None
    emit({"bench": "dlrm_uvm" if args.uvm else "dlrm_hbm", "sharding": args.sharding,
          "world_size": ws, "bytes": nbytes,
          "sync_take_s": round(sync_s, 3), "sync_GBps": round(nbytes / sync_s / 1e9, 2),
          "async_unblock_ms": round(unblock * 1e3, 1), "freeze_gpu_ms": round(freeze_ms, 2),
          "async_total_s": round(async_total, 3),
          "async_GBps": round(nbytes / async_total / 1e9, 2),
          "host_siblings": args.host_siblings, "sibling_take_ms": [round(x, 1) for x in sib_ms],
          "cold_async_total_s": round(cold_s, 3), "single_path": args.single_path,
          "uvm_residency": residency, "uvm_place": args.uvm_place,
          "restore_s": round(restore_s, 3) if restore_s else None,
          "restore_GBps": round(nbytes / restore_s / 1e9, 2) if restore_s else None,
          "restore_bitwise_ok": ok})
    if rank == 0:
        shutil.rmtree(root, ignore_errors=True)
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
