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
import time
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
    ap.add_argument("--sync-repeats", type=int, default=1,
                    help="timed sync takes (the median is reported); each one's phase split, "
                         "page-cache state and page faults go to sync_each")
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
    sync_each = []
    from hipsnapshot.utils import rank_diag

    for _ in range(max(1, args.sync_repeats)):
        before = _host_state()
        nodes_before = _node_state()
        cg0 = _cgroup_cpu()
        hb0 = _host_busy()
        if sib is not None:
            sib.go()
        d = rank_diag.measure(lambda: (Snapshot.take(p_sync, {"model": model}), sync(dev)))
        hb1 = _host_busy()
        cg1 = _cgroup_cpu()
        wall = max(d["take_ms"] / 1e3, 1e-6)
        # the whole host's busy CPUs per node during the take (this job's
        # included: ``cgroup.usage_usec`` / wall is this job's share)
        d["host_busy_cpus"] = {n: round((hb1[n] - hb0.get(n, 0)) / _HZ / wall, 1) for n in hb1}
        after = _host_state()
        # the job's CPU quota: periods throttled and the whole cgroup's CPU
        # time during this take (other processes of the job included)
        d["cgroup"] = {k: cg1[k] - cg0[k] for k in cg0 if isinstance(cg0[k], int) and k in cg1}
        d["take_s"] = max_over_ranks(d["take_ms"] / 1e3, dev)
        d["GBps"] = round(nbytes / d["take_s"] / 1e9, 2)
        d["dirty_kB_before"], d["writeback_kB_before"] = before["Dirty"], before["Writeback"]
        d["dirty_kB_after"] = after["Dirty"]
        d["minflt"] = after["minflt"] - before["minflt"]
        d["majflt"] = after["majflt"] - before["majflt"]
        d["nodes_before"] = nodes_before
        sync_each.append(d)
        if sib is not None:
            sib_ms.append(max(x[0] for x in sib.wait()) * 1e3)
        sync(dev)
    sync_s = sorted(x["take_s"] for x in sync_each)[len(sync_each) // 2]
    uvm_numa = None
    if args.uvm:
        uvm_numa = _numa_pages([(t.data_ptr(), t.numel() * t.element_size()) for t in locals_
                                if t.numel()])
    # the first async_take of a state builds its plan: untimed, reported as cold
    with Timer() as tc:
        Snapshot.async_take(p_async, {"model": model}).wait()
    cold_s = max_over_ranks(tc.s, dev)
    sync(dev)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    cg0 = _cgroup_cpu()
    with Timer() as ta:
        with Timer() as tu:
            if sib is not None:
                sib.go()
            pending = Snapshot.async_take(p_async, {"model": model})
        e1.record()
        e1.synchronize()
        pending.wait()
    freeze_ms = e0.elapsed_time(e1)  # the trainer stream's busy time (HBM freeze)
    cg1 = _cgroup_cpu()
    async_cgroup = {k: cg1[k] - cg0[k] for k in cg0 if isinstance(cg0[k], int) and k in cg1}
    async_cgroup["cpu_max"] = cg1.get("cpu_max")
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
          "sync_GBps_each": [x["GBps"] for x in sync_each], "sync_each": sync_each,
          "uvm_pages_per_numa_node": uvm_numa,
          "writer_cpus": rank_diag.cpu_set(), "writer_cpu_nodes": _cpu_nodes(),
          "async_unblock_ms": round(unblock * 1e3, 1), "freeze_gpu_ms": round(freeze_ms, 2),
          "async_total_s": round(async_total, 3),
          "uvm_capture_stats": _capture_stats(),
          # CPU time and CFS throttling of the job's cgroup over the async take
          "async_cgroup": async_cgroup,
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


def _capture_stats() -> dict:
    """The last async take's CPU capture of host UVM tables (seconds)."""
    from hipsnapshot.engine import uvm_capture
    from hipsnapshot.utils.affinity import pages_node

    out = {k: round(v, 4) for k, v in uvm_capture.last.items() if isinstance(v, (int, float))}
    tables = uvm_capture.last.get("tables") or []
    if tables:
        thp = _thp_of([ptr for *_x, ptr in tables])
        out["tables"] = [
            {"GB": round(n / 1e9, 3), "s": round(s, 4), "GBps": round(n / max(s, 1e-9) / 1e9, 1),
             "src_node": node, "dst_node": pages_node(ptr, n), "dst_thp_frac": thp.get(ptr)}
            for n, s, node, ptr in tables]
    return out


_HZ = os.sysconf("SC_CLK_TCK") if hasattr(os, "sysconf") else 100


def _host_busy() -> dict:
    """Busy CPU jiffies (all but idle and iowait) per NUMA node, summed over
    every CPU of the host (/proc/stat): load from other tenants shows here."""
    node_of = {}
    for n, ids in _node_cpu_ids().items():
        for c in ids:
            node_of[c] = n
    out: dict = {}
    try:
        with open("/proc/stat") as f:
            for line in f:
                if not line.startswith("cpu") or line.startswith("cpu "):
                    continue
                parts = line.split()
                c = int(parts[0][3:])
                v = [int(x) for x in parts[1:9]]
                busy = sum(v) - v[3] - v[4]
                n = node_of.get(c, "?")
                out[n] = out.get(n, 0) + busy
    except (OSError, ValueError):
        pass
    return out


def _node_cpu_ids() -> dict:
    base = "/sys/devices/system/node"
    out: dict = {}
    try:
        nodes = [d for d in os.listdir(base) if d.startswith("node")]
    except OSError:
        return out
    for d in nodes:
        try:
            with open(f"{base}/{d}/cpulist") as f:
                spec = f.read().strip()
        except OSError:
            continue
        ids = set()
        for part in spec.split(","):
            if "-" in part:
                a, b = part.split("-")
                ids.update(range(int(a), int(b) + 1))
            elif part:
                ids.add(int(part))
        out[d] = ids
    return out


def _cgroup_cpu() -> dict:
    """The cgroup's CPU quota and usage / throttling counters (cgroup v2)."""
    out: dict = {}
    try:
        with open("/sys/fs/cgroup/cpu.stat") as f:
            for line in f:
                k, v = line.split()
                if k in ("usage_usec", "nr_periods", "nr_throttled", "throttled_usec"):
                    out[k] = int(v)
        with open("/sys/fs/cgroup/cpu.max") as f:
            out["cpu_max"] = f.read().strip()
    except (OSError, ValueError):
        pass
    return out


def _thp_of(ptrs) -> dict:
    """Fraction of the mapping holding each address that is backed by
    transparent huge pages (/proc/self/smaps AnonHugePages / Size)."""
    want = sorted(set(ptrs))
    out, cur = {}, None
    try:
        with open("/proc/self/smaps") as f:
            for line in f:
                head = line.split(None, 1)[0]
                if "-" in head and not head.endswith(":"):
                    lo, hi = (int(x, 16) for x in head.split("-"))
                    cur = [p for p in want if lo <= p < hi] or None
                    size = hi - lo
                elif cur and head == "AnonHugePages:":
                    kb = int(line.split()[1])
                    for p in cur:
                        out[p] = round(kb * 1024 / max(size, 1), 3)
    except OSError:
        pass
    return out


def _host_state() -> dict:
    """Page-cache dirt (kB) and this process's page faults so far."""
    import resource

    out = {"Dirty": None, "Writeback": None}
    try:
        with open("/proc/meminfo") as f:
            for line in f:
                k, v = line.split(":", 1)
                if k in out:
                    out[k] = int(v.split()[0])
    except OSError:
        pass
    ru = resource.getrusage(resource.RUSAGE_SELF)
    out["minflt"], out["majflt"] = ru.ru_minflt, ru.ru_majflt
    return out


def _node_state() -> dict:
    """Per NUMA node: free memory and page cache (kB, from sysfs), and the
    rate (GB/s) one thread on that node copies 256 MiB between buffers it
    first-touched there -- what the machine leaves a writer on each node."""
    import threading

    import numpy as np

    base = "/sys/devices/system/node"
    out: dict = {}
    try:
        nodes = sorted(d for d in os.listdir(base) if d.startswith("node"))
    except OSError:
        return out
    for d in nodes:
        info = {}
        try:
            with open(f"{base}/{d}/meminfo") as f:
                for line in f:
                    parts = line.split()
                    if len(parts) >= 4 and parts[2].rstrip(":") in ("MemFree", "FilePages",
                                                                      "Dirty"):
                        info[parts[2].rstrip(":")] = int(parts[3])
        except OSError:
            pass
        try:
            from hipsnapshot.utils.affinity import node_cpus

            cpus = node_cpus(int(d[4:])) & os.sched_getaffinity(0)
        except Exception:  # noqa: BLE001
            cpus = set()
        if cpus:
            res = {}

            def copy_on_node(cpus=cpus, res=res):
                os.sched_setaffinity(0, cpus)  # this thread only
                a = np.ones(256 << 20, dtype=np.uint8)
                b = np.empty_like(a)
                np.copyto(b, a)
                t0 = time.perf_counter()
                for _ in range(4):
                    np.copyto(b, a)
                res["GBps"] = round(4 * a.nbytes / (time.perf_counter() - t0) / 1e9, 2)

            th = threading.Thread(target=copy_on_node)
            th.start()
            th.join()
            info["copy_GBps_1thread"] = res.get("GBps")
        out[d] = info
    return out


def _numa_pages(ranges) -> dict:
    """Pages of the managed tables per NUMA node (/proc/self/numa_maps)."""
    out: dict = {}
    try:
        with open("/proc/self/numa_maps") as f:
            lines = f.readlines()
    except OSError:
        return out
    for line in lines:
        parts = line.split()
        try:
            start = int(parts[0], 16)
        except (ValueError, IndexError):
            continue
        if not any(lo <= start < lo + n for lo, n in ranges):
            continue
        for p in parts[1:]:
            if p.startswith("N") and "=" in p:
                node, cnt = p[1:].split("=", 1)
                out[f"N{node}"] = out.get(f"N{node}", 0) + int(cnt)
    return out


def _cpu_nodes() -> dict:
    """NUMA node of each CPU this process may run on (count per node)."""
    out: dict = {}
    cpus = os.sched_getaffinity(0)
    base = "/sys/devices/system/node"
    try:
        nodes = [d for d in os.listdir(base) if d.startswith("node")]
    except OSError:
        return out
    for d in nodes:
        try:
            with open(f"{base}/{d}/cpulist") as f:
                spec = f.read().strip()
        except OSError:
            continue
        ids = set()
        for part in spec.split(","):
            if "-" in part:
                a, b = part.split("-")
                ids.update(range(int(a), int(b) + 1))
            elif part:
                ids.add(int(part))
        n = len(ids & cpus)
        if n:
            out[d] = n
    return out


if __name__ == "__main__":
    main()
