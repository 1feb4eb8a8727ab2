"""One rank's share of the Llama-3 FSDP save at world size W, on one GPU.

At N GPUs every rank saves 1/N of every parameter: the same 291 tensors,
each 1/N the size.  Per-take fixed costs (planning per tensor, per-blob
launch and DMA latencies, commit) do not shrink with N, so they decide the
scaling efficiency the 8-GPU node will show.  This benchmark builds exactly
that share on one GPU -- each parameter's world-W local shard (dim 0 split
like FSDP2's Shard(0)) as a DTensor over a 1-rank mesh, so the take goes
through the same DTensor / sharded-entry path -- and times take, async_take
unblock and restore.

It leaves out what only a real N-GPU run has: collectives across ranks and
N ranks sharing host memory bandwidth.  ``ideal_aggregate_GBps`` = N x the
share's bytes / the share's take time, the upper bound if nothing else
interfered.

``--host-siblings K`` adds the host side of the other ranks: K processes
(no GPU) replay, for every timed take, what a sibling rank's take does to
the host -- a write pass over its staging memory standing in for the D2H
DMA (``--sibling-dma-pass``), then the same blob sizes written through the
same native FS engine (same I/O thread count) into their own directories --
started together with the GPU rank's take.  ``contended_take_ms_median`` vs
``take_ms_median`` is the cost of N ranks sharing this host's CPUs and
memory bandwidth; ``contended_aggregate_GBps`` replaces the solo predictor.

    python benchmarks/rank_share/main.py --world 8 [--compression hsz1]
    python benchmarks/rank_share/main.py --model llama3_70b --world 8   # BASELINE config 5's share
"""

from __future__ import annotations

import argparse
import json
import os
import shutil
import statistics
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from common import Siblings as _Siblings, cpu_s as _cpu_s  # noqa: E402


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--world", type=int, default=8)
    ap.add_argument("--model", default="llama3_8b", choices=["llama3_8b", "llama3_70b"])
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--async-iters", type=int, default=5)
    ap.add_argument("--restore-iters", type=int, default=3)
    ap.add_argument("--compression", default="hsz1", choices=["none", "hsz1"])
    ap.add_argument("--dir", default=os.environ.get("HSBENCH_DIR", "/tmp"))
    ap.add_argument("--ab", default=None,
                    help="NAME=v1,v2[,...]: alternate env var NAME over the values take by "
                         "take (same process, interleaved) and report each value's takes")
    ap.add_argument("--host-siblings", type=int, default=0,
                    help="K host-only processes replaying sibling ranks' host work per take")
    ap.add_argument("--sibling-dma-pass", type=int, default=1,
                    help="siblings write their staging memory once per take (DMA stand-in)")
    ap.add_argument("--no-numa-bind", action="store_true",
                    help="leave the process unbound (a real rank binds to its GPU's NUMA "
                         "node, as bench.py does)")
    ap.add_argument("--switch-interval", type=float, default=None,
                    help="sys.setswitchinterval for the run (GIL hand-over latency)")
    args = ap.parse_args()
    if args.switch_interval:
        sys.setswitchinterval(args.switch_interval)

    import torch
    import torch.distributed as dist
    from torch.distributed.device_mesh import init_device_mesh
    from torch.distributed.tensor import DTensor, Shard

    from hipsnapshot import Snapshot, StateDict
    from hipsnapshot.models.llama import Llama, LlamaConfig

    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ.setdefault("MASTER_PORT", "29533")
    os.environ.update(RANK="0", WORLD_SIZE="1")
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    numa = None
    if not args.no_numa_bind:
        from hipsnapshot.utils.affinity import bind_to_gpu_numa

        numa = bind_to_gpu_numa(0)
    dist.init_process_group("nccl", device_id=dev)
    mesh = init_device_mesh("cuda", (1,))
    cfg = getattr(LlamaConfig, args.model)()
    with torch.device("meta"):
        meta = Llama(cfg)
    gen = torch.Generator(device=dev).manual_seed(0)
    params = {}
    for name, p in meta.named_parameters():
        rows = -(-p.shape[0] // args.world)
        local = torch.randn((rows,) + tuple(p.shape[1:]), device=dev, generator=gen)
        local = (local * 0.02).to(torch.bfloat16)
        params[name] = DTensor.from_local(local, mesh, [Shard(0)], run_check=False)
    del meta
    share = sum(t._local_tensor.numel() * 2 for t in params.values())
    app_state = {"model": StateDict(**params)}
    root = os.path.join(args.dir, f"rank_share_w{args.world}")
    shutil.rmtree(root, ignore_errors=True)
    path = os.path.join(root, "ckpt")
    torch.cuda.synchronize()

    def take():
        Snapshot.take(path, app_state, compression=args.compression)

    ab_name, ab_vals = None, [None]
    if args.ab:
        ab_name, vals = args.ab.split("=", 1)
        ab_vals = vals.split(",")
    for _ in range(args.warmup):
        for v in ab_vals:
            if ab_name:
                os.environ[ab_name] = v
            take()
    sib = None
    if args.host_siblings > 0:
        # this host runs world ranks: size I/O threads as a real W-rank job
        # would (the take's first collective sets the same hint)
        from hipsnapshot import knobs

        knobs.set_local_ranks_hint(args.host_siblings + 1)
        sizes = [os.path.getsize(os.path.join(r, f)) for r, _, fs in os.walk(path)
                 for f in fs if not f.startswith(".")]
        sib = _Siblings(args.host_siblings, sizes, root, bool(args.sibling_dma_pass))
        for _ in range(2):  # warm their engines / page cache
            sib.go()
            sib.wait()
    times = []
    contended = []
    per_val = {v: [] for v in ab_vals}
    cpu0 = _cpu_s()
    for _ in range(args.steps):
        for v in ab_vals:
            if ab_name:
                os.environ[ab_name] = v
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            take()
            dt = time.perf_counter() - t0
            per_val[v].append(dt)
            times.append(dt)
    if ab_name:
        print(json.dumps({"bench": "rank_share_ab", "world": args.world, "knob": ab_name,
                          "compression": args.compression,
                          "take_ms": {v: {"median": round(statistics.median(t) * 1e3, 2),
                                          "min": round(min(t) * 1e3, 2),
                                          "mean": round(statistics.mean(t) * 1e3, 2)}
                                      for v, t in per_val.items()}}), flush=True)
        os.environ[ab_name] = ab_vals[0]
    solo_cpu_s = (_cpu_s() - cpu0) / max(1, len(times))
    stored = sum(os.path.getsize(os.path.join(r, f)) for r, _, fs in os.walk(path)
                 for f in fs if not f.startswith("."))
    sib_ms = []
    sib_cpu = []
    cont_cpu = []
    if sib is not None:
        for _ in range(args.steps):
            torch.cuda.synchronize()
            sib.go()
            c0 = _cpu_s()
            t0 = time.perf_counter()
            take()
            contended.append(time.perf_counter() - t0)
            cont_cpu.append(_cpu_s() - c0)
            got = sib.wait()
            sib_ms.append(max(g[0] for g in got) * 1e3)
            sib_cpu.append(statistics.mean(g[1] for g in got))
        sib.stop()
    unblock, total = [], []
    for _ in range(args.async_iters):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        pending = Snapshot.async_take(path + "_async", app_state, compression=args.compression)
        unblock.append(time.perf_counter() - t0)
        pending.wait()
        total.append(time.perf_counter() - t0)
    from hipsnapshot import memory_held
    from hipsnapshot.utils import rank_diag

    held_after_takes = memory_held(dev.index or 0)  # what stays between checkpoints
    diag = rank_diag.measure(take)  # one more take with its phases captured
    refs = {k: v._local_tensor.clone() for k, v in params.items()}
    rtimes = []
    r_per_val = {v: [] for v in ab_vals}
    r_stats = {}
    for _ in range(args.restore_iters):
        for val in ab_vals:
            if ab_name:
                os.environ[ab_name] = val
            for v in params.values():
                v._local_tensor.zero_()
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            Snapshot(path).restore(app_state)
            torch.cuda.synchronize()
            rtimes.append(time.perf_counter() - t0)
            r_per_val[val].append(rtimes[-1])
            r_stats[val] = _native_restore_stats()
    if ab_name and args.restore_iters > 1:
        print(json.dumps({"bench": "rank_share_restore_ab", "world": args.world,
                          "knob": ab_name, "compression": args.compression,
                          "restore_ms": {v: {"median": round(statistics.median(t) * 1e3, 2),
                                             "min": round(min(t) * 1e3, 2)}
                                         for v, t in r_per_val.items()},
                          "native_restore_stats": r_stats}), flush=True)
        os.environ[ab_name] = ab_vals[0]
    ok = all(torch.equal(refs[k], app_state["model"][k]._local_tensor) for k in refs)
    med = statistics.median(times)
    print(json.dumps({
        "bench": "rank_share", "model": args.model, "world": args.world, "compression": args.compression,
        "tensors": len(params), "share_bytes": share,
        "take_ms_median": round(med * 1e3, 2), "take_ms_min": round(min(times) * 1e3, 2),
        "share_GBps": round(share / med / 1e9, 2),
        "ideal_aggregate_GBps": round(args.world * share / med / 1e9, 1),
        # the first async_take of the state builds its plan: reported apart
        "unblock_ms_median": (round(statistics.median(unblock[1:] or unblock) * 1e3, 2)
                              if unblock else None),
        "cold_unblock_ms": round(unblock[0] * 1e3, 2) if unblock else None,
        "async_total_ms_median": round(statistics.median(total) * 1e3, 2) if total else None,
        "restore_ms_median": round(statistics.median(rtimes) * 1e3, 2),
        "restore_bitwise_ok": ok,
        "native_restore_stats": _native_restore_stats(),
        "hbm_held_between_takes_bytes": held_after_takes["hbm_held_bytes"],
        "pinned_held_bytes": held_after_takes["pinned_held_bytes"],
        "memory_held_after_takes": held_after_takes,
        "memory_held_after_restore": memory_held(dev.index or 0),
        "rank_diag": diag,
        "numa_bind": numa,
        # host CPU time (user + system, every thread of the process) per take
        # and per stored GB; the kernel's page-cache writeback threads are
        # not charged to the process
        "stored_bytes": stored,
        "take_cpu_s": round(solo_cpu_s, 4),
        "take_cpu_s_per_stored_GB": round(solo_cpu_s / (stored / 1e9), 4) if stored else None,
        **({"host_siblings": args.host_siblings, "sibling_dma_pass": bool(args.sibling_dma_pass),
            "sibling_bytes_each": sum(sib.sizes),
            "contended_take_ms_median": round(statistics.median(contended) * 1e3, 2),
            "contended_take_ms_each": [round(t * 1e3, 1) for t in contended],
            "sibling_host_ms_median": round(statistics.median(sib_ms), 2),
            "contended_vs_solo": round(statistics.median(contended) / med, 3),
            "contended_take_cpu_s_per_stored_GB": round(
                statistics.median(cont_cpu) / (stored / 1e9), 4) if stored else None,
            "sibling_cpu_s_per_GB": round(statistics.median(sib_cpu) / (sum(sib.sizes) / 1e9), 4),
            "contended_aggregate_GBps": round(
                args.world * share / max(statistics.median(contended),
                                         statistics.median(sib_ms) / 1e3) / 1e9, 1)}
           if sib is not None else {}),
    }), flush=True)
    shutil.rmtree(root, ignore_errors=True)
    dist.destroy_process_group()


def _native_restore_stats() -> dict:
    from hipsnapshot.engine import native_restore

    return dict(native_restore.last_stats)


if __name__ == "__main__":
    main()
