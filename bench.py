#!/usr/bin/env python3
"""Headline benchmark: checkpoint save GB/s + time-to-unblock, Llama-3-8B FSDP.

BASELINE.json metric: "checkpoint save GB/s + time-to-unblock, Llama-3-8B FSDP
at 1/2/4/8 MI355X".  One *step* = one ``Snapshot.take`` of the full FSDP2
(DTensor, Shard(0)) Llama-3-8B model state (8.03 B bf16 params = 16.06 GB,
random init, synthetic) to local storage, committed (metadata written after
every rank finished).  The total model is fixed as N grows -> strong scaling;
``value`` is the whole-job GB/s = model bytes / step time (max over ranks).

After the timed steps, ``async_take`` is run ``--async-warmup`` times untimed
(the first async take of a state builds its plan: ``cold_time_to_unblock_ms``)
and then ``--async-iters`` times; its time-to-unblock (max over ranks, median
over the iterations) is reported in ``time_to_unblock_ms`` (every iteration in
``time_to_unblock_ms_each``); then
every local shard is zeroed, restored, and compared bitwise to a copy.

Blobs are written with the lossless HSZ1 codec by default (``--compression``):
the GPU Huffman-codes each bf16's sign+exponent byte before the D2H, so ~67 %
of the bytes cross PCIe and hit storage.  ``value`` is always LOGICAL model
bytes / step time; ``stored_bytes`` reports what was written.  The same save
with raw, reference-format blobs is timed afterwards (``--raw-steps``) and
reported as ``raw_GBps``; ``--compression none`` makes raw blobs the headline.

Self-audit keys next to the headline (each with its step count):

* ``freeze_gpu_ms`` -- event-timed GPU time from the start of ``async_take``
  to the end of the HBM freeze it enqueues on the trainer's stream (includes
  the host planning before the launch); ``freeze_kernel_ms`` -- the freeze
  launch alone; ``unblock_incl_freeze_ms``: host time until that stream is
  free again;
* ``fresh_path_GBps`` -- the same take into a NEW ``step_<i>/`` directory each
  time (fresh files, as a training loop writes them); the headline rewrites
  one path;
* ``vs_baseline`` (= ``vs_baseline_same_config``) -- the reference's own
  published config (DDP, 200 x 100 MB fp32 params = 20 GB, replicated, raw
  blobs) timed in the same run, vs its 13.91 s (1 GPU) / 3.38 s (8 GPUs);
  null at 2 and 4 GPUs, where the reference publishes nothing.

BASELINE configs 2 and 3 run in the same command:

* ``ddp_llama_*`` -- Llama-3-8B under DDP, bf16, ``replicated=["**"]``: the
  partitioner splits the replicated state so each rank writes ~1/N of the
  bytes (raw blobs), restore checked bitwise through per-parameter hashes;
* ``elastic_*`` (N >= 2, N even) -- the FSDP checkpoint written by the N
  ranks above restored into N/2 ranks (a fresh FSDP2 model on an N/2 mesh of
  a ``dist.new_group``), every shard checked bitwise against hashes of the
  N-rank shards it was cut from.

Launch: ``python bench.py --gpus N`` starts N ranks itself (one process per
GPU, the parent never touches the GPU) and forwards rank 0's JSON line; a
failing or hung rank fails the whole run.  Under torchrun
(``python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N``)
WORLD_SIZE must equal ``--gpus``.
"""

from __future__ import annotations

import argparse
import json
import os
import shutil
import signal
import socket
import statistics
import subprocess
import sys
import threading
import time

# published reference numbers: DDP 20 GB save on p4d.24xlarge,
# local FS -- 1 GPU 13.91 s (1.44 GB/s), 1 node x 8 GPUs 3.38 s (5.92 GB/s)
REF_DDP_S = {1: 13.91, 8: 3.38}  # the same DDP 20 GB config, seconds per save


def _free_port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _default_dir() -> str:
    for cand in (os.environ.get("HSBENCH_DIR"), "/var/tmp", "/tmp"):
        if cand and os.path.isdir(cand) and os.access(cand, os.W_OK):
            return os.path.join(cand, "hipsnapshot_bench")
    return "hipsnapshot_bench"


def _drain_stats():
    from hipsnapshot.engine import native_drain

    return dict(native_drain.last_stats) or None


def _hash_tensor(t, dev: int) -> int:
    """hs64 of a contiguous device tensor's bytes (the blob-checksum kernel)."""
    import torch

    from hipsnapshot.ops import checksum

    n = t.numel() * t.element_size()
    if n == 0:
        return 0
    assert t.is_contiguous()
    torch.cuda.synchronize()
    h = checksum.device_hash_start(dev, 0, t.data_ptr(), n)
    return checksum.device_hash_result(dev, 0, h, n)


def _shard_hashes(model, dev: int) -> dict:
    """{param: (global row offset, rows, hs64)} of this rank's FSDP shards."""
    from torch.distributed.tensor._utils import compute_local_shape_and_global_offset

    out = {}
    for name, p in model.named_parameters():
        loc = p._local_tensor
        _, off = compute_local_shape_and_global_offset(p.shape, p.device_mesh, p.placements)
        rows = int(loc.shape[0]) if loc.dim() else 0
        out[name] = (int(off[0]) if len(off) else 0, rows, _hash_tensor(loc, dev))
    return out


def _check_resharded(model, old: list, dev: int) -> list:
    """Compare every restored shard, piece by piece, with the hashes of the
    shards it was cut from (``old``: every saving rank's ``_shard_hashes``).
    Returns the mismatches."""
    from torch.distributed.tensor._utils import compute_local_shape_and_global_offset

    bad = []
    for name, p in model.named_parameters():
        loc = p._local_tensor
        _, off = compute_local_shape_and_global_offset(p.shape, p.device_mesh, p.placements)
        lo = int(off[0]) if len(off) else 0
        rows = int(loc.shape[0]) if loc.dim() else 0
        covered = 0
        for o, n, h in sorted(r[name] for r in old):
            if n == 0 or o + n <= lo or o >= lo + rows:
                continue
            if o < lo or o + n > lo + rows:  # N -> N/2 of Shard(0): whole pieces
                bad.append((name, "piece straddles the new shard"))
                continue
            covered += n
            if _hash_tensor(loc.narrow(0, o - lo, n), dev) != h:
                bad.append((name, o))
        if covered != rows:
            bad.append((name, f"{covered} of {rows} rows covered"))
    return bad


def _hsdp_phase(cfg, dev, gpu_index, world, rank, reps, root, opts, args, total_bytes,
                barrier_sync, log) -> dict:
    """The model under HSDP on a (reps, world / reps) mesh: timed takes,
    per-rank written bytes, and a bitwise restore of every local shard."""
    import statistics

    import torch
    import torch.distributed as dist
    from torch.distributed.device_mesh import init_device_mesh

    from hipsnapshot import Snapshot, release_hbm_arena
    from hipsnapshot.models.llama import build_fsdp_llama
    from hipsnapshot.snapshot import TakeStats

    release_hbm_arena()
    mesh = init_device_mesh("cuda", (reps, world // reps), mesh_dim_names=("rep", "shard"))
    model = build_fsdp_llama(cfg, dev, torch.bfloat16, mesh=mesh)
    # replicas start identical: each shard-group member takes replica 0's bytes
    rep_group = mesh.get_group("rep")
    with torch.no_grad():
        for p in model.parameters():
            dist.broadcast(p._local_tensor, group=rep_group, group_src=0)
    torch.cuda.synchronize()
    path = os.path.join(root, "hsdp")
    app = {"model": model}
    Snapshot.take(path, app, storage_options=opts, compression=args.compression)
    each, mine = [], []
    for _ in range(max(1, args.hsdp_steps)):
        barrier_sync()
        t0 = time.perf_counter()
        Snapshot.take(path, app, storage_options=opts, compression=args.compression)
        mine.append(time.perf_counter() - t0)
        barrier_sync()
        e = torch.tensor([time.perf_counter() - t0], dtype=torch.float64, device=dev)
        dist.all_reduce(e, op=dist.ReduceOp.MAX)
        each.append(float(e.item()))
    written = int(TakeStats.last.get("bytes", 0))
    before = {n: _hash_tensor(p._local_tensor, gpu_index) for n, p in model.named_parameters()}
    for p in model.parameters():
        p._local_tensor.zero_()
    barrier_sync()
    t0 = time.perf_counter()
    Snapshot(path).restore(app)
    barrier_sync()
    restore_s = time.perf_counter() - t0
    bad = sum(_hash_tensor(p._local_tensor, gpu_index) != before[n]
              for n, p in model.named_parameters())
    per = [None] * world
    dist.all_gather_object(per, (written, statistics.mean(mine) * 1e3, bad))
    wr = [r[0] for r in per]
    # the model's logical bytes: one copy of the global state
    logical = sum(p.numel() * p.element_size() for p in model.parameters())
    out = {
        "hsdp_mesh": [reps, world // reps],
        "hsdp_GBps": round(logical / statistics.median(each) / 1e9, 2),
        "hsdp_s_each": [round(x, 3) for x in each],
        "hsdp_rank_written_bytes": wr,
        "hsdp_rank_written_max_over_mean": round(max(wr) / (sum(wr) / world), 3) if sum(wr)
        else None,
        "hsdp_rank_take_ms": [round(r[1], 1) for r in per],
        "hsdp_restore_GBps": round(logical / restore_s / 1e9, 2),
        "hsdp_restore_bitwise_ok": all(r[2] == 0 for r in per),
    }
    log(f"HSDP {reps}x{world // reps}: {out}")
    del model, app
    torch.cuda.empty_cache()
    if rank == 0:
        shutil.rmtree(path, ignore_errors=True)
    dist.barrier()
    return out


def _selftest_hook(rank: int) -> None:
    """``HSBENCH_SELFTEST`` (launcher tests on CPU, before any
    torch import): ``ok`` -- rank 0 prints a JSON line, every rank exits 0;
    ``fail:<r>`` -- rank r exits 3 at once, the others block as a rank stuck
    in the rendezvous would."""
    mode = os.environ.get("HSBENCH_SELFTEST")
    if not mode:
        return
    if mode == "ok":
        if rank == 0:
            print(json.dumps({"metric": "selftest", "n_gpus": int(os.environ["WORLD_SIZE"])}),
                  flush=True)
        sys.exit(0)
    if mode.startswith("fail:") and rank == int(mode.split(":")[1]):
        sys.exit(3)
    time.sleep(3600)
    sys.exit(0)


def _launch_ranks(n: int, argv: list, timeout_s: float) -> int:
    """Start ``n`` ranks of this script (RANK/LOCAL_RANK/WORLD_SIZE/MASTER_*
    set, one process group each) and forward rank 0's stdout.  The first rank
    to fail, or the timeout, ends every rank; returns the exit code."""
    port = _free_port()
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n),
                   LOCAL_WORLD_SIZE=str(n), GROUP_RANK="0", MASTER_ADDR="127.0.0.1",
                   MASTER_PORT=str(port))
        procs.append(subprocess.Popen(
            [sys.executable, "-u", os.path.abspath(__file__)] + argv, env=env,
            stdout=subprocess.PIPE if r == 0 else None, start_new_session=True))

    def pump() -> None:
        for line in iter(procs[0].stdout.readline, b""):
            sys.stdout.write(line.decode(errors="replace"))
            sys.stdout.flush()

    out = threading.Thread(target=pump, daemon=True)
    out.start()

    def kill_all() -> None:
        for sig in (signal.SIGTERM, signal.SIGKILL):
            for p in procs:
                if p.poll() is None:
                    try:
                        os.killpg(p.pid, sig)
                    except ProcessLookupError:
                        pass
            t_end = time.monotonic() + 10
            while time.monotonic() < t_end and any(p.poll() is None for p in procs):
                time.sleep(0.1)

    deadline = time.monotonic() + timeout_s
    rc = 0
    try:
        while True:
            codes = [p.poll() for p in procs]
            bad = [(r, c) for r, c in enumerate(codes) if c not in (None, 0)]
            if bad:
                r, rc = bad[0]
                print(f"bench launcher: rank {r} exited with {rc}; stopping every rank",
                      file=sys.stderr, flush=True)
                break
            if all(c == 0 for c in codes):
                break
            if time.monotonic() > deadline:
                print(f"bench launcher: timed out after {timeout_s:.0f} s; stopping every rank",
                      file=sys.stderr, flush=True)
                rc = 124
                break
            time.sleep(0.2)
    finally:
        kill_all()
        out.join(timeout=5)
    return rc


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--model", default="llama3_8b", choices=["llama3_8b", "llama3_70b", "tiny"])
    ap.add_argument("--path", default=None)
    ap.add_argument("--async-iters", type=int, default=3)
    ap.add_argument("--async-warmup", type=int, default=1,
                    help="untimed async_takes before the timed ones (the first builds the "
                         "async take plan and runs the one full GC pass that follows a plan "
                         "build); their unblock is reported as cold_time_to_unblock_ms")
    ap.add_argument("--no-restore-check", action="store_true")
    ap.add_argument("--raw-steps", type=int, default=3,
                    help="after the headline, also time this many takes with raw "
                         "(reference-format, uncompressed) blobs -> raw_GBps (0 = skip)")
    ap.add_argument("--restore-iters", type=int, default=3,
                    help="restores to time (median reported); each is checked bitwise")
    ap.add_argument("--verify-iters", type=int, default=2,
                    help="restores with verify=True (every blob checked against the take's "
                         "checksums) -> restore_verify_GBps (0 = skip)")
    ap.add_argument("--fresh-steps", type=int, default=3,
                    help="takes to a NEW step_<i>/ directory each (as a training loop "
                         "writes them), timed one by one -> fresh_path_GBps (0 = skip)")
    ap.add_argument("--ddp-steps", type=int, default=2,
                    help="timed takes of the reference's own DDP config (200 x 100 MB fp32 "
                         "params, replicated, raw blobs) -> vs_baseline_same_config (0 = skip)")
    ap.add_argument("--fsync", action="store_true")
    ap.add_argument("--direct-io", action="store_true")
    ap.add_argument("--backend", default="nccl", choices=["nccl", "gloo"])
    ap.add_argument("--no-numa-bind", action="store_true",
                    help="do not restrict the rank to the CPUs of its GPU's NUMA node")
    ap.add_argument("--compression", default="hsz1", choices=["none", "hsz1"],
                    help="hsz1 (default) = lossless GPU-side exponent-nibble compression of "
                         "the bf16 blobs, restore verified bitwise; none = raw blobs "
                         "(reference-compatible format)")
    ap.add_argument("--ddp-llama-steps", type=int, default=2,
                    help="BASELINE config 2: timed takes of the model under DDP, bf16, "
                         "replicated=['**'] (partitioned across ranks, raw blobs) (0 = skip)")
    ap.add_argument("--ddp-llama-layers", type=int, default=None,
                    help="layers of the DDP model (default: all; a gloo rehearsal of 8 ranks "
                         "on one GPU cannot hold 8 replicas + DDP buckets of Llama-3-8B)")
    ap.add_argument("--elastic-iters", type=int, default=1,
                    help="BASELINE config 3 (N >= 2, N even): restores of the N-rank FSDP "
                         "checkpoint into N/2 ranks, each checked bitwise (0 = skip)")
    ap.add_argument("--hsdp", type=int, default=None,
                    help="HSDP phase: the model on a (R, N/R) (replicate, shard) mesh, each "
                         "replicated box written by the R replicas in row ranges "
                         "(io/sharded.py); reports per-rank written bytes and a bitwise "
                         "restore (default R = 2 when N >= 4 is even, 0 = skip)")
    ap.add_argument("--hsdp-steps", type=int, default=2)
    ap.add_argument("--launch-timeout", type=float, default=3600.0,
                    help="self-launched ranks (--gpus N > 1 without torchrun): seconds before "
                         "every rank is stopped and the run fails")
    ap.add_argument("--no-plan-gc", action="store_true",
                    help="A/B probe: skip the full GC pass after a take that built a plan "
                         "(knobs.TUNING.gc_after_plan)")
    args = ap.parse_args()

    torchrun = "RANK" in os.environ and "WORLD_SIZE" in os.environ
    if not torchrun and args.gpus > 1:
        # one process per GPU; this parent never initialises the GPU
        sys.exit(_launch_ranks(args.gpus, sys.argv[1:], args.launch_timeout))
    if torchrun:
        _selftest_hook(int(os.environ["RANK"]))

    import torch
    import torch.distributed as dist

    if not torchrun:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        os.environ.setdefault("MASTER_PORT", str(_free_port()))
        os.environ.update(RANK="0", WORLD_SIZE="1", LOCAL_RANK="0")
    rank = int(os.environ["RANK"])
    world = int(os.environ["WORLD_SIZE"])
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        print(f"error: --gpus {args.gpus} but WORLD_SIZE is {world}", file=sys.stderr)
        sys.exit(2)
    # --backend gloo rehearses the multi-rank path with several ranks sharing
    # one GPU (RCCL refuses that); the measured numbers are then NOT scaling data
    gpu_index = local_rank % max(torch.cuda.device_count(), 1)
    torch.cuda.set_device(gpu_index)
    dev = torch.device("cuda", gpu_index)
    numa_rep = None
    if not args.no_numa_bind:
        # before any I/O-engine / staging thread exists: they inherit it
        from hipsnapshot.utils.affinity import bind_to_gpu_numa

        rep = numa_rep = bind_to_gpu_numa(gpu_index)
        if local_rank == 0:
            print(f"numa: {rep}", file=sys.stderr, flush=True)
    if args.backend == "nccl":
        dist.init_process_group("nccl", device_id=dev)
    else:
        dist.init_process_group("gloo")

    from hipsnapshot import Snapshot
    from hipsnapshot.models.llama import LlamaConfig, build_fsdp_llama
    from hipsnapshot.snapshot import TakeStats
    from hipsnapshot.ops import native

    native.require_gpu_lib()  # the HIP data plane must be the one running
    if args.no_plan_gc:
        from hipsnapshot import knobs

        knobs.TUNING.gc_after_plan = False
    cfg = {"llama3_8b": LlamaConfig.llama3_8b, "llama3_70b": LlamaConfig.llama3_70b,
           "tiny": LlamaConfig.tiny}[args.model]()
    from torch.distributed.device_mesh import init_device_mesh

    mesh = init_device_mesh("cuda", (world,))
    model = build_fsdp_llama(cfg, dev, torch.bfloat16, mesh=mesh)
    torch.cuda.synchronize()
    local_bytes = sum(p._local_tensor.numel() * p._local_tensor.element_size()
                      for p in model.parameters())
    t = torch.tensor([local_bytes], dtype=torch.int64, device=dev)
    dist.all_reduce(t)
    total_bytes = int(t.item())

    root = args.path or _default_dir()
    path = os.path.join(root, "ckpt")
    if rank == 0:
        shutil.rmtree(root, ignore_errors=True)
        os.makedirs(root, exist_ok=True)
    dist.barrier()
    opts = {"fsync": args.fsync, "direct_io": args.direct_io}
    app_state = {"model": model}

    def barrier_sync():
        torch.cuda.synchronize()
        dist.barrier()
        torch.cuda.synchronize()

    def log(msg):
        if rank == 0:
            print(msg, file=sys.stderr, flush=True)

    for i in range(args.warmup):
        t0 = time.monotonic()
        Snapshot.take(path, app_state, storage_options=opts, compression=args.compression)
        log(f"warmup {i}: {time.monotonic() - t0:.3f}s")

    from hipsnapshot.utils.tracing import GcWatch

    gcw = GcWatch().start()  # Python GC time inside the timed regions (reported)
    barrier_sync()
    t0 = time.perf_counter()
    my_step_s = []  # this rank's own take times (no barrier inside a step)
    for i in range(args.steps):
        ts = time.perf_counter()
        Snapshot.take(path, app_state, storage_options=opts, compression=args.compression)
        my_step_s.append(time.perf_counter() - ts)
        log(f"step {i}: {my_step_s[-1]:.3f}s")
    my_stored = int(TakeStats.last.get("bytes", 0))
    barrier_sync()
    t_end = time.perf_counter()
    elapsed = t_end - t0
    gc_take_ms = gcw.ms_between(t0, t_end)
    e = torch.tensor([elapsed], dtype=torch.float64, device=dev)
    dist.all_reduce(e, op=dist.ReduceOp.MAX)
    elapsed = float(e.item())
    ms_per_step = elapsed / args.steps * 1e3
    gbps = total_bytes / (ms_per_step / 1e3) / 1e9
    # per-rank view: mean take time and stored bytes of every rank
    per_rank = [None] * world
    dist.all_gather_object(per_rank, (statistics.mean(my_step_s) * 1e3, my_stored))
    rank_take_ms = sorted(r[0] for r in per_rank)
    rank_stored = [r[1] for r in per_rank]
    # one more (untimed) take with its phases captured on every rank: what a
    # multi-GPU curve needs to be attributed without another run
    from hipsnapshot.utils import rank_diag

    barrier_sync()
    my_diag = rank_diag.measure(lambda: Snapshot.take(path, app_state, storage_options=opts,
                                                      compression=args.compression))
    my_diag["numa"] = numa_rep

    # async_take: time-to-unblock
    # time_to_unblock: host time until async_take returns.  The HBM freeze
    # it enqueued on the trainer's stream runs after that: freeze_gpu_ms is
    # the GPU time between events recorded before and after the call (the
    # host planning before the launch included), freeze_kernel_ms the launch
    # alone, unblock_incl_freeze_ms the host time until the stream is free
    # again -- what a trainer whose next kernel waits sees.
    cold_unblock = []
    for i in range(args.async_warmup):
        barrier_sync()
        ts = time.perf_counter()
        pending = Snapshot.async_take(path + "_async", app_state, storage_options=opts,
                                      compression=args.compression)
        tu = time.perf_counter() - ts
        pending.wait()
        u = torch.tensor([tu], dtype=torch.float64, device=dev)
        dist.all_reduce(u, op=dist.ReduceOp.MAX)
        cold_unblock.append(float(u.item()) * 1e3)
        log(f"async warmup {i}: unblock {cold_unblock[-1]:.1f} ms")
    unblock = []
    drain = []
    freeze = []
    freeze_kernel = []
    unblock_gpu = []
    from hipsnapshot.engine.hbm_staging import last_freeze_ms

    for i in range(args.async_iters):
        barrier_sync()
        e0 = torch.cuda.Event(enable_timing=True)
        e1 = torch.cuda.Event(enable_timing=True)
        e0.record()
        ts = time.perf_counter()
        pending = Snapshot.async_take(path + "_async", app_state, storage_options=opts,
                                      compression=args.compression)
        tu = time.perf_counter() - ts
        e1.record()
        e1.synchronize()
        tg = time.perf_counter() - ts
        pending.wait()
        torch.cuda.synchronize()
        td = time.perf_counter() - ts
        fk = last_freeze_ms(gpu_index) or 0.0
        u = torch.tensor([tu, td, e0.elapsed_time(e1) / 1e3, tg, fk / 1e3], dtype=torch.float64,
                         device=dev)
        dist.all_reduce(u, op=dist.ReduceOp.MAX)
        unblock.append(float(u[0].item()) * 1e3)
        drain.append(float(u[1].item()) * 1e3)
        freeze.append(float(u[2].item()) * 1e3)
        unblock_gpu.append(float(u[3].item()) * 1e3)
        freeze_kernel.append(float(u[4].item()) * 1e3)
        log(f"async {i}: unblock {unblock[-1]:.1f} ms (stream free at {unblock_gpu[-1]:.1f} ms, "
            f"freeze kernel {freeze[-1]:.2f} ms), total {drain[-1]:.1f} ms")

    from hipsnapshot import memory_held

    held_after_takes = memory_held(gpu_index)  # between checkpoints: what stays
    stored = 0
    if rank == 0:
        for r, _, fs in os.walk(path):
            stored += sum(os.path.getsize(os.path.join(r, f)) for f in fs)

    restore_ok = None
    restore_gbps = None
    restore_each = None
    restore_info = {}
    gc_restore_ms = None
    if not args.no_restore_check:
        # bitwise restore check of EVERY local shard (HBM holds the copies)
        named = list(model.named_parameters())
        refs = [p._local_tensor.clone() for _, p in named]
        times, bad = [], []
        gc_restore_ms = 0.0
        from hipsnapshot.engine import native_restore, restore_cache

        rc0 = dict(restore_cache.stats)
        for _ in range(max(1, args.restore_iters)):
            for _, p in named:
                p._local_tensor.zero_()
            barrier_sync()
            tr = time.perf_counter()
            Snapshot(path).restore(app_state)
            barrier_sync()
            times.append(time.perf_counter() - tr)
            gc_restore_ms += gcw.ms_between(tr, tr + times[-1])
            # compare against the parameters as they are NOW (load_state_dict
            # may re-point a module's parameter)
            named = list(model.named_parameters())
            bad += [(n, r, p._local_tensor) for (n, p), r in zip(named, refs)
                    if not torch.equal(r, p._local_tensor)]
        restore_s = statistics.median(times)
        for n, r, cur in bad[:5]:
            nz = int((cur != 0).sum().item())
            print(f"rank {rank}: restore mismatch in {n}: shape {tuple(cur.shape)}, "
                  f"{nz}/{cur.numel()} nonzero, first diff at "
                  f"{int((r != cur).flatten().nonzero()[0].item())}", file=sys.stderr)
        ok = torch.tensor([int(not bad)], device=dev)
        dist.all_reduce(ok, op=dist.ReduceOp.MIN)
        restore_ok = bool(ok.item())
        restore_gbps = total_bytes / restore_s / 1e9
        restore_each = [round(total_bytes / t / 1e9, 2) for t in times]
        # the first restore plans from scratch, later ones of the same
        # snapshot into the same tensors reuse its plan (engine/restore_cache.py)
        my_diag["native_restore_stats"] = dict(native_restore.last_stats)
        restore_info = {"restore_cold_GBps": restore_each[0],
                        "restore_plan_cache": {k: restore_cache.stats[k] - rc0.get(k, 0)
                                               for k in ("hits", "misses", "stores")},
                        "native_restore_stats": dict(native_restore.last_stats)}
        # the same restores with every blob checked against the take's hs64
        # checksums (restore(verify=True): hashed in HBM inside the native job)
        vtimes, vbad = [], 0
        for _ in range(max(0, args.verify_iters)):
            for _, p in named:
                p._local_tensor.zero_()
            barrier_sync()
            tr = time.perf_counter()
            Snapshot(path).restore(app_state, verify=True)
            barrier_sync()
            vtimes.append(time.perf_counter() - tr)
            named = list(model.named_parameters())
            vbad += sum(not torch.equal(r, p._local_tensor) for (_n, p), r in zip(named, refs))
        del refs
        if vtimes:
            restore_info["restore_verify_bitwise_ok"] = vbad == 0
            restore_info["restore_verify_GBps"] = round(
                total_bytes / statistics.median(vtimes) / 1e9, 2)
            restore_info["restore_verify_GBps_each"] = [round(total_bytes / t / 1e9, 2)
                                                        for t in vtimes]
        log(f"restore: {restore_s:.3f}s ({restore_gbps:.2f} GB/s) ok={restore_ok} "
            f"each {restore_each} GB/s; {restore_info}")

    # BASELINE config 3: the N-rank FSDP checkpoint restored into N/2 ranks
    elastic = {}
    if args.elastic_iters > 0 and world >= 2 and world % 2 == 0:
        from torch.distributed.device_mesh import DeviceMesh

        from hipsnapshot import release_hbm_arena

        release_hbm_arena()
        mine = _shard_hashes(model, gpu_index)
        old = [None] * world
        dist.all_gather_object(old, mine)
        half = world // 2
        sub = dist.new_group(list(range(half)))
        submesh = DeviceMesh("cuda", list(range(half)))  # every rank constructs it
        times, bad = [], []
        if rank < half:
            model2 = build_fsdp_llama(cfg, dev, torch.bfloat16, mesh=submesh)
            for _ in range(args.elastic_iters):
                for p in model2.parameters():
                    p._local_tensor.zero_()
                torch.cuda.synchronize()
                dist.barrier(group=sub)
                tr = time.perf_counter()
                Snapshot(path, pg=sub).restore({"model": model2})
                torch.cuda.synchronize()
                dist.barrier(group=sub)
                times.append(time.perf_counter() - tr)
                bad += _check_resharded(model2, old, gpu_index)
            for n_, what in bad[:5]:
                print(f"rank {rank}: elastic restore mismatch in {n_}: {what}", file=sys.stderr)
            del model2
            torch.cuda.empty_cache()
        res = torch.tensor([max(times) if times else 0.0, float(bool(bad))],
                           dtype=torch.float64, device=dev)
        dist.all_reduce(res, op=dist.ReduceOp.MAX)
        each = [None] * world
        dist.all_gather_object(each, times)
        per_iter = [max(e[i] for e in each[:half]) for i in range(len(each[0]))]
        elastic = {
            "elastic_from_ranks": world, "elastic_to_ranks": half,
            "elastic_restore_s": round(statistics.median(per_iter), 3),
            "elastic_restore_GBps": round(total_bytes / statistics.median(per_iter) / 1e9, 2),
            "elastic_restore_GBps_each": [round(total_bytes / t / 1e9, 2) for t in per_iter],
            "elastic_bitwise_ok": not bool(res[1].item()),
        }
        log(f"elastic restore {world} -> {half} ranks: {elastic}")
        dist.barrier()

    # HSDP: replicated DTensor boxes split over the replica group
    hsdp = {}
    reps = args.hsdp if args.hsdp is not None else (2 if world >= 4 and world % 2 == 0 else 0)
    if reps > 1 and world % reps == 0 and world // reps >= 1:
        hsdp = _hsdp_phase(cfg, dev, gpu_index, world, rank, reps, root, opts, args, total_bytes,
                           barrier_sync, log)

    # the same save with raw, reference-format blobs (no HSZ1): what the
    # headline would be without the codec, measured in the same process
    raw_gbps = None
    if args.raw_steps > 0 and args.compression != "none":
        if rank == 0:
            shutil.rmtree(path + "_async", ignore_errors=True)
        dist.barrier()
        raw_path = path + "_raw"
        Snapshot.take(raw_path, app_state, storage_options=opts, compression="none")
        barrier_sync()
        t0 = time.perf_counter()
        for _ in range(args.raw_steps):
            Snapshot.take(raw_path, app_state, storage_options=opts, compression="none")
        barrier_sync()
        e = torch.tensor([time.perf_counter() - t0], dtype=torch.float64, device=dev)
        dist.all_reduce(e, op=dist.ReduceOp.MAX)
        raw_gbps = total_bytes / (float(e.item()) / args.raw_steps) / 1e9
        log(f"raw (uncompressed) save: {raw_gbps:.2f} GB/s")
        if rank == 0:
            shutil.rmtree(raw_path, ignore_errors=True)
        dist.barrier()

    # the headline rewrites one path; a training loop writes step_<i>/
    # directories: every take here creates fresh files (page cache
    # allocation, metadata).  Only the take is timed; removing the
    # directory from two steps back (keep-last-2) is not.
    fresh_gbps = fresh_each = None
    if args.fresh_steps > 0:
        if rank == 0:
            shutil.rmtree(path + "_async", ignore_errors=True)
        fdir = os.path.join(root, "fresh")
        # untimed: write back what the earlier sections left dirty.  New
        # files need new page-cache pages, and under a cgroup's dirty limit
        # the first fresh take otherwise paid for that writeback (1.6-2.6 s
        # instead of 0.2 s after the GPU test suite ran in the same box call)
        os.sync()
        dist.barrier()
        Snapshot.take(os.path.join(fdir, "warm"), app_state, storage_options=opts,
                      compression=args.compression)
        fresh_each = []
        for i in range(args.fresh_steps):
            barrier_sync()
            tf = time.perf_counter()
            Snapshot.take(os.path.join(fdir, f"step_{i}"), app_state, storage_options=opts,
                          compression=args.compression)
            barrier_sync()
            e = torch.tensor([time.perf_counter() - tf], dtype=torch.float64, device=dev)
            dist.all_reduce(e, op=dist.ReduceOp.MAX)
            fresh_each.append(float(e.item()))
            if rank == 0:
                shutil.rmtree(os.path.join(fdir, "warm" if i == 0 else f"step_{i - 1}"),
                              ignore_errors=True)
        fresh_gbps = total_bytes / statistics.mean(fresh_each) / 1e9
        log(f"fresh-directory save: {fresh_gbps:.2f} GB/s "
            f"({[round(x * 1e3, 1) for x in fresh_each]} ms)")
        if rank == 0:
            shutil.rmtree(fdir, ignore_errors=True)
        dist.barrier()

    # the reference's published config, in this same process: DDP, 200 x
    # 100 MB fp32 parameters, replicated=["**"], reference-format blobs
    # (/root/reference/benchmarks/ddp/main.py:18-70: 13.91 s on 1 GPU,
    # 3.38 s on 8 GPUs of a p4d.24xlarge)
    ddp_s = ddp_each = None
    if args.ddp_steps > 0:
        from torch.nn.parallel import DistributedDataParallel as DDP

        from hipsnapshot.models.ddp_bench import ManyParams

        ddp = DDP(ManyParams(200, 100, dev), device_ids=[gpu_index])
        ddp_bytes = 200 * 100 * 1000 * 1000
        dpath = os.path.join(root, "ddp20gb")
        Snapshot.take(dpath, {"model": ddp}, replicated=["**"], storage_options=opts,
                      compression="none")
        ddp_each = []
        for _ in range(args.ddp_steps):
            barrier_sync()
            tf = time.perf_counter()
            Snapshot.take(dpath, {"model": ddp}, replicated=["**"], storage_options=opts,
                          compression="none")
            barrier_sync()
            e = torch.tensor([time.perf_counter() - tf], dtype=torch.float64, device=dev)
            dist.all_reduce(e, op=dist.ReduceOp.MAX)
            ddp_each.append(float(e.item()))
        ddp_s = statistics.median(ddp_each)
        log(f"DDP 20 GB fp32 (reference config): {ddp_s:.3f} s "
            f"({ddp_bytes / ddp_s / 1e9:.2f} GB/s)")
        del ddp
        torch.cuda.empty_cache()
        if rank == 0:
            shutil.rmtree(dpath, ignore_errors=True)

    # BASELINE config 2: the model under DDP, bf16, replicated=["**"]: the
    # partitioner spreads the replicated state over the ranks' writers
    ddp_llama = {}
    if args.ddp_llama_steps > 0:
        from torch.nn.parallel import DistributedDataParallel as DDP

        from hipsnapshot import release_hbm_arena
        from hipsnapshot.models.llama import Llama, init_weights_

        release_hbm_arena()
        dcfg = {"llama3_8b": LlamaConfig.llama3_8b, "llama3_70b": LlamaConfig.llama3_70b,
                "tiny": LlamaConfig.tiny}[args.model]()
        if args.ddp_llama_layers:
            dcfg.n_layers = args.ddp_llama_layers
        with torch.device("meta"):
            dm = Llama(dcfg).to(torch.bfloat16)
        dm.to_empty(device=dev)
        init_weights_(dm, std=0.02)
        ddp = DDP(dm, device_ids=[gpu_index])  # broadcasts rank 0's weights
        dbytes = sum(p.numel() * p.element_size() for p in dm.parameters())
        dpath = os.path.join(root, "ddp_llama")
        dapp = {"model": ddp}
        Snapshot.take(dpath, dapp, replicated=["**"], storage_options=opts, compression="none")
        d_each, d_mine = [], []
        for _ in range(args.ddp_llama_steps):
            barrier_sync()
            tf = time.perf_counter()
            Snapshot.take(dpath, dapp, replicated=["**"], storage_options=opts,
                          compression="none")
            d_mine.append(time.perf_counter() - tf)
            barrier_sync()
            e = torch.tensor([time.perf_counter() - tf], dtype=torch.float64, device=dev)
            dist.all_reduce(e, op=dist.ReduceOp.MAX)
            d_each.append(float(e.item()))
        d_written = int(TakeStats.last.get("bytes", 0))
        # bitwise restore check through per-parameter hashes
        before = {n: _hash_tensor(p.data, gpu_index) for n, p in dm.named_parameters()}
        for p in dm.parameters():
            p.data.zero_()
        barrier_sync()
        tr = time.perf_counter()
        Snapshot(dpath).restore(dapp)
        barrier_sync()
        d_restore = time.perf_counter() - tr
        dbad = [n for n, p in dm.named_parameters() if _hash_tensor(p.data, gpu_index) != before[n]]
        for n in dbad[:5]:
            print(f"rank {rank}: DDP restore mismatch in {n}", file=sys.stderr)
        per = [None] * world
        dist.all_gather_object(per, (d_written, statistics.mean(d_mine) * 1e3, d_restore,
                                     len(dbad)))
        d_s = statistics.median(d_each)
        wr = [r[0] for r in per]
        ddp_llama = {
            "ddp_llama_GBps": round(dbytes / d_s / 1e9, 2),
            "ddp_llama_s": round(d_s, 3),
            "ddp_llama_s_each": [round(x, 3) for x in d_each],
            "ddp_llama_bytes": dbytes,
            "ddp_llama_layers": dcfg.n_layers,
            "ddp_llama_rank_written_bytes": wr,
            "ddp_llama_rank_written_max_over_mean": round(max(wr) / (sum(wr) / world), 3)
            if sum(wr) else None,
            "ddp_llama_rank_take_ms": [round(r[1], 1) for r in per],
            "ddp_llama_restore_GBps": round(dbytes / max(r[2] for r in per) / 1e9, 2),
            "ddp_llama_restore_bitwise_ok": all(r[3] == 0 for r in per),
        }
        log(f"DDP Llama partitioned save: {ddp_llama}")
        del ddp, dm, dapp
        torch.cuda.empty_cache()
        if rank == 0:
            shutil.rmtree(dpath, ignore_errors=True)
        dist.barrier()

    all_diag = [None] * world
    dist.all_gather_object(all_diag, my_diag)
    held_after_restore = memory_held(gpu_index)
    if rank == 0:
        out = {
            "metric": "checkpoint save GB/s + time-to-unblock, Llama-3-8B FSDP",
            "value": round(gbps, 3),
            "unit": "GB/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(ms_per_step, 2),
            "higher_is_better": True,
            "scaling": "strong",
            # same config only (the reference's DDP 20 GB, timed below): null
            # where the reference publishes no number (2 and 4 GPUs)
            "vs_baseline": round(REF_DDP_S[world] / ddp_s, 2)
            if ddp_s and world in REF_DDP_S else None,
            "dtype": "bf16",
            "data": "synthetic (random-init weights)",
            "config": {"model": {"llama3_8b": "Llama-3-8B", "llama3_70b": "Llama-3-70B",
                                 "tiny": "tiny-llama"}[args.model],
                       "global_batch": None, "seq_len": None,
                       "parallelism": f"fsdp{world}",
                       "checkpoint_bytes": total_bytes,
                       "storage": "local fs" + (" fsync" if args.fsync else ""),
                       "compression": args.compression},
            "world_size": dist.get_world_size(),
            "backend": str(dist.get_backend()),
            "rank_take_ms": {"max": round(rank_take_ms[-1], 2),
                             "median": round(statistics.median(rank_take_ms), 2),
                             "min": round(rank_take_ms[0], 2)},
            "rank_stored_bytes": rank_stored,
            # median over the async iterations (each value listed below)
            "time_to_unblock_ms": round(statistics.median(unblock), 2) if unblock else None,
            "time_to_unblock_ms_each": [round(u, 2) for u in unblock],
            "cold_time_to_unblock_ms": [round(u, 2) for u in cold_unblock],
            "async_warmup": args.async_warmup,
            "freeze_gpu_ms": round(statistics.median(freeze), 3) if freeze else None,
            "freeze_gpu_ms_each": [round(f, 3) for f in freeze],
            # the freeze launch alone (events around it inside async_take)
            "freeze_kernel_ms": round(statistics.median(freeze_kernel), 3) if freeze_kernel
            else None,
            "unblock_incl_freeze_ms": round(statistics.median(unblock_gpu), 2)
            if unblock_gpu else None,
            "async_iters": args.async_iters,
            # rank 0's last native drain, seconds per phase (summed over its threads)
            "async_drain_stats": _drain_stats(),
            "async_total_ms": round(statistics.median(drain), 2) if drain else None,
            "restore_bitwise_ok": restore_ok,
            "restore_GBps": round(restore_gbps, 2) if restore_gbps else None,
            "restore_GBps_each": restore_each, **restore_info,
            "compression": args.compression,
            "stored_bytes": stored,
            # rank 0's Python cyclic-GC time inside the timed takes / restores
            "gc_ms_in_timed_takes": round(gc_take_ms, 2),
            "gc_ms_in_timed_restores": round(gc_restore_ms, 2) if gc_restore_ms is not None
            else None,
            "raw_GBps": round(raw_gbps, 3) if raw_gbps else None,
            "raw_note": "same save with uncompressed reference-format blobs "
                        f"({args.raw_steps} timed takes after 1 warmup)",
            "fresh_path_GBps": round(fresh_gbps, 3) if fresh_gbps else None,
            "fresh_path_ms_each": [round(x * 1e3, 1) for x in fresh_each] if fresh_each
            else None,
            "fresh_path_steps": args.fresh_steps,
            "ddp20gb_fp32_s": round(ddp_s, 3) if ddp_s else None,
            "ddp20gb_fp32_s_each": [round(x, 3) for x in ddp_each] if ddp_each else None,
            "ddp20gb_fp32_GBps": round(20.0 / ddp_s, 2) if ddp_s else None,
            "ddp20gb_steps": args.ddp_steps,
            "vs_baseline_same_config": round(REF_DDP_S[world] / ddp_s, 2)
            if ddp_s and world in REF_DDP_S else None,
            "baseline_note": "reference DDP 20GB save, p4d: 1 GPU 1.44 GB/s, 8 GPU 5.92 GB/s; "
                             "no published number for 2/4 GPUs",
            **ddp_llama,
            **elastic,
            **hsdp,
            # what rank 0 holds between checkpoints (engine/memory.py): after
            # the async takes (arena, pools, pinned) and after the restores
            "hbm_held_between_takes_bytes": held_after_takes["hbm_held_bytes"],
            "pinned_held_bytes": held_after_takes["pinned_held_bytes"],
            "memory_held_after_takes": held_after_takes,
            "memory_held_after_restore": held_after_restore,
            # one untimed take per rank with its phases captured
            # (utils/rank_diag.py), and the one-line skew summary
            "rank_skew": rank_diag.skew(all_diag),
            "rank_diag": all_diag,
        }
        print(json.dumps(out), flush=True)
    dist.barrier()
    if rank == 0:
        shutil.rmtree(root, ignore_errors=True)
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
