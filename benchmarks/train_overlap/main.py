#!/usr/bin/env python3
"""Checkpointing a TRAINING job: Llama-3 FSDP2 model + AdamW state, taken with
``async_take`` while training continues (BASELINE config 5's "train-step
overlap", on local storage or the in-process fake S3).

Reported (max over ranks):

* baseline step time (fwd + bwd + AdamW, synthetic tokens);
* ``Snapshot.take`` (blocking) time of model + optimizer state;
* ``async_take`` time-to-unblock, background drain time, the number of
  training steps that ran while the snapshot drained, and their mean / max
  step time (the slowdown the checkpoint costs the trainer);
* a bitwise restore check of every model and optimizer shard.

The reference publishes no such number (time-to-unblock is printed but not
reported by `/root/reference/benchmarks/torchrec/main.py:133-151`).

    python benchmarks/train_overlap/main.py --layers 32 --seq 2048
    python benchmarks/train_overlap/main.py --layers 16 --master-dtype fp32
    torchrun --nproc-per-node 8 benchmarks/train_overlap/main.py
"""

from __future__ import annotations

import argparse
import os
import shutil
import statistics
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402
import torch.nn.functional as F  # noqa: E402

from common import emit, init_dist, log, max_over_ranks, sync  # noqa: E402
from hipsnapshot import Snapshot  # noqa: E402
from hipsnapshot.models.llama import LlamaConfig, build_fsdp_llama  # noqa: E402


def _cgroup_cpu() -> dict:
    """cgroup v2 CPU accounting of this job (throttling = CFS quota stalls:
    every thread of the cgroup waits for the next period)."""
    out = {}
    try:
        with open("/sys/fs/cgroup/cpu.stat") as f:
            for line in f:
                k, v = line.split()
                out[k] = int(v)
        with open("/sys/fs/cgroup/cpu.max") as f:
            out["max"] = f.read().strip()
    except OSError:
        pass
    import resource

    ru = resource.getrusage(resource.RUSAGE_SELF)
    out["proc_cpu_s"] = ru.ru_utime + ru.ru_stime
    return out


def _cpu_khz():
    """Current clock (kHz) of the CPU this thread last ran on (cpufreq), or
    None: a launch-bound step is as fast as that core's clock."""
    from hipsnapshot.utils.affinity import current_cpu

    cpu = current_cpu()
    if cpu is None:
        return None
    try:
        with open(f"/sys/devices/system/cpu/cpu{cpu}/cpufreq/scaling_cur_freq") as f:
            return int(f.read())
    except (OSError, ValueError):
        return None


def _local(t):
    return t._local_tensor if hasattr(t, "_local_tensor") else t


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="llama3_8b", choices=["llama3_8b", "llama3_70b", "tiny"])
    ap.add_argument("--layers", type=int, default=None)
    ap.add_argument("--seq", type=int, default=2048)
    ap.add_argument("--batch", type=int, default=1)
    ap.add_argument("--baseline-steps", type=int, default=10)
    ap.add_argument("--window-steps", type=int, default=12,
                    help="train_time_lost_ms covers at least this many steps after async_take")
    ap.add_argument("--warm-async", type=int, default=1,
                    help="async_takes (waited for) before the measured window: the first "
                         "one of a job allocates its HBM arena and pinned drain slots, a "
                         "one-time cost reported as cold_async_* ")
    ap.add_argument("--gap-steps", type=int, default=0,
                    help="training steps between one checkpoint's commit and the next "
                         "async_take (the page cache writes the previous one back meanwhile)")
    ap.add_argument("--checkpoints", type=int, default=1,
                    help="async_takes back to back (each starts when the previous one has "
                         "committed) inside ONE measured window: enough steps overlap a "
                         "drain to rank changes; train_time_lost_ms is per checkpoint")
    ap.add_argument("--compression", default="hsz1", choices=["none", "hsz1"])
    ap.add_argument("--storage", default="fs", choices=["fs", "s3"])
    ap.add_argument("--path", default=None)
    ap.add_argument("--switch-interval-ms", type=float, default=None,
                    help="sys.setswitchinterval for this process (GIL hand-over period; "
                         "Python's default is 5 ms)")
    ap.add_argument("--step-sync", default="stream", choices=["stream", "device"],
                    help="how a training step waits for its GPU work: the trainer's stream "
                         "(what loss.item() does) or the whole device (torch.cuda."
                         "synchronize(), which also waits for the snapshot drain's copy "
                         "streams and so charges their work to the step)")
    ap.add_argument("--master-dtype", default="bf16", choices=["bf16", "fp32"],
                    help="stored parameter (and AdamW state) dtype; fp32 = mixed precision "
                         "with bf16 compute")
    args = ap.parse_args()

    if args.switch_interval_ms is not None:
        sys.setswitchinterval(args.switch_interval_ms / 1e3)
    rank, ws, dev = init_dist()
    if dev.type == "cuda":
        from hipsnapshot.utils.affinity import bind_to_gpu_numa

        bind_to_gpu_numa(dev.index)
    from torch.distributed.device_mesh import init_device_mesh

    cfg = getattr(LlamaConfig, args.model)()
    if args.layers:
        cfg.n_layers = args.layers
    mesh = init_device_mesh(dev.type, (ws,))
    master = torch.float32 if args.master_dtype == "fp32" else torch.bfloat16
    model = build_fsdp_llama(cfg, dev, master, mesh=mesh, compute_dtype=torch.bfloat16)
    opt = torch.optim.AdamW(model.parameters(), lr=1e-5, foreach=True)
    gen = torch.Generator(device=dev).manual_seed(1234 + rank)

    from hipsnapshot.utils.tracing import timeline

    freq_log = []  # (step end time, kHz of the CPU the trainer thread ran on)

    def step() -> float:
        t0 = time.perf_counter()
        try:
            return _step(t0)
        finally:
            t1 = time.perf_counter()
            timeline.add("train_step", "train", t0, t1)
            f = _cpu_khz()
            if f is not None:
                freq_log.append((t1, f))

    def _step(t0: float) -> float:
        tok = torch.randint(0, cfg.vocab_size, (args.batch, args.seq + 1), device=dev,
                            generator=gen)
        logits = model(tok[:, :-1])
        loss = F.cross_entropy(logits.float().flatten(0, 1), tok[:, 1:].flatten())
        loss.backward()
        opt.step()
        opt.zero_grad(set_to_none=True)
        if dev.type == "cuda":
            if args.step_sync == "device":
                torch.cuda.synchronize()
            else:
                torch.cuda.current_stream(dev).synchronize()
        return time.perf_counter() - t0

    for _ in range(2):  # creates the AdamW state
        step()
    sync(dev)
    base = [step() for _ in range(args.baseline_steps)]
    base_ms = max_over_ranks(statistics.median(base), dev) * 1e3  # provisional (log only)
    ckpt_bytes = sum(_local(p).numel() * _local(p).element_size() for p in model.parameters())
    for st in opt.state.values():
        for v in st.values():
            if torch.is_tensor(v):
                ckpt_bytes += _local(v).numel() * _local(v).element_size()
    t = torch.tensor([ckpt_bytes], dtype=torch.int64, device=dev)
    dist.all_reduce(t)
    ckpt_bytes = int(t.item())
    log(f"baseline step {base_ms:.1f} ms; checkpoint {ckpt_bytes / 1e9:.2f} GB (model + AdamW)")

    srv = None
    opts = None
    if args.storage == "s3":
        from hipsnapshot.storage.fake_servers import FakeS3Process

        srv = FakeS3Process() if rank == 0 else None
        url = [srv.url if srv else None]
        dist.broadcast_object_list(url, src=0)
        opts = {"aws_access_key_id": "AKIDFAKE", "aws_secret_access_key": "fake-secret",
                "endpoint_url": url[0], "multipart_threshold": 64 << 20, "part_size": 64 << 20}
        root = "s3://ckpt/train_overlap"
    else:
        root = args.path or os.path.join(os.environ.get("HSBENCH_DIR", "/tmp"),
                                         "train_overlap")
        if rank == 0:
            shutil.rmtree(root, ignore_errors=True)
    app = {"model": model, "optim": opt}

    # blocking take (reference semantics) for comparison: median of 3, the
    # first one also builds the take plan
    log("phase: sync take")
    sync_each = []
    for _ in range(3):
        sync(dev)
        t0 = time.perf_counter()
        Snapshot.take(f"{root}/sync", app, storage_options=opts, compression=args.compression)
        sync_each.append(max_over_ranks(time.perf_counter() - t0, dev))
    sync_s = statistics.median(sync_each)
    if args.storage == "fs" and rank == 0:
        shutil.rmtree(f"{root}/sync", ignore_errors=True)  # keep the disk footprint to one copy

    cold = []
    for _ in range(args.warm_async):
        sync(dev)
        tw = time.perf_counter()
        p = Snapshot.async_take(f"{root}/async", app, storage_options=opts,
                                compression=args.compression)
        tu = time.perf_counter() - tw
        p.wait()
        sync(dev)
        cold.append((tu, time.perf_counter() - tw))
    # async takes while training continues: --checkpoints of them back to
    # back, each starting at the first step boundary after the previous one
    # committed (same path: a rewrite, as a ring of checkpoints would do)
    log(f"phase: async take x{args.checkpoints} (sync take {sync_s:.3f} s)")
    sync(dev)
    k_total = max(1, args.checkpoints)
    pending, taken, t_ck = None, 0, 0.0
    during, unblocks, drains = [], [], []
    during_k, gap_k = [], []  # per checkpoint: steps during its drain / after it
    drain_stats = []  # per checkpoint: the native drain's phase seconds
    ref, clone_s = None, 0.0
    def all_done(p) -> bool:
        """``p.done()`` agreed across ranks (a step runs FSDP collectives:
        every rank must run the same number of them)."""
        d = p is None or p.done()
        if ws == 1:
            return d
        f = torch.tensor([int(d)], device=dev)
        dist.all_reduce(f, op=dist.ReduceOp.MIN)
        return bool(f.item())

    gap = []  # steps between checkpoints (no drain running)
    ck_starts = []
    from hipsnapshot.utils.tracing import GcWatch

    gcw = GcWatch().start()
    unblock_gc = []
    cg0 = _cgroup_cpu()
    t0 = time.perf_counter()
    while True:
        if all_done(pending):
            if pending is not None:
                pending.wait()
                drains.append(time.perf_counter() - t_ck)
                from hipsnapshot.engine import native_drain

                drain_stats.append(dict(native_drain.last_stats))
                if taken < k_total:
                    gap_k.append([step() for _ in range(args.gap_steps)])
                    gap += gap_k[-1]
            if taken == k_total:
                break
            if taken == k_total - 1:  # the restore check compares with this state
                tc = time.perf_counter()
                ref = {n: _local(p).detach().clone() for n, p in model.named_parameters()}
                torch.cuda.current_stream(dev).synchronize() if dev.type == "cuda" else None
                clone_s = time.perf_counter() - tc
            t_ck = time.perf_counter()
            ck_starts.append(t_ck)
            pending = Snapshot.async_take(f"{root}/async", app, storage_options=opts,
                                          compression=args.compression)
            unblocks.append(time.perf_counter() - t_ck)
            unblock_gc.append(gcw.ms_between(t_ck, t_ck + unblocks[-1]))
            during_k.append([])
            taken += 1
        during.append(step())
        during_k[-1].append(during[-1])
    drain = statistics.mean(drains)
    windows = [(t, t + d) for t, d in zip(ck_starts, drains)]
    f_in = [f for t, f in freq_log if any(a <= t <= b for a, b in windows)]
    f_out = [f for t, f in freq_log if not any(a <= t <= b for a, b in windows)]
    freq = {"trainer_cpu_MHz_during_drain": round(statistics.median(f_in) / 1e3) if f_in else None,
            "trainer_cpu_MHz_otherwise": round(statistics.median(f_out) / 1e3) if f_out else None}
    unblock = statistics.median(unblocks)
    # training time lost to the checkpoints: wall time from the first
    # async_take call through a window of at least --window-steps steps (the
    # unblocks and every step slowed by a drain inside it) minus the same
    # steps at baseline, per checkpoint (the reference clone is not counted)
    extra = 0
    while len(during) + extra < args.window_steps:
        step()
        extra += 1
    window_s = time.perf_counter() - t0
    cg1 = _cgroup_cpu()
    cgroup = {"cpu_max": cg1.get("max"), "window_s": round(window_s, 3),
              "process_cpu_s": round(cg1["proc_cpu_s"] - cg0["proc_cpu_s"], 2)}
    for k in ("usage_usec", "nr_periods", "nr_throttled", "throttled_usec"):
        if k in cg0 and k in cg1:
            cgroup[k] = cg1[k] - cg0[k]
    gc_window_ms = gcw.ms_between(t0, t0 + window_s)
    gcw.stop()
    # the step-time baseline: median of EVERY step no drain overlapped (before
    # the first checkpoint, between checkpoints and after the window), so
    # clock / thermal drift over the run does not count as checkpoint cost
    post = [step() for _ in range(args.baseline_steps)]
    base_ms = max_over_ranks(statistics.median(base + gap + post), dev) * 1e3
    base_pre_ms = max_over_ranks(statistics.median(base), dev) * 1e3
    base_post_ms = max_over_ranks(statistics.median(post), dev) * 1e3
    # the same cost against a LOCAL baseline: each checkpoint's drain steps vs
    # the no-drain steps right before and after it (the box's step time drifts
    # by up to 10 % over a run with clocks and temperature; adjacent steps
    # share the regime)
    lost_local, slow_local = [], []
    for k in range(k_total):
        before = gap_k[k - 1] if k > 0 else base
        after = gap_k[k] if k < len(gap_k) else post
        # with --gap-steps 0 the checkpoints run back to back: no drain-free
        # steps between them, the run's own baseline steps stand in
        loc = statistics.median((before + after) or (base + post))
        d = during_k[k]
        lost_local.append(unblocks[k] + sum(d) - len(d) * loc)
        slow_local.append(statistics.median(d) / loc - 1.0 if d else 0.0)
    lost_local_ms = max_over_ranks(statistics.mean(lost_local), dev) * 1e3
    lost = (window_s - clone_s - (len(during) + len(gap) + extra) * base_ms / 1e3) / k_total
    # every rank must finish its loop before collectives resume
    unblock = max_over_ranks(unblock, dev)
    drain = max_over_ranks(drain, dev)
    n_during = int(max_over_ranks(float(len(during)), dev))
    lost = max_over_ranks(lost, dev)
    mean_ms = max_over_ranks(statistics.mean(during) if during else 0.0, dev) * 1e3
    med_ms = max_over_ranks(statistics.median(during) if during else 0.0, dev) * 1e3
    max_ms = max_over_ranks(max(during) if during else 0.0, dev) * 1e3

    log(f"phase: restore (unblock {unblock * 1e3:.1f} ms, {len(during)} steps during drain)")
    stored = None
    if args.storage == "fs" and rank == 0:
        stored = sum(os.path.getsize(os.path.join(r, f))
                     for r, _, fs in os.walk(f"{root}/async") for f in fs)
    # restore the async snapshot: parameters must equal the values at the
    # async_take call, not the ones the overlapped steps produced
    Snapshot(f"{root}/async", storage_options=opts).restore(app)
    ok = all(torch.equal(_local(p), ref[n]) for n, p in model.named_parameters())
    okt = torch.tensor([int(ok)], device=dev)
    dist.all_reduce(okt, op=dist.ReduceOp.MIN)

    emit({"bench": "train_overlap_async_take", "model": args.model, "layers": cfg.n_layers,
          "world_size": ws, "seq": args.seq, "batch": args.batch, "storage": args.storage,
          "compression": args.compression, "master_dtype": args.master_dtype,
          "switch_interval_ms": sys.getswitchinterval() * 1e3, "step_sync": args.step_sync,
          "checkpoint_bytes": ckpt_bytes,
          "baseline_step_ms": round(base_ms, 2), "baseline_step_ms_pre": round(base_pre_ms, 2),
          "baseline_step_ms_post": round(base_post_ms, 2),
          "async_unblock_gc_ms_each": [round(g, 1) for g in unblock_gc],
          "gc_ms_in_window": round(gc_window_ms, 1), **freq, "cgroup_cpu_in_window": cgroup, "sync_take_s": round(sync_s, 3),
          "sync_take_GBps": round(ckpt_bytes / sync_s / 1e9, 2),
          "async_unblock_ms": round(unblock * 1e3, 2), "async_drain_s": round(drain, 3),
          "cold_async_unblock_ms": [round(c[0] * 1e3, 1) for c in cold],
          "cold_async_total_s": [round(c[1], 3) for c in cold],
          "checkpoints": k_total, "async_unblock_ms_each": [round(u * 1e3, 2) for u in unblocks],
          "async_drain_s_each": [round(d, 3) for d in drains],
          "native_drain_stats_each": drain_stats,
          "steps_during_drain": n_during, "step_ms_during_drain_mean": round(mean_ms, 2),
          "step_ms_during_drain_median": round(med_ms, 2),
          "step_ms_during_drain_max": round(max_ms, 2),
          "step_ms_during_drain_each": [round(x * 1e3, 1) for x in during],
          "slowdown_during_drain": round(mean_ms / base_ms - 1.0, 4) if during else None,
          "gap_steps": args.gap_steps,
          "step_ms_between_checkpoints_median": round(statistics.median(gap) * 1e3, 2)
          if gap else None,
          "window_steps": len(during) + len(gap) + extra,
          "train_time_lost_ms": round(lost * 1e3, 1),
          "train_time_lost_vs_sync_take": round(lost / sync_s, 3),
          "train_time_lost_local_ms": round(lost_local_ms, 1),
          "train_time_lost_local_vs_sync_take": round(lost_local_ms / 1e3 / sync_s, 3),
          "train_time_lost_local_ms_each": [round(x * 1e3, 1) for x in lost_local],
          "slowdown_local_median_each": [round(x, 4) for x in slow_local],
          "restore_bitwise_ok": bool(okt.item()), "stored_bytes": stored,
          "data": "synthetic tokens, random init"})
    sync(dev)
    if srv:
        srv.stop()
    elif rank == 0:
        shutil.rmtree(root, ignore_errors=True)
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
