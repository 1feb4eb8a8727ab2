#!/usr/bin/env python3
"""ZeRO-3 OPT checkpoint benchmark through the DeepSpeed trick.

Reference: /root/reference/benchmarks/deepspeed_opt/main.py:27-160 (OPT with
48 layers / hidden 7168 / 56 heads, fp16, ZeRO-3 Adam; times
``engine.save_checkpoint`` and ``load_checkpoint`` with the torchsnapshot patch
vs DeepSpeed's own torch.save path).

DeepSpeed is not installed here, so the per-rank ZeRO-3 state is built by
``hipsnapshot.models.zero3`` (fp16 partition + fp32 master sub-groups + Adam
moments, all in HBM) and saved through the same patched
``_save_zero_checkpoint`` / ``_load_zero_checkpoint`` methods
(``hipsnapshot.tricks.deepspeed``).  Reports time-to-unblock of the async save,
total save time, restore time, and a ``torch.save`` per-rank baseline.

The full 30B-parameter config is 420 GB of state; ``--max-total-gb`` scales
the layer count down to what the box's disk holds (reported in the output).
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
from hipsnapshot.models.zero3 import (EmulatedZero3Engine, EmulatedZero3Optimizer,  # noqa: E402
                                      OPTShape)
from hipsnapshot.tricks.deepspeed import patch_engine_to_use_hipsnapshot  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--layers", type=int, default=48)
    ap.add_argument("--hidden", type=int, default=7168)
    ap.add_argument("--heads", type=int, default=56)
    ap.add_argument("--max-total-gb", type=float, default=40.0,
                    help="shrink the layer count so the whole snapshot fits this size")
    ap.add_argument("--work-dir", default=os.environ.get("HSBENCH_DIR", "/tmp"))
    ap.add_argument("--torch-save", action="store_true")
    ap.add_argument("--no-load", action="store_true")
    args = ap.parse_args()
    rank, ws, dev = init_dist()
    shape = OPTShape(num_hidden_layers=args.layers, hidden_size=args.hidden,
                     num_attention_heads=args.heads)
    while shape.num_hidden_layers > 1 and shape.num_params() * 14 > args.max_total_gb * 1e9:
        shape.num_hidden_layers -= 1
    opt = EmulatedZero3Optimizer(shape, rank, ws, dev)
    engine = EmulatedZero3Engine(opt, rank)
    patch_engine_to_use_hipsnapshot(engine)
    nbytes_rank = opt.nbytes()
    total = max_over_ranks(float(nbytes_rank), dev) * ws
    log(f"OPT shape: {shape.num_hidden_layers} layers, {shape.num_params() / 1e9:.2f} B params, "
        f"ZeRO-3 state {total / 1e9:.1f} GB over {ws} ranks")
    root = os.path.join(args.work_dir, "hs_zero3_bench")
    if rank == 0:
        shutil.rmtree(root, ignore_errors=True)
    sync(dev)
    path = os.path.join(root, "global_step1000")
    with Timer() as t_total:
        with Timer() as t_unblock:
            engine._save_zero_checkpoint(path, "global_step1000")
        engine._hipsnapshot_pending.wait()
        sync(dev)
    unblock = max_over_ranks(t_unblock.s, dev)
    save = max_over_ranks(t_total.s, dev)
    log(f"save: unblock {unblock * 1e3:.1f} ms, total {save:.2f}s ({total / save / 1e9:.2f} GB/s)")
    out = {"bench": "zero3_opt_save", "world_size": ws, "layers": shape.num_hidden_layers,
           "params_B": round(shape.num_params() / 1e9, 2), "bytes": int(total),
           "time_to_unblock_ms": round(unblock * 1e3, 2), "save_seconds": round(save, 3),
           "save_GBps": round(total / save / 1e9, 2)}
    if not args.no_load:
        ref = [t.clone() for t in opt.exp_avg]
        for t in opt.exp_avg:
            t.zero_()
        sync(dev)
        with Timer() as t_load:
            engine._load_zero_checkpoint(path, "global_step1000")
            sync(dev)
        load = max_over_ranks(t_load.s, dev)
        ok = all(torch.equal(a, b) for a, b in zip(ref, opt.exp_avg))
        log(f"load: {load:.2f}s ({total / load / 1e9:.2f} GB/s) ok={ok}")
        out.update(load_seconds=round(load, 3), load_GBps=round(total / load / 1e9, 2),
                   load_bitwise_ok=ok)
    if args.torch_save:
        p = os.path.join(root, f"torch_save_rank{rank}.pt")
        sync(dev)
        with Timer() as t_ts:
            torch.save(opt.state_dict(), p)
            sync(dev)
        out["torch_save_seconds"] = round(max_over_ranks(t_ts.s, dev), 3)
    sync(dev)
    emit(out)
    if rank == 0:
        shutil.rmtree(root, ignore_errors=True)
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
