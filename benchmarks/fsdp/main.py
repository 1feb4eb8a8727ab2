#!/usr/bin/env python3
"""FSDP nn.Transformer checkpoint benchmark (save + load, vs torch.save).

Reference: /root/reference/benchmarks/fsdp/main.py:33-152 -- nn.Transformer
(d_model 864, 1 encoder + 20 decoder layers, 12 heads, FFN 50257; 1.9 B params,
7.8 GB fp32) wrapped per layer with FSDP and saved with LOCAL_STATE_DICT.

torch 2.10 FSDP2 (``fully_shard``) yields DTensor(Shard(0)) parameters; those
are written as sharded entries, so the snapshot restores onto any world size.
The ``torch.save`` baseline saves each rank's sharded state dict (the
reference's LOCAL_STATE_DICT equivalent) to its own file.
"""

import argparse
import os
import shutil
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402
import torch.nn as nn  # noqa: E402

from common import Timer, emit, init_dist, log, max_over_ranks, sync  # noqa: E402
from hipsnapshot import Snapshot  # noqa: E402


def create_model(dev, d_model: int, dec_layers: int, nhead: int, ffn: int) -> nn.Module:
    from torch.distributed.fsdp import fully_shard

    with torch.device("meta"):
        model = nn.Transformer(d_model=d_model, num_encoder_layers=1,
                               num_decoder_layers=dec_layers, nhead=nhead,
                               dim_feedforward=ffn)
    for m in list(model.modules()):
        if isinstance(m, (nn.TransformerEncoderLayer, nn.TransformerDecoderLayer)):
            fully_shard(m)
    fully_shard(model)
    model.to_empty(device=dev)
    g = torch.Generator(device=dev).manual_seed(0)
    with torch.no_grad():
        for p in model.parameters():
            p.to_local().normal_(0, 0.02, generator=g)
    return model


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--d-model", type=int, default=864)
    ap.add_argument("--dec-layers", type=int, default=20)
    ap.add_argument("--nhead", type=int, default=12)
    ap.add_argument("--ffn", type=int, default=50257)
    ap.add_argument("--work-dir", default=os.environ.get("HSBENCH_DIR", "/tmp"))
    ap.add_argument("--torch-save", action="store_true")
    ap.add_argument("--repeats", type=int, default=2)
    args = ap.parse_args()
    rank, ws, dev = init_dist()
    model = create_model(dev, args.d_model, args.dec_layers, args.nhead, args.ffn)
    nbytes = sum(p.numel() * p.element_size() for p in model.parameters())
    nparams = sum(p.numel() for p in model.parameters())
    log(f"model parameters: {nparams:,}, size {nbytes / 1e9:.2f} GB, world size {ws}")
    root = os.path.join(args.work_dir, "hs_fsdp_bench")
    if rank == 0:
        shutil.rmtree(root, ignore_errors=True)
    sync(dev)
    app_state = {"model": model}
    best = None
    for i in range(args.repeats):
        sync(dev)
        with Timer() as t:
            Snapshot.take(os.path.join(root, "snap"), app_state)
            sync(dev)
        s = max_over_ranks(t.s, dev)
        log(f"take {i}: {s:.2f}s ({nbytes / s / 1e9:.2f} GB/s)")
        best = s if best is None else min(best, s)
    ref = {k: v.to_local().clone() for k, v in model.state_dict().items()}
    with torch.no_grad():
        for p in model.parameters():
            p.to_local().zero_()
    sync(dev)
    with Timer() as t:
        Snapshot(os.path.join(root, "snap")).restore(app_state)
        sync(dev)
    load = max_over_ranks(t.s, dev)
    ok = all(torch.equal(ref[k], v.to_local()) for k, v in model.state_dict().items())
    log(f"restore: {load:.2f}s ({nbytes / load / 1e9:.2f} GB/s) ok={ok}")
    out = {"bench": "fsdp_transformer", "world_size": ws, "params": nparams, "bytes": nbytes,
           "save_seconds": round(best, 3), "save_GBps": round(nbytes / best / 1e9, 2),
           "load_seconds": round(load, 3), "load_GBps": round(nbytes / load / 1e9, 2),
           "load_bitwise_ok": ok}
    if args.torch_save:
        os.makedirs(root, exist_ok=True)
        p = os.path.join(root, f"state_dict-{rank}.pt")
        sync(dev)
        with Timer() as t:
            torch.save(model.state_dict(), p)
            sync(dev)
        out["torch_save_seconds"] = round(max_over_ranks(t.s, dev), 3)
        sync(dev)
        with Timer() as t:
            model.load_state_dict(torch.load(p, weights_only=True))
            sync(dev)
        out["torch_load_seconds"] = round(max_over_ranks(t.s, dev), 3)
    sync(dev)
    emit(out)
    if rank == 0:
        shutil.rmtree(root, ignore_errors=True)
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
