#!/usr/bin/env python3
"""DLRM with row-wise sharded embedding tables: train, snapshot, resume.

    python -m torch.distributed.run --nproc-per-node 2 --master-addr 127.0.0.1 \
        examples/dlrm_example.py --snapshot-path /tmp/dlrm_snap

    # resume (any world size: the tables are sharded entries)
    python -m torch.distributed.run --nproc-per-node 1 --master-addr 127.0.0.1 \
        examples/dlrm_example.py --restore-path /tmp/dlrm_snap/epoch_1

Counterpart of the reference's TorchRec example
(`/root/reference/examples/torchrec/main.py`): embedding tables are
DTensor(Shard(0)) shards (optionally in managed memory with ``--uvm``), the
dense MLPs are DDP-replicated, and progress + RNG state are snapshotted with
``async_take`` so training continues while the checkpoint drains.
"""

import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

from hipsnapshot import RNGState, Snapshot, StateDict  # noqa: E402
from hipsnapshot.models.dlrm import DLRM  # noqa: E402


def batch(n, tables, dev, gen):
    dense = torch.randn(n, 13, device=dev, generator=gen)
    sparse = []
    for rows in tables:
        ids = torch.randint(0, rows, (n * 4,), device=dev, generator=gen)
        offs = torch.arange(0, n * 4, 4, device=dev)
        sparse.append((ids, offs))
    label = torch.randint(0, 2, (n, 1), device=dev, generator=gen).float()
    return dense, sparse, label


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--snapshot-path", default="/tmp/hipsnapshot_dlrm")
    ap.add_argument("--restore-path", default=None)
    ap.add_argument("--epochs", type=int, default=2)
    ap.add_argument("--steps-per-epoch", type=int, default=10)
    ap.add_argument("--uvm", action="store_true", help="tables in managed memory (GPU only)")
    args = ap.parse_args()
    gpu = torch.cuda.is_available()
    local_rank = int(os.environ.get("LOCAL_RANK", 0))
    if gpu:
        torch.cuda.set_device(local_rank)
    if "RANK" not in os.environ:
        os.environ.update(RANK="0", WORLD_SIZE="1", MASTER_ADDR="127.0.0.1",
                          MASTER_PORT=os.environ.get("MASTER_PORT", "29533"))
    dist.init_process_group("nccl" if gpu else "gloo")
    dev = torch.device("cuda", local_rank) if gpu else torch.device("cpu")
    from torch.distributed.device_mesh import init_device_mesh

    mesh = init_device_mesh(dev.type, (dist.get_world_size(),))
    tables = [100_000, 50_000, 20_000]
    torch.manual_seed(0)
    model = DLRM(tables, dim=64, device=dev, mesh=mesh, uvm=args.uvm and gpu)
    dense_params = list(model.bottom.parameters()) + list(model.top.parameters())
    optim = torch.optim.Adagrad(dense_params, lr=0.01)
    progress = StateDict(epoch=0)
    app_state = {"model": model, "optim": optim, "progress": progress, "rng": RNGState()}
    if args.restore_path:
        Snapshot(args.restore_path).restore(app_state)
        if dist.get_rank() == 0:
            print(f"restored from {args.restore_path} at epoch {progress['epoch']}")
    gen = torch.Generator(device=dev).manual_seed(dist.get_rank())
    pending = None
    while progress["epoch"] < args.epochs:
        for _ in range(args.steps_per_epoch):
            dense, sparse, label = batch(64, tables, dev, gen)
            loss = torch.nn.functional.binary_cross_entropy_with_logits(
                model(dense, sparse), label)
            optim.zero_grad()
            loss.backward()
            for p in dense_params:  # dense MLPs are data-parallel
                if p.grad is not None and dist.get_world_size() > 1:
                    dist.all_reduce(p.grad)
                    p.grad /= dist.get_world_size()
            optim.step()
        progress["epoch"] += 1
        if pending is not None:
            pending.wait()
        path = os.path.join(args.snapshot_path, f"epoch_{progress['epoch']}")
        # dense MLPs are identical on every rank: store them once
        pending = Snapshot.async_take(path, app_state,
                                      replicated=["model/bottom/**", "model/top/**", "optim/**"])
        if dist.get_rank() == 0:
            print(f"epoch {progress['epoch']}: loss {loss.item():.4f}, snapshot -> {path}")
    if pending is not None:
        pending.wait()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
