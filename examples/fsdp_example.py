#!/usr/bin/env python3
"""FSDP2 (DTensor) Llama training with async snapshots and elastic resume.

    python -m torch.distributed.run --nproc-per-node 8 --master-addr 127.0.0.1 \
        examples/fsdp_example.py --model tiny --work-dir /tmp/fsdp_run
    # later, on 4 ranks: the sharded snapshot reshards on restore
    python -m torch.distributed.run --nproc-per-node 4 ... examples/fsdp_example.py --resume

``async_take`` freezes the sharded parameters into spare HBM with one gather
kernel and returns in milliseconds; D2H + writes drain while training runs.
"""

import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

from hipsnapshot import Snapshot, StateDict  # noqa: E402
from hipsnapshot.models.llama import LlamaConfig, build_fsdp_llama  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--work-dir", default="/tmp/hipsnapshot_fsdp")
    ap.add_argument("--model", default="tiny", choices=["tiny", "llama3_8b"])
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--resume", action="store_true")
    args = ap.parse_args()
    gpu = torch.cuda.is_available()
    local_rank = int(os.environ.get("LOCAL_RANK", 0))
    if gpu:
        torch.cuda.set_device(local_rank)
    dist.init_process_group("nccl" if gpu else "gloo")
    dev = torch.device("cuda", local_rank) if gpu else torch.device("cpu")
    from torch.distributed.device_mesh import init_device_mesh

    mesh = init_device_mesh(dev.type, (dist.get_world_size(),))
    cfg = getattr(LlamaConfig, args.model)()
    model = build_fsdp_llama(cfg, dev, torch.bfloat16 if gpu else torch.float32, mesh=mesh)
    optim = torch.optim.AdamW(model.parameters(), lr=1e-4)
    progress = StateDict(step=0)
    app_state = {"model": model, "optim": optim, "progress": progress}
    path = os.path.join(args.work_dir, "snap")
    if args.resume:
        Snapshot(path).restore(app_state)
    pending = None
    while progress["step"] < args.steps:
        tokens = torch.randint(0, cfg.vocab_size, (2, 64), device=dev)
        loss = model(tokens).float().logsumexp(-1).mean()
        optim.zero_grad()
        loss.backward()
        optim.step()
        progress["step"] += 1
        if progress["step"] % 5 == 0:
            if pending is not None:
                pending.wait()
            pending = Snapshot.async_take(path, app_state)
    if pending is not None:
        pending.wait()
    if dist.get_rank() == 0:
        print(f"done at step {progress['step']}")
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
