#!/usr/bin/env python3
"""DDP training with replicated snapshots (write load spread over ranks).

    python -m torch.distributed.run --nproc-per-node 2 --master-addr 127.0.0.1 \
        examples/ddp_example.py --work-dir /tmp/ddp_run

On MI355X each rank owns one GPU (RCCL); on CPU it runs on gloo.  DDP modules
are recognised automatically: their parameters are saved once (replicated),
partitioned across ranks, and any world size can restore them.
"""

import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402
from torch.nn.parallel import DistributedDataParallel as DDP  # noqa: E402

from hipsnapshot import Snapshot, StateDict  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--work-dir", default="/tmp/hipsnapshot_ddp")
    ap.add_argument("--steps", type=int, default=50)
    args = ap.parse_args()
    gpu = torch.cuda.is_available()
    local_rank = int(os.environ.get("LOCAL_RANK", 0))
    if gpu:
        torch.cuda.set_device(local_rank)
    dist.init_process_group("nccl" if gpu else "gloo")
    dev = torch.device("cuda", local_rank) if gpu else torch.device("cpu")
    torch.manual_seed(0)
    model = DDP(torch.nn.Linear(1024, 1024).to(dev), device_ids=[local_rank] if gpu else None)
    optim = torch.optim.SGD(model.parameters(), lr=0.01)
    progress = StateDict(step=0)
    app_state = {"model": model, "optim": optim, "progress": progress}
    path = os.path.join(args.work_dir, "snap")
    if os.path.exists(os.path.join(path, ".snapshot_metadata")):
        Snapshot(path).restore(app_state)
    while progress["step"] < args.steps:
        loss = model(torch.randn(32, 1024, device=dev)).pow(2).mean()
        optim.zero_grad()
        loss.backward()
        optim.step()
        progress["step"] += 1
        if progress["step"] % 10 == 0:
            pending = Snapshot.async_take(path, app_state)  # training continues
            pending.wait()
            if dist.get_rank() == 0:
                print(f"step {progress['step']}: snapshot committed")
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
