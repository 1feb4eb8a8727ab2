#!/usr/bin/env python3
"""BASELINE config 1: ResNet-18 DDP world_size=2 on CPU/gloo, take + restore to local FS.

Run: python -m torch.distributed.run --nproc-per-node 2 --master-addr 127.0.0.1 \
        benchmarks/resnet_ddp/main.py
"""

import os
import shutil
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402
from torch.nn.parallel import DistributedDataParallel as DDP  # noqa: E402

from common import Timer, emit, init_dist, max_over_ranks, sync  # noqa: E402
from hipsnapshot import RNGState, Snapshot, StateDict  # noqa: E402
from hipsnapshot.models.resnet import resnet18  # noqa: E402


def main():
    rank, ws, dev = init_dist("gloo", gpu=False)
    torch.manual_seed(0)
    model = DDP(resnet18(100))
    opt = torch.optim.SGD(model.parameters(), lr=0.01, momentum=0.9)
    for _ in range(2):
        loss = model(torch.randn(4, 3, 64, 64)).logsumexp(-1).mean()
        opt.zero_grad()
        loss.backward()
        opt.step()
    root = os.path.join(os.environ.get("HSBENCH_DIR", "/tmp"), "hs_resnet")
    if rank == 0:
        shutil.rmtree(root, ignore_errors=True)
    sync(dev)
    app = {"model": model, "optim": opt, "progress": StateDict(step=2), "rng": RNGState()}
    with Timer() as t:
        Snapshot.take(root, app)
    ref = {k: v.clone() for k, v in model.state_dict().items()}
    torch.manual_seed(123)
    model2 = DDP(resnet18(100))
    opt2 = torch.optim.SGD(model2.parameters(), lr=0.01, momentum=0.9)
    prog = StateDict(step=0)
    with Timer() as tr:
        Snapshot(root).restore({"model": model2, "optim": opt2, "progress": prog,
                                "rng": RNGState()})
    ok = all(torch.equal(v, ref[k]) for k, v in model2.state_dict().items()) and prog["step"] == 2
    emit({"bench": "resnet18_ddp_gloo", "world_size": ws,
          "take_s": round(max_over_ranks(t.s, dev), 3),
          "restore_s": round(max_over_ranks(tr.s, dev), 3), "ok": ok})
    sync(dev)
    if rank == 0:
        shutil.rmtree(root, ignore_errors=True)
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
